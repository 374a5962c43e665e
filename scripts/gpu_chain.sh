# One-batch-in-flight kernel timeline of the default C2 bench (rocprofv3 kernel trace), then a
# same-box A/B of whole trees (scripts/gpu_heads_ab.sh).
# usage: gpurun -- 'TAG=r4o VARIANTS="ab/<sha>|." bash scripts/gpu_chain.sh'   env: EXTRA (bench args)
set -u
TAG=${TAG:-chain}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_p1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --inflight 1 ${EXTRA:-} > gpurun_out/prof_${TAG}_p1.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py gpurun_out/prof_${TAG}_p1/run_kernel_trace.csv ${PERCALL:-k_grid_level} > gpurun_out/timeline_${TAG}_p1.txt; cat gpurun_out/timeline_${TAG}_p1.txt
rm -f gpurun_out/prof_${TAG}_p1/run_kernel_trace.csv
if [ -n "${VARIANTS:-}" ]; then bash scripts/gpu_heads_ab.sh; fi
