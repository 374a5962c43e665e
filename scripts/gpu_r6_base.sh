# Round-6 baseline kernel profiles of the non-headline workloads: C3 (one batch in flight, for a clean
# one-batch timeline), the heavy-tail point and one C5 expand call chain.
# usage: gpurun -- 'TAG=r6a bash scripts/gpu_r6_base.sh'
set -u
TAG=${TAG:-r6a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
Q="--cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
if [ "${C3:-1}" = "1" ]; then
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c3 -o run --output-format csv -- python3 bench.py --preset 1 --tuples 1e7 --inflight 1 --steps 10 --warmup 3 $Q > gpurun_out/prof_${TAG}_c3.log 2>&1; rc=$?; echo "c3 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py gpurun_out/prof_${TAG}_c3/run_kernel_trace.csv > gpurun_out/timeline_${TAG}_c3.txt || true
fi
if [ "${HEAVY:-1}" = "1" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_heavy -o run --output-format csv -- python3 bench.py --heavy-tail --steps 20 --warmup 4 $Q > gpurun_out/prof_${TAG}_heavy.log 2>&1; rc=$?; echo "heavy rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py gpurun_out/prof_${TAG}_heavy/run_kernel_trace.csv > gpurun_out/timeline_${TAG}_heavy.txt || true
fi
if [ "${EXPAND:-1}" = "1" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_expand -o run --output-format csv -- python3 bench.py --mode expand --inflight 1 --steps 3 --warmup 1 --cpu-seconds 0 --parity-roots 0 > gpurun_out/prof_${TAG}_expand.log 2>&1; rc=$?; echo "expand rc=$rc"
[ $rc -eq 0 ] || exit $rc
fi
exit 0
