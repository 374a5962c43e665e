# Sharded-mode evidence: per-level record counts (KG_SHARD_TRACE) and a rocprofv3 kernel trace of
# the world-1 bench.  usage: gpurun -- 'TAG=r2s5 bash scripts/gpu_shard_prof.sh'  env: EXTRA
set -u
TAG=${TAG:-r2s}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KG_SHARD_TRACE=1 timeout -k 10 300 python3 bench.py --mode sharded --tuples 1e9 --steps 3 --warmup 1 ${EXTRA:-} > gpurun_out/shard_trace_${TAG}.json 2> gpurun_out/shard_trace_${TAG}.err; rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --mode sharded --tuples 1e9 --steps 10 --warmup 2 ${EXTRA:-} > gpurun_out/prof_${TAG}.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
ANCHOR=k_shard_seed python3 scripts/timeline.py gpurun_out/prof_${TAG}/run_kernel_trace.csv k_shard_level > gpurun_out/timeline_${TAG}.txt || true
rm -f gpurun_out/prof_${TAG}/run_kernel_trace.csv
exit 0
