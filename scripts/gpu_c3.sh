# C3 (OPL view/edit/share) at 1e9 tuples: bench at 6 batches in flight, then a kernel-trace profile.
# usage: gpurun -- 'bash scripts/gpu_c3.sh'    env: TAG (log suffix), TUPLES (default 1e9), INFLIGHT (6)
set -u
TAG=${TAG:-r2c3}
TUPLES=${TUPLES:-1e9}
INFLIGHT=${INFLIGHT:-6}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --preset 1 --tuples $TUPLES --inflight $INFLIGHT --steps 40 --warmup 6 --cpu-seconds ${CPU_SECONDS:-0} > gpurun_out/bench_${TAG}.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_${TAG}.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --preset 1 --tuples $TUPLES --inflight $INFLIGHT --steps 12 --warmup 4 --cpu-seconds 0 > gpurun_out/prof_${TAG}.log 2>&1; rc=$?; echo "prof rc=$rc"
fi
exit $rc
