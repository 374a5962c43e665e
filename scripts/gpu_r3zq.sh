# Round-3 closing check at HEAD: whole GPU suite, smoke, default bench, sharded C4 and C3 (world 1, with
# the oracle parity leg).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r3zq BENCH2="--mode sharded --steps 40 --warmup 6" bash scripts/gpu_tests.sh || exit $?
timeout -k 10 400 python bench.py --mode sharded --preset 1 --steps 20 --warmup 4 --cpu-seconds 0 > gpurun_out/bench3_r3zq.log 2>&1; rc=$?; echo "bench3 rc=$rc"; tail -1 gpurun_out/bench3_r3zq.log | cut -c1-300
exit $rc
