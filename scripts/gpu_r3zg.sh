# After the sub-bucket flag-index fix and the reachable-bad-node pruning rule: sharded GPU tests, the
# C3 leftover debug, C3 / C4 sharded lines.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3zg.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3zg.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/dbg/sharded_c3_left.py 1e8 > gpurun_out/dbg_c3left.log 2>&1; rc=$?; echo "dbg rc=$rc"; grep -v "^\[W\|amdgpu.ids" gpurun_out/dbg_c3left.log | tail -6
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_${tag}.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/bench_${tag}.log | cut -c1-260; return $rc; }
run r3z_sharded_c3 --mode sharded --preset 1 --steps 20 --warmup 4 --cpu-seconds 0 || exit $?
run r3z_sharded --mode sharded --steps 40 --warmup 6 --cpu-seconds 0 || exit $?
