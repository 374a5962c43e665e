# Round 3: shard + check GPU tests (k_stream4 default, native one-rank level loop), sharded bench,
# then the headline's profile / PMC / bench line.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_shard.py tests/test_gpu_check.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3f.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3f.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode sharded --steps 20 --warmup 4 > gpurun_out/bench_r3f_sharded.log 2>&1; rc=$?; echo "sharded rc=$rc"; tail -1 gpurun_out/bench_r3f_sharded.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
TAG=r3f bash scripts/gpu_profile.sh
