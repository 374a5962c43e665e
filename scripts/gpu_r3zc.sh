# Round-3 closing evidence, part C (after the expand buffer fix): expand GPU tests, C5 expand, C4 / C3
# hash-sharded, the heavy-tail point, the host boundary, incremental refresh.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_expand.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3zc.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3zc.log
[ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_${tag}.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/bench_${tag}.log | cut -c1-260; return $rc; }
run r3z_expand --mode expand --cpu-seconds 6 || exit $?
run r3z_sharded --mode sharded --steps 40 --warmup 6 --cpu-seconds 0 || exit $?
run r3z_sharded_c3 --mode sharded --preset 1 --steps 20 --warmup 4 --cpu-seconds 0 || exit $?
run r3z_heavy --heavy-tail --batch 250000 --steps 8 --warmup 2 --cpu-seconds 6 --host-calls 0 --parity-canonical 0 || exit $?
run r3z_host --mode host || exit $?
run r3z_refresh --mode refresh || exit $?
