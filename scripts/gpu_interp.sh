# Rewrite-path parity (random rewrites + C3 incl. the bounded pass-2 cap), then the C3 bench line
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -q -x --timeout 120 --timeout-method thread -k "rewrite or c3 or relation_not_found" > gpurun_out/pytest_interp.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_interp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --preset 1 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/r1w_c3b.log 2>&1; rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/r1w_c3b.log | cut -c1-330
exit $rc
