# Expand parity, then the C5 bench line
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_expand.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_expand.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_expand.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode expand --cpu-seconds 0 > gpurun_out/r1w_c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/r1w_c5.log | cut -c1-300
exit $rc
