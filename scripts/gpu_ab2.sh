# GPU parity suite then bench sweep (PS) -- A/B of a kernel change
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_sweep.sh
