# GPU parity for the snapshot persister + request batcher (empty-snapshot case last, on its own)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_persister.py -m gpu -v -x --timeout 120 --timeout-method thread -k "not empty" > gpurun_out/pytest_persister.log 2>&1; rc=$?; echo "persister rc=$rc"; tail -3 gpurun_out/pytest_persister.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -m pytest tests/test_gpu_persister.py -m gpu -v -x --timeout 60 --timeout-method thread -k "empty" > gpurun_out/pytest_empty.log 2>&1; rc=$?; echo "empty rc=$rc"; tail -3 gpurun_out/pytest_empty.log
exit $rc
