# Rewrite-path parity, then C3 bench lines over interp_wgs
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -q -x --timeout 120 --timeout-method thread -k "rewrite or c3 or relation_not_found or beyond_lds" > gpurun_out/pytest_interp.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_interp.log
[ $rc -eq 0 ] || exit $rc
for W in ${WGS:-2 4 6 8}; do
  timeout -k 10 300 python bench.py --preset 1 --steps 20 --warmup 3 --cpu-seconds 0 --interp-wgs $W > gpurun_out/c3_w$W.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "wgs $W rc=$rc"; tail -3 gpurun_out/c3_w$W.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c3_w$W.log').read().strip().splitlines()[-1]); print('wgs $W', '%.4g'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'p99 %.1f'%d['p99_batch_ms'])"
done
