# Re-entry check: full GPU parity suite, smoke, bench at 1/2/3 batches in flight
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
for P in ${PS:-1 2 3}; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --inflight $P > gpurun_out/bench_q$P.log 2>&1; rc=$?; echo "bench P=$P rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_q$P.log').read().strip().splitlines()[-1]); print($P, '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'p99 %.3f'%d['p99_batch_ms'], 'stream %.3f ms'%d['roofline']['launch_ms'], d['tiers'])"
done
