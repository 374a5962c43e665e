# In-flight batches: concurrent-stream parity, then bench at 1/2/3 batches in flight per GPU
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_check.py -q -x --timeout 120 --timeout-method thread -k "concurrent or synthetic_graph" > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_q.log
[ $rc -eq 0 ] || exit $rc
for P in 1 2 3 4; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --inflight $P > gpurun_out/bench_q$P.log 2>&1; rc=$?; echo "bench P=$P rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_q$P.log').read().strip().splitlines()[-1]); print($P, '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'p99 %.3f'%d['p99_batch_ms'], 'stream %.3f ms'%d['roofline']['launch_ms'], d['tiers'])"
done
