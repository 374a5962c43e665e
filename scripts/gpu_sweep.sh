# Bench sweep over batches in flight (PS="..."), extra bench args in BARGS
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for P in ${PS:-1 2 3}; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --inflight $P ${BARGS:-} > gpurun_out/bench_q$P.log 2>&1; rc=$?; echo "bench P=$P rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_q$P.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_q$P.log').read().strip().splitlines()[-1]); print($P, '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'p99 %.3f'%d['p99_batch_ms'], 'stream %.3f ms'%d['roofline']['launch_ms'], d['tiers'])"
done
