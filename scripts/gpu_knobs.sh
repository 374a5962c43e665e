# Knob sweep at the default 4 batches in flight: one bench line per BARGS set (separated by ';')
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${KNOBS:-}"
i=0
for K in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --cpu-seconds 0 $K > gpurun_out/knob_$i.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "[$K] rc=$rc"; tail -5 gpurun_out/knob_$i.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/knob_$i.log').read().strip().splitlines()[-1]); print('[$K]', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'p99 %.3f'%d['p99_batch_ms'], 'stream %.3f ms'%d['roofline']['launch_ms'], 'back', d['tiers']['back'], 'grid', d['tiers']['grid'])"
done
