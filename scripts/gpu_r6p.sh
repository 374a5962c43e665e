# round 6: the default line at 16 vs 32 hardware queues (alternating, two rounds)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6p_queues STEPS=20 AB_TIMEOUT=500 ARGS="--warmup 5 --cpu-seconds 4" VARIANTS="- --hw-queues 16|- --hw-queues 32" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_r6p_queues.jsonl'):
    d = json.loads(l)
    print(d['ab'], 'headline %.4g' % d['value'], 'c3 %.4g' % d['c3']['value'], 'heavy %.4g' % d['heavy']['value'],
          'c5 %.4g' % d['expand']['value'], 'sharded %.4g' % d['sharded']['value'], 'xch %.4g' % d['sharded']['exchange']['value'])
PY
