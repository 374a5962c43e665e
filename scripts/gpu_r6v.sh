# round 6: C3 tier budgets at the round's code
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6v_c3 STEPS=20 ARGS="--preset 1 --tuples 1e7 --inflight 6 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 60" VARIANTS="-|- --back-edges 16384|- --back-edges 1024|- --stream-ecap 2048|- --back-wgs 2" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open('gpurun_out/ab_r6v_c3.jsonl'):
    d = json.loads(l)
    agg[d['ab']].append((d['value'], d['steady']['value'], d['tiers']['back'], d['tiers']['grid']))
for k, v in agg.items():
    print('%-26s value %s steady %s back/grid %s' % (k, ' '.join('%.3g' % x[0] for x in v), ' '.join('%.3g' % x[1] for x in v), v[0][2:]))
PY
