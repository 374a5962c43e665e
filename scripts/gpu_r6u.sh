# round 6: headline tier knobs at the round's code (two edges per lane, shorter grid chain, inline rows)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6u_knobs STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 120" VARIANTS="-|- --stream-ecap 256|- --stream-ecap 1024|- --stream-wgs 3|- --back-wgs 2|- --back-edges 8192" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open('gpurun_out/ab_r6u_knobs.jsonl'):
    d = json.loads(l)
    agg[d['ab']].append((d['value'], d['steady']['value']))
for k, v in agg.items():
    print('%-28s value %s steady %s' % (k, ' '.join('%.3g' % x[0] for x in v), ' '.join('%.3g' % x[1] for x in v)))
PY
