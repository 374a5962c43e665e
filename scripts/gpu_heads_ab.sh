# Same-box A/B of whole source trees (earlier rounds' heads staged under ab/<sha>/ with their own
# bench.py and built library, and this tree "."), alternating, one JSON line per run.
# usage: TAG=r4ab VARIANTS="ab/25ed21d --tuples 1062976915|ab/b0bf7a5|." ROUNDS=3 bash scripts/gpu_heads_ab.sh
set -u
TAG=${TAG:-heads}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROOT=$(pwd)
mkdir -p gpurun_out
: > gpurun_out/ab_${TAG}.jsonl
IFS='|' read -ra VS <<< "${VARIANTS}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "${VS[@]}"; do
    dir=${v%% *}; args=""; [ "$dir" != "$v" ] && args=${v#* }
    (cd "$ROOT/$dir" && timeout -k 10 ${AB_TIMEOUT:-200} python bench.py --cpu-seconds 0 --steps ${STEPS:-100} $args) \
      > gpurun_out/ab_one.log 2>&1; rc=$?
    if [ $rc -ne 0 ]; then echo "variant [$v] rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_one.log').read().strip().splitlines()[-1]); d['ab']=sys.argv[1]; print(json.dumps(d))" "$v" >> gpurun_out/ab_${TAG}.jsonl
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_one.log').read().strip().splitlines()[-1]); print(repr(sys.argv[1]), '%.4g' % d['value'], 'p99', round(d.get('p99_batch_ms') or 0,3), 'rows', d['config'].get('tuples'), 'steady', (d.get('steady') or {}).get('value'))" "$v"
  done
done
exit 0
