# Same-box A/B of library builds / bench knobs (alternating rounds, so box drift shows as noise).
# VARIANTS: "|"-separated "LIB ARGS..." entries; LIB is a file under keto_amd/lib/ab/ (loaded via
# KG_LIB_PATH) or "-" for the in-tree build.
# usage: TAG=r2ab VARIANTS="libketogpu_head.so|-|- --resolve-unheld 0" ROUNDS=2 bash scripts/gpu_ab.sh
set -u
TAG=${TAG:-r2ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab_${TAG}.jsonl
IFS='|' read -ra VS <<< "${VARIANTS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    lib=${v%% *}; args=""; [ "$lib" != "$v" ] && args=${v#* }
    if [ "$lib" != "-" ]; then export KG_LIB_PATH="$GRAFT_REPO_ROOT/keto_amd/lib/ab/$lib"; else unset KG_LIB_PATH; fi
    # leading VAR=value tokens of a variant are environment settings for that run (e.g. KG_DREC=0)
    envs=""; rest=""
    for tok in $args; do
      if [ -z "$rest" ] && [[ "$tok" == *=* ]] && [[ "$tok" != -* ]]; then envs="$envs $tok"; else rest="$rest $tok"; fi
    done
    timeout -k 10 ${AB_TIMEOUT:-180} env $envs python bench.py --cpu-seconds 0 --steps ${STEPS:-100} ${ARGS:-} $rest > gpurun_out/ab_one.log 2>&1; rc=$?
    if [ $rc -ne 0 ]; then echo "variant [$v] rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_one.log').read().strip().splitlines()[-1]); d['ab']=sys.argv[1]; print(json.dumps(d))" "$v" >> gpurun_out/ab_${TAG}.jsonl
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_one.log').read().strip().splitlines()[-1]); print(repr(sys.argv[1]), '%.4g' % d['value'], 'p99', round(d.get('p99_batch_ms') or 0,3), 'kernel ms', round((d.get('roofline') or {}).get('launch_ms') or 0,4), 'wave', round((d.get('stream_diag') or {}).get('mean_wave_us',0),1), 'span', round((d.get('stream_diag') or {}).get('span_us',0),1), 'steps', (d.get('stream_diag') or {}).get('steps'))" "$v"
  done
done
exit 0
