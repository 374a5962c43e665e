# k_stream2 edge-budget sweep (kg_snapshot_tune "stream_ecap") on the default workload.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for E in ${ECAPS:-0 512 2048 8192}; do
  timeout -k 10 240 python3 bench.py --steps 40 --warmup 6 --cpu-seconds 0 --stream-ecap $E > gpurun_out/ecap_$E.json 2> gpurun_out/ecap_$E.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ecap_$E.json').read().strip().splitlines()[-1]); print($E, d['value'], d['p99_batch_ms'], d['tiers'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
