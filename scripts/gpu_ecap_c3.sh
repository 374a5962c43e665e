set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for E in 0 512; do
  timeout -k 10 300 python3 bench.py --preset 1 --inflight 6 --steps 30 --warmup 6 --cpu-seconds 0 --stream-ecap $E > gpurun_out/ecap3_$E.json 2> gpurun_out/ecap3_$E.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ecap3_$E.json').read().strip().splitlines()[-1]); print($E, d['value'], d['p99_batch_ms'], d['tiers'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
