# Bench knob sweep: one JSON line per configuration into gpurun_out/sweep_${TAG}.jsonl.
# usage: TAG=r2i CONFIGS="--inflight 2|--inflight 4 --stream-wgs 4" bash scripts/gpu_sweep.sh
set -u
TAG=${TAG:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/sweep_${TAG}.jsonl
IFS='|' read -ra CF <<< "${CONFIGS}"
for c in "${CF[@]}"; do
  timeout -k 10 180 python bench.py --cpu-seconds 0 --steps ${STEPS:-100} $c > gpurun_out/sweep_one.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then echo "config [$c] rc=$rc"; tail -5 gpurun_out/sweep_one.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_one.log').read().strip().splitlines()[-1]); d['sweep_args']=sys.argv[1]; print(json.dumps(d))" "$c" >> gpurun_out/sweep_${TAG}.jsonl
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_one.log').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e9,3), 'G/s p99', round(d.get('p99_batch_ms',0),3), 'stream', round(d['roofline']['launch_ms'],4))" "$c"
done
exit 0
