# C2/C4 (or PRESET=1 C3) in-flight / hardware-queue sweep: CONFIGS="queues:inflight ..."
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for C in ${CONFIGS:-0:4 8:8}; do
  Q=${C%%:*}; P=${C##*:}
  timeout -k 10 200 python3 bench.py --preset ${PRESET:-0} --steps ${STEPS:-60} --warmup 8 --cpu-seconds 0 --hw-queues $Q --inflight $P > gpurun_out/cs_${Q}_${P}.json 2> gpurun_out/cs_${Q}_${P}.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/cs_${Q}_${P}.json').read().strip().splitlines()[-1]); print($Q, $P, d['value'], d['p99_batch_ms'], d['roofline']['launch_ms'])"
done
