# C5 in-flight / hardware-queue sweep: CONFIGS="queues:inflight ..." STEPS=30
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for C in ${CONFIGS:-8:6 12:10 16:12}; do
  Q=${C%%:*}; P=${C##*:}
  timeout -k 10 200 python3 bench.py --mode expand --steps ${STEPS:-30} --warmup 4 --hw-queues $Q --inflight $P > gpurun_out/xs_${Q}_${P}.json 2> gpurun_out/xs_${Q}_${P}.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/xs_${Q}_${P}.json').read().strip().splitlines()[-1]); print($Q, $P, d['value'], d['ms_per_step'])"
done
