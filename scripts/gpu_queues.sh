# Batches in flight vs HIP hardware queues: C5 expand and C2 checks at several (hw-queues, inflight).
# usage: gpurun -- 'TAG=r2q bash scripts/gpu_queues.sh'
set -u
TAG=${TAG:-r2q}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/queues_${TAG}.jsonl
for C in ${CONFIGS:-"expand 0 4" "expand 8 4" "expand 8 6" "check 0 4" "check 8 6" "check 8 8" "check 16 8"}; do
  set -- $C
  timeout -k 10 300 python bench.py --mode $1 --hw-queues $2 --inflight $3 --steps ${STEPS:-16} --warmup 4 --cpu-seconds 0 > gpurun_out/q_${TAG}.log 2>&1; rc=$?
  echo "$C rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/q_${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['_cfg']='$C'; print(json.dumps(d))" >> gpurun_out/queues_${TAG}.jsonl
done
