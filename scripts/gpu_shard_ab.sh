# Sharded exchange-protocol knob A/B (tools/shard_ab.py) on one GPU.
# usage: gpurun -- 'TAG=r5a CFGS="- shard_budget=1024" bash scripts/gpu_shard_ab.sh'  env: ARGS (tool args)
set -u
TAG=${TAG:-r5a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/shard_ab.py ${ARGS:-} $CFGS > gpurun_out/shard_ab_${TAG}.jsonl 2> gpurun_out/shard_ab_${TAG}.err; rc=$?
echo "ab rc=$rc"; cut -c1-200 gpurun_out/shard_ab_${TAG}.jsonl
exit $rc
