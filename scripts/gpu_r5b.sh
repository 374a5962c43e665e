# Round 5b: sharded GPU parity tests (remote child metadata at world 2 over gloo), a two-rank
# rehearsal on one GPU with the metadata on and off (records sent / to peers), and the exchange knob A/B.
set -u
TAG=${TAG:-r5b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${TAG}.log
[ $rc -eq 0 ] || exit $rc
R="--gpus 2 --tuples 2e8 --steps 4 --warmup 2 --expand-steps 0 --c3-steps 0 --host-calls 0 --cpu-seconds 0 --parity 20000 --latency-batches 0 --sharded-steps 4"
for M in ${METAS:-1 0}; do
  timeout -k 10 300 python bench.py $R --shard-remote-meta $M > gpurun_out/rehearse_${TAG}_m$M.json 2> gpurun_out/rehearse_${TAG}_m$M.err; rc=$?; echo "rehearse m$M rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 500 python3 -u tools/shard_ab.py ${ABARGS:-} $CFGS > gpurun_out/shard_ab_${TAG}.jsonl 2> gpurun_out/shard_ab_${TAG}.err; rc=$?
echo "ab rc=$rc"; cut -c1-160 gpurun_out/shard_ab_${TAG}.jsonl
exit $rc
