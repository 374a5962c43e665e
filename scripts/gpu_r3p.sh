# Round 3: the one-rank sharded level loop with workgroup-aggregated hub-row lists walked flat by
# k_shard_heavy (threshold 0 = every expansion), sub-bucket counters, speculative probe / row loads:
# sharded parity tests, then old vs new at several thresholds, then a kernel trace of the best.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3p.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3p.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_r3pshard.jsonl
for r in 1 2; do
  for V in "ms_old.so 0" "- 4096" "- 512" "- 64" "- 0"; do
    set -- $V
    if [ "$1" != "-" ]; then export KG_LIB_PATH="$GRAFT_REPO_ROOT/keto_amd/lib/ab/$1"; A=""; else unset KG_LIB_PATH; A="--shard-heavy $2"; fi
    timeout -k 10 200 python bench.py --mode sharded --steps 20 --warmup 4 $A > gpurun_out/ab_one.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "[$V] rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; }
    tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['ab']=sys.argv[1]; print(json.dumps(d))" "$V" >> gpurun_out/ab_r3pshard.jsonl
    tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], '%.4g' % d['value'], d['ms_per_step'], d['p99_batch_ms'])" "$V"
  done
done
unset KG_LIB_PATH
