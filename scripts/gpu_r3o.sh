# Round 3: the one-rank sharded level loop -- flat edge-parallel hub rows (k_shard_heavy over a tile
# map) and per-XCD sub-bucket counters (no single counter word for every workgroup's appends):
# sharded parity tests (hub path forced at 256 edges), then old / flat-hub / flat-hub+sub-buckets at
# 4 batches in flight, and the hub threshold with both.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3o.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3o.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_r3oshard.jsonl
for r in 1 2; do
  for V in "ms_old.so 4096" "flatheavy.so 4096" "- 4096" "- 1024" "- 512"; do
    set -- $V
    if [ "$1" != "-" ]; then export KG_LIB_PATH="$GRAFT_REPO_ROOT/keto_amd/lib/ab/$1"; else unset KG_LIB_PATH; fi
    A="--shard-heavy $2"; [ "$1" = "ms_old.so" ] && A=""
    timeout -k 10 200 python bench.py --mode sharded --steps 20 --warmup 4 $A > gpurun_out/ab_one.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "[$V] rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; }
    tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['ab']=sys.argv[1]; print(json.dumps(d))" "$V" >> gpurun_out/ab_r3oshard.jsonl
    tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], '%.4g' % d['value'], d['ms_per_step'], d['p99_batch_ms'])" "$V"
  done
done
unset KG_LIB_PATH
