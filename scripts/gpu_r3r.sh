# Round 3: the sharded seed with 4 queries per thread (one workgroup append per 1024 queries) and the
# holder bit before the node map; level workgroups per CU -- sharded parity tests, then the A/B.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3r.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3r.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_r3rshard.jsonl
for r in 1 2; do
  for V in "shard_prev.so" "-" "- --shard-wgs 4" "- --shard-wgs 2" "- --inflight 8"; do
    set -- $V; lib=$1; shift; A="$*"
    if [ "$lib" != "-" ]; then export KG_LIB_PATH="$GRAFT_REPO_ROOT/keto_amd/lib/ab/$lib"; else unset KG_LIB_PATH; fi
    timeout -k 10 200 python bench.py --mode sharded --steps 20 --warmup 4 $A > gpurun_out/ab_one.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "[$V] rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; }
    tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['ab']=sys.argv[1]; print(json.dumps(d))" "$V" >> gpurun_out/ab_r3rshard.jsonl
    tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], '%.4g' % d['value'], d['ms_per_step'], d['p99_batch_ms'])" "$V"
  done
done
unset KG_LIB_PATH
