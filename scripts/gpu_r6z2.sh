# round 6 closing: the default bench line (the driver's command) after capping C5's host-buffer leg at 4 callers,
# then a same-box A/B of reading back only the grid round's summary without stats (keto_amd/lib/ab/gridsum.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_r6z2.log 2>&1; rc=$?; echo "bench rc=$rc"
tail -1 gpurun_out/bench_r6z2.log > gpurun_out/r6z2_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/r6z2_bench.json')); print('%.4g' % d['value'], {k: (d[k].get('value') if isinstance(d[k], dict) else None) for k in ('c3','heavy','expand','sharded') if k in d}); print(json.dumps(d.get('expand'))[:600])"
[ $rc -eq 0 ] || exit $rc
TAG=r6z2_gridsum STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 60" VARIANTS="gridsum.so|-" ROUNDS=3 bash scripts/gpu_ab.sh
