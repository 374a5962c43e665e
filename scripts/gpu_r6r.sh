# round 6: 1024-edge grid tiles (keto_amd/lib/ab/grid4.so, -DKG_GRID_EPT=4) vs 512 on C3 and the headline,
# check-path GPU tests, then the default line (C5 sub-line now a child process at 32 hardware queues)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6r.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r6r.log
[ $rc -eq 0 ] || exit $rc
TAG=r6r_grid4_c3 STEPS=20 ARGS="--preset 1 --tuples 1e7 --inflight 6 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 100000 --parity-canonical 10000 --latency-batches 60" VARIANTS="grid4.so|-" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
TAG=r6r_grid4 STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 60" VARIANTS="grid4.so|-" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6r.log 2>&1; rc=$?; echo "bench rc=$rc"
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/bench_r6r.log').read().strip().splitlines()[-1])
print('headline %.4g steady %.4g' % (d['value'], d['steady']['value']))
for k in ('c3', 'heavy', 'expand', 'sharded'):
    v = d.get(k, {})
    print(k, v.get('value'), (v.get('parity') or {}).get('mismatches'), v.get('error'))
print('expand host', d.get('expand', {}).get('host_path'))
PY
