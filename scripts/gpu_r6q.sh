# round 6: k_stream6 (two pipelined query groups per wave) -- check-path GPU tests, smoke, A/B against k_stream4
# (keto_amd/lib/ab/dual0.so) on the headline and C3, then the default line at 16 vs 32 hardware queues
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6q.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r6q.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6q.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=r6q_dual STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 60" VARIANTS="dual0.so|-" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
TAG=r6q_dual_c3 STEPS=20 ARGS="--preset 1 --tuples 1e7 --inflight 6 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 100000 --parity-canonical 10000 --latency-batches 60" VARIANTS="dual0.so|-" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
TAG=r6q_queues STEPS=20 AB_TIMEOUT=500 ARGS="--warmup 5 --cpu-seconds 4" VARIANTS="- --hw-queues 16|- --hw-queues 32" ROUNDS=1 bash scripts/gpu_ab.sh || exit 1
python3 - <<'PY'
import json
for l in open('gpurun_out/ab_r6q_queues.jsonl'):
    d = json.loads(l)
    print(d['ab'], 'headline %.4g' % d['value'], 'c3 %.4g' % d['c3']['value'], 'heavy %.4g' % d['heavy']['value'],
          'c5 %.4g' % d['expand']['value'], 'sharded %.4g' % d['sharded']['value'], 'xch %.4g' % d['sharded']['exchange']['value'])
PY
