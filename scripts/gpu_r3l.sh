# Round 3: k_ms_level with blind ORs and two edges per lane group -- MS-BFS parity tests, then the
# heavy-tail point old vs new; the sharded general-rewrite phase (parity leg on), then the new one with the latency phase (p99).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py tests/test_shard.py -m gpu -x -q --timeout 200 --timeout-method thread -k "grid or workgroup or random_graphs or synthetic_graph or bench_tune or general or impure" > gpurun_out/pytest_r3l.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3l.log
[ $rc -eq 0 ] || exit $rc
TAG=r3lheavy STEPS=8 ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 50000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=2 VARIANTS="ms_old.so|-" bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 python bench.py --heavy-tail --batch 250000 --steps 8 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 200 --host-calls 0 > gpurun_out/bench_r3l_heavy.log 2>&1; rc=$?; echo "heavy rc=$rc"; tail -1 gpurun_out/bench_r3l_heavy.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p99_batch_ms'], d.get('batch_ms_p50'))"
