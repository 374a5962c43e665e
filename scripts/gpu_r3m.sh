# Round 3: sharded impure union seeds at their owner + general phase; k_ms_level blind ORs -- the
# sharded and MS-BFS parity tests, the world-2 debug table, then the heavy-tail A/B old vs new and a
# latency run of the new one.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python tools/dbg/general_w2.py > gpurun_out/dbg_general.log 2>&1; rc=$?; echo "dbg rc=$rc"; grep "^world\|^  " gpurun_out/dbg_general.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_shard.py tests/test_gpu_check.py -m gpu -x -q --timeout 200 --timeout-method thread -k "general or impure or c3 or formula or c4 or grid or workgroup or random_graphs or synthetic_graph or bench_tune or hip_vs" > gpurun_out/pytest_r3m.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3m.log
[ $rc -eq 0 ] || exit $rc
TAG=r3mheavy STEPS=8 ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 50000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=2 VARIANTS="ms_old.so|-" bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 python bench.py --heavy-tail --batch 250000 --steps 8 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 200 --host-calls 0 > gpurun_out/bench_r3m_heavy.log 2>&1; rc=$?; echo "heavy rc=$rc"; tail -1 gpurun_out/bench_r3m_heavy.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p99_batch_ms'], d.get('batch_ms_p50'))"
