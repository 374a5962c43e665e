# Remaining round-3 bring-up: TTU formula tests (one GPU + sharded), C5 expand bench with parity, the
# heavy-tail point with grid_bidir on / off, sharded world-1 with batches in flight.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_shard.py tests/test_gpu_persister.py -m gpu -q -x --timeout 200 --timeout-method thread -k "formula_ttu or batcher" > gpurun_out/pytest_r3c.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3c.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode expand --steps 12 --warmup 4 > gpurun_out/bench_r3c_expand.log 2>&1; rc=$?; echo "expand rc=$rc"; tail -1 gpurun_out/bench_r3c_expand.log | cut -c1-900
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode sharded --steps 20 --warmup 4 > gpurun_out/bench_r3c_sharded.log 2>&1; rc=$?; echo "sharded rc=$rc"; tail -1 gpurun_out/bench_r3c_sharded.log | cut -c1-700
[ $rc -eq 0 ] || exit $rc
TAG=r3cgrid STEPS=6 ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 50000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=1 VARIANTS="- --grid-bidir 1|- --grid-bidir 0" bash scripts/gpu_ab.sh
