# Round-3 bring-up of the bidirectional grid tier and the LDS-cached expand tail: their parity tests,
# the heavy-tail point with grid_bidir on / off, and the C5 expand bench with its oracle parity leg.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_check.py tests/test_gpu_expand.py tests/test_shard.py -m gpu -q -x --timeout 200 --timeout-method thread -k "grid_bidirectional or workgroup_tiers or heavy_path or synthetic_graph or bench_tune or expand or shard or formula" > gpurun_out/pytest_r3b.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode expand --steps 12 --warmup 4 > gpurun_out/bench_r3b_expand.log 2>&1; rc=$?; echo "expand rc=$rc"; tail -1 gpurun_out/bench_r3b_expand.log | cut -c1-700
[ $rc -eq 0 ] || exit $rc
TAG=r3bgrid STEPS=6 ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 50000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=1 VARIANTS="- --grid-bidir 1|- --grid-bidir 0" bash scripts/gpu_ab.sh
