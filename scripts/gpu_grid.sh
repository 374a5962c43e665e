# Bidirectional grid tier: its parity tests, then the heavy-tail point with grid_bidir on / off.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_check.py -q -x --timeout 120 --timeout-method thread -k "${TESTK:-grid_bidirectional or workgroup_tiers or heavy_path or synthetic_graph or bench_tune}" > gpurun_out/pytest_grid.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_grid.log
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r3grid} STEPS=${STEPS:-8} ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 50000 --parity-canonical 0 --latency-batches 0 --host-calls 0 ${HARGS:-}" ROUNDS=1 VARIANTS="${VARIANTS:-- --grid-bidir 1|- --grid-bidir 0}" bash scripts/gpu_ab.sh
