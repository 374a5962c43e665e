# Bidirectional grid tier with holder-gated slots: parity tests, then the heavy-tail point (hold caps).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_check.py -m gpu -q -x --timeout 200 --timeout-method thread -k "grid_bidirectional or workgroup_tiers or heavy_path or synthetic_graph" > gpurun_out/pytest_r3d.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3d.log
[ $rc -eq 0 ] || exit $rc
TAG=r3dgrid STEPS=6 ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 50000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=1 VARIANTS="- --grid-bidir 1|- --grid-bidir 0|- --grid-bidir 64|- --grid-bidir 16384" bash scripts/gpu_ab.sh
for v in 1 0; do
  timeout -k 10 300 python bench.py --mode expand --steps 12 --warmup 4 --expand-tail $v --parity-roots 100 > gpurun_out/bench_r3d_expand_$v.log 2>&1; rc=$?; echo "expand tail=$v rc=$rc"; tail -1 gpurun_out/bench_r3d_expand_$v.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
