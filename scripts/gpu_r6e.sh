# round 6: parity subset, headline A/B round 5 vs HEAD, heavy-tail line, C3 knob A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_check.py tests/test_gpu_expand.py -x -q -k "grid_dense or synthetic_graph or heavy or expand or tail_tiers" --timeout 150 --timeout-method thread > gpurun_out/pytest_r6e.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r6e.log
[ $rc -eq 0 ] || exit $rc
TAG=r6e_ab VARIANTS="libketogpu_r5.so|-" ROUNDS=3 STEPS=20 ARGS="--expand-steps 0 --c3-steps 0 --sharded-steps 0 --heavy-steps 0 --host-calls 0 --parity 0 --latency-batches 100" bash scripts/gpu_ab.sh || exit 1
timeout -k 10 200 python bench.py --heavy-tail --steps 20 --warmup 4 --cpu-seconds 0 --parity 62500 --parity-canonical 5000 --latency-batches 120 --host-calls 0 > gpurun_out/heavy_r6e.log 2>&1; rc=$?; echo "heavy rc=$rc"; tail -1 gpurun_out/heavy_r6e.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6d.sh
