# round 6: MS-BFS parity (dense grid tests), same-box A/B round 5 vs HEAD library, then scripts/gpu_r6_prof.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_check.py tests/test_gpu_expand.py -x -q -k "grid_dense or synthetic_graph or heavy or expand" --timeout 150 --timeout-method thread > gpurun_out/pytest_r6c.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r6c.log
[ $rc -eq 0 ] || exit $rc
TAG=r6c_ab VARIANTS="libketogpu_r5.so|-" ROUNDS=3 STEPS=20 ARGS="--expand-steps 0 --c3-steps 0 --sharded-steps 0 --heavy-steps 0 --host-calls 0 --parity 0 --latency-batches 100" bash scripts/gpu_ab.sh && TAG=r6c bash scripts/gpu_r6_prof.sh
