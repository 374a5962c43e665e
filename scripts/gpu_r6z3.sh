# round 6: k_grid_finish stores the grid round's summary straight into the pinned host buffer (no copy after the
# batch's last kernel without stats; keto_amd/lib/ab/hostsum.so) -- check-path GPU tests on that build, then a
# same-box A/B against the in-tree build on the headline (20-step lines, as the driver runs them)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
KG_LIB_PATH=$GRAFT_REPO_ROOT/keto_amd/lib/ab/hostsum.so timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6z3.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r6z3.log
[ $rc -eq 0 ] || exit $rc
TAG=r6z3_hostsum STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 120" VARIANTS="hostsum.so|-" ROUNDS=4 bash scripts/gpu_ab.sh
