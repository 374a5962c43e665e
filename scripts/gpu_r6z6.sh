# round 6: k_stream4 at 6 waves per SIMD (amdgpu_waves_per_eu 6: 80 VGPRs, 3 spilled; keto_amd/lib/ab/wpe6.so)
# against the in-tree build (5 per SIMD, 95 VGPRs) -- check-path GPU tests on it, then a same-box headline A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
KG_LIB_PATH=$GRAFT_REPO_ROOT/keto_amd/lib/ab/wpe6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6z6.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_r6z6.log
[ $rc -eq 0 ] || exit $rc
TAG=r6z6_stream_wpe6 STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 120" VARIANTS="wpe6.so|-|wpe6.so --stream-wgs 3" ROUNDS=3 bash scripts/gpu_ab.sh
