# round 6: k_stream4's LDS (33.7 KB per workgroup: 4 per CU) below 32 KB -- 5 workgroups per CU, the VGPR limit --
# with a 128-entry FIFO (keto_amd/lib/ab/qc128.so) or a 256-key visited cache (vt8.so): check-path GPU tests on
# both, then a same-box A/B on the headline (20-step lines) against the in-tree build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in qc128 vt8; do
  KG_LIB_PATH=$GRAFT_REPO_ROOT/keto_amd/lib/ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6z4_$v.log 2>&1; rc=$?; echo "pytest $v rc=$rc"; tail -1 gpurun_out/pytest_r6z4_$v.log
  [ $rc -eq 0 ] || exit $rc
done
TAG=r6z4_stream_lds STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 120" VARIANTS="qc128.so|vt8.so|-|vt8.so --stream-wgs 3" ROUNDS=3 bash scripts/gpu_ab.sh
