# round 6: node-map slots with inline check rows -- check-path and sharded GPU tests, smoke, headline A/B against
# the 32-B slot build (keto_amd/lib/ab/nslot32.so), TCC request counts of k_resolve / k_stream4 for both, then the
# C5 line on the device path at 8 / 12 / 16 calls in flight
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_check.py tests/test_shard.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6m.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r6m.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6m.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=r6m_inline STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 60" VARIANTS="nslot32.so|-" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
B="python3 bench.py --steps 6 --warmup 4 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0"
for V in nslot32 inline; do
  if [ $V = nslot32 ]; then export KG_LIB_PATH="$GRAFT_REPO_ROOT/keto_amd/lib/ab/nslot32.so"; else unset KG_LIB_PATH; fi
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_resolve|k_stream4|k_back" --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_r6m_$V -o run --output-format csv -- $B > gpurun_out/pmc_r6m_$V.log 2>&1; rc=$?; echo "pmc $V rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
unset KG_LIB_PATH
for P in 8 12 16; do
  timeout -k 10 300 python bench.py --mode expand --inflight $P --steps $((2 * P)) --warmup $P --cpu-seconds 0 --parity-roots 0 > gpurun_out/expand_r6m_$P.log 2>&1; rc=$?; echo "expand $P rc=$rc"; tail -1 gpurun_out/expand_r6m_$P.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_path']['value'], d['kernel_ms_per_step'])"
  [ $rc -eq 0 ] || exit $rc
done
