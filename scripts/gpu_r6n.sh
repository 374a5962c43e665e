# round 6: inline check rows in the 32-B node-map slot -- check-path and sharded GPU tests, smoke, headline A/B
# against the plain 32-B slot build (keto_amd/lib/ab/nslot32.so), TCC request counts, then the default line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_check.py tests/test_shard.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6n.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r6n.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6n.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=r6n_inline2 STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 60" VARIANTS="nslot32.so|-" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
B="python3 bench.py --steps 6 --warmup 4 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0"
timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_resolve|k_stream4|k_back" --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_r6n -o run --output-format csv -- $B > gpurun_out/pmc_r6n.log 2>&1; rc=$?; echo "pmc rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6n.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_r6n.log | cut -c1-300
