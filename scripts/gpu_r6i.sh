# round 6 (second session): k_stream4 with two edges per lane and device-resident expand -- the check-path and
# expand GPU tests, a same-box A/B of the headline against the one-edge build (keto_amd/lib/ab/epl1.so) as
# 20-step lines like the driver's, the C5 sub-line with device-resident trees, then scripts/gpu_r6h.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_check.py tests/test_gpu_expand.py tests/test_shard.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6i.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r6i.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6i.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=r6i_epl STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 60" VARIANTS="epl1.so|-" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --c3-steps 0 --heavy-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 0 --expand-steps 8 > gpurun_out/bench_r6i_c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/bench_r6i_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('expand'))[:1500])"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6h.sh
