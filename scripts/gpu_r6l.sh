# round 6: the shorter k_grid_level chain and the interpreter control block by kernel -- check-path GPU tests,
# A/B against the previous grid level (keto_amd/lib/ab/grid0.so) on the headline and C3 (20-step lines), a C3
# one-batch kernel trace, then the default bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6l.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r6l.log
[ $rc -eq 0 ] || exit $rc
TAG=r6l_grid STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 60" VARIANTS="grid0.so|-" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
TAG=r6l_grid_c3 STEPS=20 ARGS="--preset 1 --tuples 1e7 --inflight 6 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 100000 --parity-canonical 10000 --latency-batches 60" VARIANTS="grid0.so|-" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6l_c3 -o run --output-format csv -- python3 bench.py --preset 1 --tuples 1e7 --inflight 6 --steps 24 --warmup 6 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0 --heavy-steps 0 > gpurun_out/prof_r6l_c3.log 2>&1; rc=$?; echo "c3 prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py gpurun_out/prof_r6l_c3/run_kernel_trace.csv > gpurun_out/timeline_r6l_c3.txt; cat gpurun_out/timeline_r6l_c3.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6l.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_r6l.log | cut -c1-300
