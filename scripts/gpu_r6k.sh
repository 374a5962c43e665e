# round 6: the default bench line at the current code (what the driver runs), then a C3 one-batch kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6k.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_r6k.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6k_c3 -o run --output-format csv -- python3 bench.py --preset 1 --tuples 1e7 --inflight 6 --steps 24 --warmup 6 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0 --heavy-steps 0 > gpurun_out/prof_r6k_c3.log 2>&1; rc=$?; echo "c3 prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py gpurun_out/prof_r6k_c3/run_kernel_trace.csv > gpurun_out/timeline_r6k_c3.txt; cat gpurun_out/timeline_r6k_c3.txt
