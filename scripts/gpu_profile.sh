# Round-1 evidence (4 batches in flight): GPU parity, rocprofv3 kernel stats + timeline, PMC traffic, default bench line
# passes (FETCH_SIZE, WRITE_SIZE) over the hot kernels, then the default bench line (with CPU baseline)
set -u
TAG=${TAG:-r1s}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --cpu-seconds 0 > gpurun_out/prof_${TAG}.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py gpurun_out/prof_${TAG}/run_kernel_trace.csv > gpurun_out/timeline_${TAG}.txt || true
B="python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_stream|k_resolve|k_back|k_grid_level" --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch -o run --output-format csv -- $B > gpurun_out/pmc_${TAG}_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_stream|k_resolve|k_back|k_grid_level" --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write -o run --output-format csv -- $B > gpurun_out/pmc_${TAG}_write.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
exit $rc
