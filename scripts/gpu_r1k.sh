# kernel timeline of one batch (rocprofv3 kernel trace) + PMC traffic of k_stream with the current default
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1k -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/prof_r1k.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/prof_r1k.log | cut -c1-400
python3 scripts/timeline.py gpurun_out/prof_r1k/run_kernel_trace.csv gaps
B="python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_stream|k_resolve|k_back|k_grid_level" --pmc FETCH_SIZE -d gpurun_out/pmc_r1k_fetch -o run --output-format csv -- $B > gpurun_out/pmc_r1k_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_stream|k_resolve|k_back|k_grid_level" --pmc WRITE_SIZE -d gpurun_out/pmc_r1k_write -o run --output-format csv -- $B > gpurun_out/pmc_r1k_write.log 2>&1; rc=$?; echo "write rc=$rc"
exit $rc
