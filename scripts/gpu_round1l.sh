set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 400 python -m pytest tests -m gpu -q -rs -x > gpurun_out/pytest12.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench default rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1b_l -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/prof_1b_l.log 2>&1; rc=$?; echo "prof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_fetch.log 2>&1; rc=$?; echo "pmc fetch rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_write.log 2>&1; rc=$?; echo "pmc write rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --preset 1 --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench_c3.log 2>&1; rc=$?; echo "bench c3 rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --mode expand --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench_c5.log 2>&1; rc=$?; echo "bench c5 rc=$rc"
exit $rc
