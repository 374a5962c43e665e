set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 400 python -m pytest tests -m gpu -q -rs -x > gpurun_out/pytest13.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/bench_m.log 2>&1; rc=$?; echo "bench rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1b_m -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/prof_1b_m.log 2>&1; rc=$?; echo "prof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_m -o run --output-format csv -- python3 bench.py --preset 1 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_c3_m.log 2>&1; rc=$?; echo "prof c3 rc=$rc"
exit $rc
