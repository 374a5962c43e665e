# Round-1 closing evidence: full GPU parity, smoke, default bench line, C3 bench + kernel stats
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --preset 1 --cpu-seconds 0 > gpurun_out/r1w_c3.log 2>&1; rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/r1w_c3.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1w_c3 -o run --output-format csv -- python3 bench.py --preset 1 --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/prof_r1w_c3.log 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
