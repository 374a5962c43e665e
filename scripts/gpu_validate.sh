# round 6 closing validation at the final code: the whole GPU suite, smoke, the default bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 180 --timeout-method thread --durations 15 > gpurun_out/pytest_r6zz.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r6zz.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6zz.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6zz.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_r6zz.log | cut -c1-300
