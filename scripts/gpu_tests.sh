# GPU parity suite + smoke + default bench line, then an optional second bench (BENCH2 args).
# usage: gpurun -- 'bash scripts/gpu_tests.sh'
#   env: TESTS="tests -m gpu" (pytest args), TAG=r2a (log suffix), BENCH=1 (0 skips the default
#        bench), BENCH_EXTRA (args of the default bench), BENCH2 (args of a second bench run),
#        PYTEST_X ("" runs past failures; default -x), PYTEST_TIMEOUT (seconds, 900), KEXPR (pytest -k
#        expression, may hold spaces)
set -u
TAG=${TAG:-r2}
TESTS=${TESTS:-tests -m gpu}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -q -rs ${PYTEST_X--x} --timeout 180 --timeout-method thread --durations 15 > gpurun_out/pytest_${TAG}.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${TAG}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1; rc=$?; echo "smoke rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py ${BENCH_EXTRA:-} > gpurun_out/bench_${TAG}.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_${TAG}.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BENCH2:-}" ]; then
  timeout -k 10 300 python bench.py $BENCH2 > gpurun_out/bench2_${TAG}.log 2>&1; rc=$?; echo "bench2 rc=$rc"; tail -1 gpurun_out/bench2_${TAG}.log | cut -c1-600
fi
exit $rc
