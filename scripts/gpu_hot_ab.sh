# Hot-first adjx: the full GPU suite, then the headline with adjx in node order (KG_ADJX_ORDER=0) vs
# hot-first, alternating, and TCC requests of the hot kernels for both.
# usage: gpurun -- 'TAG=r5g bash scripts/gpu_hot_ab.sh'   env: TESTS (0 skips the suite)
set -u
TAG=${TAG:-r5g}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${TAG}.log
  [ $rc -eq 0 ] || exit $rc
fi
B="--steps 40 --warmup 6 --cpu-seconds 0 --parity 200000 --parity-canonical 0 --latency-batches 200 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
for R in 1 2; do
  for O in 0 1; do
    KG_ADJX_ORDER=$O timeout -k 10 300 python3 bench.py $B > gpurun_out/hot_${TAG}_o${O}_r$R.json 2> gpurun_out/hot_${TAG}_o${O}_r$R.err; rc=$?
    echo "order=$O round=$R rc=$rc"; tail -1 gpurun_out/hot_${TAG}_o${O}_r$R.json | cut -c1-120
    [ $rc -eq 0 ] || exit $rc
  done
done
P="python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
for O in 0 1; do
  KG_ADJX_ORDER=$O timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_stream4|k_resolve|k_back" --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/hot_pmc_${TAG}_o$O -o run --output-format csv -- $P > gpurun_out/hot_pmc_${TAG}_o$O.log 2>&1; rc=$?; echo "pmc o$O rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
