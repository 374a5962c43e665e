# Packed device queries: their GPU tests, then the headline with 28-B kg_query (--packed 0) vs 16-B packed,
# alternating, and k_resolve's TCC requests for both.  usage: gpurun -- 'TAG=r5m bash scripts/gpu_packed_ab.sh'
set -u
TAG=${TAG:-r5m}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q -k "packed" --timeout 180 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_${TAG}.log
[ $rc -eq 0 ] || exit $rc
B="--steps 60 --warmup 6 --cpu-seconds 0 --parity 200000 --parity-canonical 0 --latency-batches 200 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
for R in 1 2; do
  for K in 0 1; do
    timeout -k 10 300 python3 bench.py $B --packed $K > gpurun_out/pk_${TAG}_p${K}_r$R.json 2> gpurun_out/pk_${TAG}_p${K}_r$R.err; rc=$?
    echo "packed=$K round=$R rc=$rc"; tail -1 gpurun_out/pk_${TAG}_p${K}_r$R.json | cut -c1-120
    [ $rc -eq 0 ] || exit $rc
  done
done
P="python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
for K in 0 1; do
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_stream4|k_resolve" --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pk_pmc_${TAG}_p$K -o run --output-format csv -- $P --packed $K > gpurun_out/pk_pmc_${TAG}_p$K.log 2>&1; rc=$?; echo "pmc p$K rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
