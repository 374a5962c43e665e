# which queues / streams the headline's batches land on, --packed 0 vs 1 (kernel trace kept, k_resolve rows only)
set -u
TAG=${TAG:-r5p}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P="python3 bench.py --steps 30 --warmup 4 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
for K in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pks_${TAG}_p$K -o run --output-format csv -- $P --packed $K > gpurun_out/pks_${TAG}_p$K.log 2>&1; rc=$?; echo "trace p$K rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  f=$(ls gpurun_out/pks_${TAG}_p$K/*kernel_trace.csv | head -1)
  head -1 $f > gpurun_out/pks_${TAG}_p${K}_resolve.csv
  grep -E "k_resolve|k_stream4|k_grid_level" $f >> gpurun_out/pks_${TAG}_p${K}_resolve.csv || true
  rm -f $f
done
exit 0
