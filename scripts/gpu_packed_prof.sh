# kernel stats of the headline with --packed 0 / 1 (why is the packed path slower?)
set -u
TAG=${TAG:-r5n}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P="python3 bench.py --steps 30 --warmup 4 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
for K in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pkp_${TAG}_p$K -o run --output-format csv -- $P --packed $K > gpurun_out/pkp_${TAG}_p$K.log 2>&1; rc=$?; echo "prof p$K rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 scripts/timeline.py gpurun_out/pkp_${TAG}_p$K/run_kernel_trace.csv gaps > gpurun_out/pkp_${TAG}_p${K}_timeline.txt || true
  rm -f gpurun_out/pkp_${TAG}_p$K/run_kernel_trace.csv
done
exit 0
