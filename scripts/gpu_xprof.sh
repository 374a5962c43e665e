# The default bench line (what the driver runs), then a rocprofv3 kernel trace of the sharded
# sub-line's exchange protocol at one batch in flight (RCCL kernels included) and its per-exchange
# timeline.  usage: gpurun -- 'TAG=r5x bash scripts/gpu_xprof.sh'   env: EXTRA (bench args), BENCH (0: skip)
set -u
TAG=${TAG:-r5x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python3 bench.py ${EXTRA:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; rc=$?
  echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_${TAG}.json
  [ $rc -eq 0 ] || exit $rc
fi
NOSUB="--steps 4 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof_${TAG} -o run --output-format csv -- python3 bench.py $NOSUB --sharded-steps 6 --sharded-warmup 2 --sharded-inflight 1 ${EXTRA:-} > gpurun_out/xprof_${TAG}.log 2>&1; rc=$?
echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
ANCHOR=k_shard_seed python3 scripts/timeline.py gpurun_out/xprof_${TAG}/run_kernel_trace.csv gaps > gpurun_out/xtimeline_${TAG}.txt || true
gzip -f gpurun_out/xprof_${TAG}/run_kernel_trace.csv
exit 0
