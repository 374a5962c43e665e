# Round evidence for one workload: rocprofv3 kernel stats + timeline of the bench, PMC HBM traffic
# (FETCH_SIZE and WRITE_SIZE, one pass each) of the hot kernels, summarised for bench.py's
# roofline.traffic, then the bench line itself.
# usage: gpurun -- 'TAG=r2p bash scripts/gpu_profile.sh'   env: EXTRA (bench args, e.g. "--preset 1
#        --inflight 6"), PRESET (0/1, names the PMC summary), TUPLES (1e9), INFLIGHT (4), CPU (bench
#        CPU-baseline seconds for the final line, default 12)
set -u
TAG=${TAG:-r2p}
PRESET=${PRESET:-0}
TUPLES=${TUPLES:-1e9}
INFLIGHT=${INFLIGHT:-4}
EXTRA="--preset $PRESET --tuples $TUPLES --inflight $INFLIGHT ${EXTRA:-}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NOSUB="--expand-steps 0 --c3-steps 0 --sharded-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 40 --warmup 6 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 $NOSUB $EXTRA > gpurun_out/prof_${TAG}.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py gpurun_out/prof_${TAG}/run_kernel_trace.csv > gpurun_out/timeline_${TAG}.txt || true
B="python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 $NOSUB $EXTRA"
RX="k_stream4|k_resolve|k_back|k_grid_level|k_fsplit"
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch -o run --output-format csv -- $B > gpurun_out/pmc_${TAG}_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write -o run --output-format csv -- $B > gpurun_out/pmc_${TAG}_write.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
for K in k_stream4 k_resolve k_back; do
  python3 scripts/pmc_summary.py --kernel $K --fetch gpurun_out/pmc_${TAG}_fetch --write gpurun_out/pmc_${TAG}_write --tuples $TUPLES --batch 1000000 --preset $PRESET --inflight $INFLIGHT --out profiles/pmc_${K}_p${PRESET}.json > /dev/null || true
done
cp profiles/pmc_k_*_p${PRESET}.json gpurun_out/ 2>/dev/null || true  # the bench below reads them; copied back for committing
timeout -k 10 300 python bench.py --cpu-seconds ${CPU:-12} $EXTRA > gpurun_out/bench_${TAG}.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_${TAG}.log | cut -c1-300
exit $rc
