# PMC passes over a short bench (one rocprofv3 run per pass: counters are never split over passes),
# plus the kernel stats of the same command.  usage: TAG=r4g KRX="k_stream4|k_resolve" \
#   PASSES="TCC_HIT_sum TCC_MISS_sum|SQ_WAVES SQ_WAVE_CYCLES" bash scripts/gpu_pmc_sq.sh
#   env: STEPS (6), INFLIGHT (1), EXTRA (bench args)
set -u
TAG=${TAG:-r2}
KRX=${KRX:-k_stream4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="python3 bench.py --steps ${STEPS:-6} --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --inflight ${INFLIGHT:-1} ${EXTRA:-}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- $B > gpurun_out/prof_${TAG}.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
PASSES=${PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS}
IFS='|' read -ra PS <<< "$PASSES"
i=0
for P in "${PS[@]}"; do
  [ -n "$P" ] || continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$KRX" --pmc $P -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- $B > gpurun_out/pmc_${TAG}_$i.log 2>&1; rc=$?; echo "pmc$i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
