# Where k_stream's wave cycles go: SQ counters (wait / issue / LDS) over a short single-stream bench,
# plus the kernel stats of the same command.  usage: TAG=r2d bash scripts/gpu_pmc_sq.sh
set -u
TAG=${TAG:-r2}
KRX=${KRX:-k_stream}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="python3 bench.py --steps ${STEPS:-6} --warmup 2 --cpu-seconds 0 --inflight ${INFLIGHT:-1} ${EXTRA:-}"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_${TAG}.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- $B > gpurun_out/prof_${TAG}.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
i=0
for P in "${PASS1:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS}" "${PASS2:-}" "${PASS3:-}"; do
  [ -n "$P" ] || continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$KRX" --pmc $P -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- $B > gpurun_out/pmc_${TAG}_$i.log 2>&1; rc=$?; echo "pmc$i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
