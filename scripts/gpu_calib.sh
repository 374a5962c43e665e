# Calibrate FETCH_SIZE / TCC_EA0_RDREQ for random 16-B and 64-B gathers (tools/randprobe over a 32 GiB
# table: every load misses L2 and the Infinity Cache).  One counter set per rocprofv3 pass.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for B in 16 64; do
  for CT in FETCH_SIZE TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum; do
    timeout -s KILL 90 rocprofv3 --kernel-include-regex k_gather --pmc $CT -d gpurun_out/calib_${B}_${CT} -o run --output-format csv -- tools/randprobe 32 8 $B > gpurun_out/calib_${B}_${CT}.log 2>&1; rc=$?; echo "calib $B $CT rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    python3 scripts/pmc_calib.py --dir gpurun_out/calib_${B}_${CT} --counter $CT --bytes $B > gpurun_out/calib_${B}_${CT}.json; cat gpurun_out/calib_${B}_${CT}.json | cut -c1-600
  done
done
