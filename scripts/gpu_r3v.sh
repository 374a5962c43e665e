# Does TCC_EA0_RDREQ_DRAM separate Infinity-Cache hits from HBM reads?  tools/randprobe's random
# 16-B gathers over a 32 GiB table (every load misses the 256 MiB Infinity Cache) and over a 64 MiB
# one (misses the 4 MiB per-XCD L2, stays in the Infinity Cache); one counter per rocprofv3 pass.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for G in 32 0.0625; do
  for CT in TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_128B_sum; do
    timeout -s KILL 90 rocprofv3 --kernel-include-regex k_gather --pmc $CT -d gpurun_out/cal2_${G}_${CT} -o run --output-format csv -- tools/randprobe $G 8 16 > gpurun_out/cal2_${G}_${CT}.log 2>&1; rc=$?; echo "cal $G $CT rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    python3 scripts/pmc_calib.py --dir gpurun_out/cal2_${G}_${CT} --counter $CT --bytes 16 > gpurun_out/cal2_${G}_${CT}.json
    python3 -c "import json,sys;d=json.load(open('gpurun_out/cal2_${G}_${CT}.json'));print('$G','$CT',[round(x['per_load'],3) for x in d['dispatches']])"
  done
done
