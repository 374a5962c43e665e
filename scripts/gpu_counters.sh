# Which memory-side counters this rocprofv3 exposes (looking for DRAM vs Infinity-Cache splits).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1; rc=$?; echo "list rc=$rc"
grep -i -E "TCC_EA|DRAM|MALL|HBM|FETCH|WRITE_SIZE|RDREQ" gpurun_out/rocprof_counters.txt | sort -u | head -60
