# PMC passes over the hot kernels (each counter group in its own rocprofv3 run, kernel trace only;
# no sys/runtime trace).  usage: bash scripts/gpu_pmc.sh TAG [KERNEL_REGEX]
set -u
TAG=${1:-r1}
KRE=${2:-k_stream|k_resolve|k_back|k_grid_level}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
B="python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$KRE" --pmc "$@" -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- $B > gpurun_out/pmc_${TAG}_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES
