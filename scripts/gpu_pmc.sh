# PMC passes (each counter group in its own rocprofv3 run, kernel trace only; no sys/runtime trace)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
B="python3 bench.py --tuples 1e9 --steps 3 --warmup 1 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_write.log 2>&1; rc=$?; echo "write rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_tcc -o run --output-format csv -- $B > gpurun_out/pmc_tcc.log 2>&1; rc=$?; echo "tcc rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d gpurun_out/pmc_sq -o run --output-format csv -- $B > gpurun_out/pmc_sq.log 2>&1; rc=$?; echo "sq rc=$rc"
exit $rc
