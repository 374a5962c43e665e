set -u
mkdir -p gpurun_out
nproc > gpurun_out/host.txt; grep -m1 "model name" /proc/cpuinfo >> gpurun_out/host.txt; rocm-smi --showproductname >> gpurun_out/host.txt 2>&1
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 420 python -m pytest tests -m gpu -q > gpurun_out/pytest1.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --tuples 1e7 --steps 5 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_10m.log 2>&1; rc=$?; echo "bench10m rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --tuples 1e9 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_1b.log 2>&1; rc=$?; echo "bench1b rc=$rc"
exit $rc
