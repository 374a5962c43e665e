# profile + PMC traffic of the default bench, and the 2-rank sharded rehearsal (gloo, one GPU)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1g -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/prof_r1g.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_stream|k_resolve|k_back|k_grid_level" --pmc FETCH_SIZE -d gpurun_out/pmc_r1g_fetch -o run --output-format csv -- $B > gpurun_out/pmc_r1g_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_stream|k_resolve|k_back|k_grid_level" --pmc WRITE_SIZE -d gpurun_out/pmc_r1g_write -o run --output-format csv -- $B > gpurun_out/pmc_r1g_write.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode sharded --backend gloo --steps 3 --warmup 1 --tuples 2e8 > gpurun_out/bench_shard2.log 2>&1; rc=$?; echo "shard2 rc=$rc"; tail -1 gpurun_out/bench_shard2.log
exit $rc
