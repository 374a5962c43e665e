# GPU tests + default bench + sharded-mode bench at 1 rank and at 2 ranks on the one GPU (gloo)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rs -x --timeout 150 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --mode sharded --steps 5 --warmup 2 > gpurun_out/bench_shard1.log 2>&1; rc=$?; echo "shard1 rc=$rc"; tail -1 gpurun_out/bench_shard1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode sharded --backend gloo --steps 3 --warmup 1 --tuples 2e8 > gpurun_out/bench_shard2.log 2>&1; rc=$?; echo "shard2 rc=$rc"; tail -1 gpurun_out/bench_shard2.log
exit $rc
