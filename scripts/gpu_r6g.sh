# round 6: the GPU suite, smoke and the default bench line at HEAD, then C5 at 16 calls in flight
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6g PYTEST_TIMEOUT=700 BENCH_EXTRA="--steps 20 --warmup 5" bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --mode expand --inflight 16 --hw-queues 32 --steps 8 --warmup 2 --cpu-seconds 0 --parity-roots 0 > gpurun_out/expand16_r6g.log 2>&1; rc=$?; echo "expand16 rc=$rc"; tail -1 gpurun_out/expand16_r6g.log | cut -c1-300
