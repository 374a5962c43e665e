# Round-3 closing evidence, part A: the whole GPU suite + smoke, the C2 headline with rocprof kernel
# stats / timeline / PMC traffic (scripts/gpu_profile.sh), and C2 at round 2's graph size.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r3z BENCH=0 bash scripts/gpu_tests.sh || exit $?
TAG=r3z bash scripts/gpu_profile.sh || exit $?
timeout -k 10 300 python bench.py --tuples 9.45e8 --steps 100 --warmup 10 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 > gpurun_out/bench_r3z_r2size.log 2>&1; rc=$?; echo "r2-size rc=$rc"; tail -1 gpurun_out/bench_r3z_r2size.log | cut -c1-300
