# Round 3 re-entry: the whole GPU suite + smoke + the default bench line on HEAD (MS-BFS grid tier
# on by default), then the heavy-tail point with MS-BFS on / off.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r3j BENCH_EXTRA="--steps 40 --warmup 8" bash scripts/gpu_tests.sh; rc=$?
[ $rc -eq 0 ] || exit $rc
TAG=r3jheavy STEPS=6 ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 50000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=1 VARIANTS="- --grid-ms 1|- --grid-ms 0" bash scripts/gpu_ab.sh
