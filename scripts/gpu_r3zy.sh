# Round-3 closing check at HEAD: whole GPU suite, smoke, default bench, C3 bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r3zy BENCH2="--preset 1 --steps 30 --warmup 5" bash scripts/gpu_tests.sh
