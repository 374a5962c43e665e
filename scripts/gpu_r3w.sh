# Round-3 check after the node_bad change: whole GPU suite, smoke, default bench, sharded C4 bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r3w BENCH2="--mode sharded --steps 40 --warmup 6" bash scripts/gpu_tests.sh
