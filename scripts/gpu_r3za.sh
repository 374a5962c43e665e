# Round 3: packed local records in the one-rank sharded level loop -- sharded parity tests, then the
# A/B on C4 world 1 (4 in flight).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3za.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3za.log
[ $rc -eq 0 ] || exit $rc
TAG=r3za STEPS=30 ARGS="--mode sharded --warmup 5" ROUNDS=2 VARIANTS="- --shard-pack 0|- --shard-pack 1" bash scripts/gpu_ab.sh
