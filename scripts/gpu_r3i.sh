# Round 3: the grid tier as MS-BFS (kg_msbfs.hip): GPU check tests, then the heavy-tail point with
# MS-BFS on / off (alternating), then the headline with it on (C2's grid tier stays per-query: its
# 2 x 10^8 nodes do not fit dense masks).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3i.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_r3i.log
[ $rc -eq 0 ] || exit $rc
TAG=r3iheavy STEPS=6 ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 50000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=1 VARIANTS="- --grid-ms 1|- --grid-ms 0|- --grid-ms-tg-cap 0|- --grid-ms-tg-cap 4096" bash scripts/gpu_ab.sh
