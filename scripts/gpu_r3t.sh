# Round 3: k_stream5 (two interleaved FIFO engines per wave) -- stream-tier parity tests (variant 16
# included), then k_stream4 vs k_stream5 on C2 (4 in flight and one in flight).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stream_tier or random_graphs or synthetic_graph" > gpurun_out/pytest_r3t.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3t.log
[ $rc -eq 0 ] || exit $rc
TAG=r3t STEPS=60 ARGS="--parity 0 --latency-batches 0 --host-calls 0" ROUNDS=2 VARIANTS="-|- --stream 16|- --stream 16 --stream-wgs 4|- --inflight 1|- --inflight 1 --stream 16" bash scripts/gpu_ab.sh
