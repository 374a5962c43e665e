# Round 3: stream-tier work order with small claims inside the front run (a 64-query chunk of it puts
# 64 long walks on one wave) -- parity tests, then the A/B on C2 at 4 in flight.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stream_order or synthetic_graph or bench_tune" > gpurun_out/pytest_r3y.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3y.log
[ $rc -eq 0 ] || exit $rc
TAG=r3y STEPS=60 ARGS="--parity 200000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=2 VARIANTS="-|- --stream-order 8 --stream-big-chunk 2|- --stream-order 32 --stream-big-chunk 1|- --stream-order 2:8 --stream-big-chunk 2|- --stream-order 8 --stream-chunk 8 --stream-big-chunk 1" bash scripts/gpu_ab.sh
