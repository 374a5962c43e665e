# Round 3: stream-tier work order (k_resolve puts likely-long walks first) -- parity tests, then the A/B
# on C2 at 4 in flight.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stream_order or synthetic_graph or bench_tune" > gpurun_out/pytest_r3x.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3x.log
[ $rc -eq 0 ] || exit $rc
TAG=r3x STEPS=60 ARGS="--parity 200000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=2 VARIANTS="-|- --stream-order 8|- --stream-order 32|- --stream-order 4:6|- --stream-order 2:8" bash scripts/gpu_ab.sh
