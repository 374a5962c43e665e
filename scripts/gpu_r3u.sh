# Round 3: k_stream4's tail edge budget (queries past it go to the next tier once a wave's list is
# drained) -- parity tests, then the budget A/B on C2 (4 in flight).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 200 --timeout-method thread -k "synthetic_graph or bench_tune" > gpurun_out/pytest_r3u.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3u.log
[ $rc -eq 0 ] || exit $rc
TAG=r3u STEPS=60 ARGS="--parity 0 --latency-batches 0 --host-calls 0" ROUNDS=2 VARIANTS="-|- --stream-tail-ecap 256|- --stream-tail-ecap 64|- --stream-tail-ecap 16" bash scripts/gpu_ab.sh
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1; echo "list rc=$?"
