# k_stream4 (variant 15) bring-up: its parity tests, then a same-box A/B against variant 12.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_check.py -q -x --timeout 120 --timeout-method thread -k "random_graphs or long_rows or synthetic_graph or bench_tune" > gpurun_out/pytest_s4.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_s4.log
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r3s4} STEPS=40 ARGS="--parity 200000 --parity-canonical 0 --latency-batches 0 --host-calls 0" ROUNDS=1 VARIANTS="${VARIANTS}" bash scripts/gpu_ab.sh
