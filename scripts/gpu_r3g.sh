# Round 3: grid-bidir off by default + staged slot state in k_grid_level + coalesced LQuery appends:
# GPU check tests, heavy-tail point, headline bench, PMC of k_resolve, FETCH_SIZE calibration.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3g.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3g.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --heavy-tail --tuples 1.2e8 --batch 250000 --steps 6 --warmup 4 --cpu-seconds 0 --host-calls 0 --parity-canonical 0 > gpurun_out/bench_r3g_heavy.log 2>&1; rc=$?; echo "heavy rc=$rc"; tail -1 gpurun_out/bench_r3g_heavy.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('p99_batch_ms'), d['edges_per_batch'], d['parity']['mismatches'])"
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0"
for CT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_resolve|k_stream4" --pmc $CT -d gpurun_out/pmc_r3g_$CT -o run --output-format csv -- $B > gpurun_out/pmc_r3g_$CT.log 2>&1; rc=$?; echo "pmc $CT rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
for K in k_resolve k_stream4; do
  python3 scripts/pmc_summary.py --kernel $K --fetch gpurun_out/pmc_r3g_FETCH_SIZE --write gpurun_out/pmc_r3g_WRITE_SIZE --tuples 1e9 --batch 1000000 --preset 0 --inflight 4 --out gpurun_out/pmc_${K}_p0.json && python3 -c "import json; d=json.load(open('gpurun_out/pmc_${K}_p0.json')); print('$K', d['hbm_bytes_per_launch']/1e6, d['fetch_size_kib_raw'], d['write_size_kib_raw'])"
done
bash scripts/gpu_calib.sh
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --host-calls 0 > gpurun_out/bench_r3g.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_r3g.log | cut -c1-400
