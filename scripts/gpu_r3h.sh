# Round 3: where the one-rank sharded batch spends its levels (records per level), and the forward
# edge budget (escalation to the backward phase) swept at 4 batches in flight.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KG_SHARD_TRACE=1 timeout -k 10 300 python bench.py --mode sharded --steps 4 --warmup 2 --inflight 1 > gpurun_out/bench_r3h_trace.log 2>&1; rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/bench_r3h_trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('level_records'))"
[ $rc -eq 0 ] || exit $rc
for SB in 0 512 2048 8192; do
  timeout -k 10 300 python bench.py --mode sharded --steps 20 --warmup 4 --shard-budget $SB > gpurun_out/bench_r3h_sb$SB.log 2>&1; rc=$?; echo "budget $SB rc=$rc"; tail -1 gpurun_out/bench_r3h_sb$SB.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p99_batch_ms'], d['backward_levels_per_batch'], d['final_levels_per_batch'])"
  [ $rc -eq 0 ] || exit $rc
done
# C3 (OPL view / edit / share): k_stream4 (default now) against k_stream2 at 6 batches in flight
TAG=r3hc3 STEPS=40 ARGS="--preset 1 --inflight 6 --back-wgs 1 --parity 0 --latency-batches 0 --host-calls 0" ROUNDS=2 VARIANTS="-|- --stream 12" bash scripts/gpu_ab.sh
# k_resolve without scratch: PMC (FETCH / WRITE) and the headline line
B="python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0"
for CT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_resolve|k_stream4" --pmc $CT -d gpurun_out/pmc_r3h_$CT -o run --output-format csv -- $B > gpurun_out/pmc_r3h_$CT.log 2>&1; rc=$?; echo "pmc $CT rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
for K in k_resolve k_stream4; do
  python3 scripts/pmc_summary.py --kernel $K --fetch gpurun_out/pmc_r3h_FETCH_SIZE --write gpurun_out/pmc_r3h_WRITE_SIZE --tuples 1e9 --batch 1000000 --preset 0 --inflight 4 --out gpurun_out/pmc_${K}_p0.json && python3 -c "import json; d=json.load(open('gpurun_out/pmc_${K}_p0.json')); print('$K', d['hbm_bytes_per_launch']/1e6, d['fetch_size_kib_raw'], d['write_size_kib_raw'])"
done
cp gpurun_out/pmc_k_*_p0.json profiles/
TAG=r3hv STEPS=100 ARGS="--parity 0 --latency-batches 0 --host-calls 0" ROUNDS=2 VARIANTS="-|- --stream 12" bash scripts/gpu_ab.sh
