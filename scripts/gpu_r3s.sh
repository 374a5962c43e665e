# Round 3: where one C2 batch's latency goes at one batch in flight (kernel timeline), and the
# in-flight sweep with k_stream4 (throughput = batches in flight / batch latency).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3s -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --inflight 1 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 > gpurun_out/prof_r3s.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
t=$(find gpurun_out/prof_r3s -name '*kernel_trace.csv' | head -1)
python3 scripts/timeline.py "$t" k_ > gpurun_out/r3s_c2_p1_timeline.txt; cat gpurun_out/r3s_c2_p1_timeline.txt | head -60
: > gpurun_out/ab_r3sinflight.jsonl
for P in 2 4 6 8; do
  timeout -k 10 200 python bench.py --steps 60 --warmup 8 --inflight $P --cpu-seconds 0 --parity 0 --latency-batches 64 --host-calls 0 > gpurun_out/ab_one.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "P=$P rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; }
  tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['ab']='inflight '+sys.argv[1]; print(json.dumps(d))" $P >> gpurun_out/ab_r3sinflight.jsonl
  tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('P', sys.argv[1], '%.4g' % d['value'], 'p50', d.get('batch_ms_p50'), 'p99', d['p99_batch_ms'])" $P
done
