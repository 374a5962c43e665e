# round 6: operating points -- heavy-tail batches in flight (p99 bound 50 ms), C5 callers at 32 queues,
# C3 grid / stream workgroups per CU at the round's code
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/r6t_points.txt
for P in 2 3 4 6; do
  timeout -k 10 300 python bench.py --heavy-tail --inflight $P --steps 20 --warmup 4 --cpu-seconds 0 --parity 0 --latency-batches 120 --host-calls 0 > gpurun_out/heavy_r6t_$P.log 2>&1; rc=$?; echo "heavy $P rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/heavy_r6t_$P.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('heavy inflight $P: %.4g checks/s steady %.4g p99 %.1f ms' % (d['value'], d['steady']['value'], d['p99_batch_ms']))" | tee -a gpurun_out/r6t_points.txt
done
for P in 12 16 20; do
  timeout -k 10 300 python bench.py --mode expand --inflight $P --steps $((2 * P)) --warmup $P --cpu-seconds 0 --parity-roots 0 --hw-queues 32 > gpurun_out/expand_r6t_$P.log 2>&1; rc=$?; echo "expand $P rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/expand_r6t_$P.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 inflight $P (32 queues): device %.4g trees/s, host path %.4g' % (d['value'], d['host_path']['value']))" | tee -a gpurun_out/r6t_points.txt
done
for G in "--grid-wgs 4 --stream-wgs 3" "--grid-wgs 6 --stream-wgs 3" "--grid-wgs 4 --stream-wgs 2" "--grid-wgs 4 --stream-wgs 3 --inflight 8"; do
  timeout -k 10 300 python bench.py --preset 1 --tuples 1e7 --inflight 6 --steps 20 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --cpu-seconds 0 --latency-batches 60 $G > gpurun_out/c3_r6t.log 2>&1; rc=$?; echo "c3 [$G] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/c3_r6t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3 [$G]: %.4g checks/s steady %.4g' % (d['value'], d['steady']['value']))" | tee -a gpurun_out/r6t_points.txt
done
