# round 6: staggered callers (the four in-flight batches otherwise run their tail tiers in lockstep) on the
# headline, and the C5 sub-line's hardware queues (16 vs 32)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6o_stagger STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 60" VARIANTS="-|- --stagger-us 130|- --stagger-us 260" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
for Q in 16 32; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --c3-steps 0 --heavy-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 0 --parity-roots 0 --hw-queues $Q > gpurun_out/c5q_r6o_$Q.log 2>&1; rc=$?; echo "c5 q$Q rc=$rc"; tail -1 gpurun_out/c5q_r6o_$Q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['expand']; print('headline %.4g' % d['value'], 'expand %.4g' % e['value'], 'host %.4g' % e['host_path']['value'], e['ms_per_step'])"
  [ $rc -eq 0 ] || exit $rc
done
