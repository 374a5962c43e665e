# round 6: the C3 sub-line (inside the default line's process, after the headline) at 3 vs 6 batches in flight,
# alternating on one box; then C3 stream workgroups per CU (2 / 3 / 4) standalone at 3 in flight
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/r6z11_c3_subline.txt
for r in 1 2 3; do for P in 3 6; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --parity 0 --latency-batches 0 --cpu-seconds 0 --host-calls 0 --c3-parity 0 --c3-inflight $P > gpurun_out/r6z11_one.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "P=$P rc=$rc"; tail -5 gpurun_out/r6z11_one.log; exit $rc; }
  tail -1 gpurun_out/r6z11_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['c3']; print('C3 sub-line inflight $P: %.4g checks/s, ms/step %.3f' % (d['value'], d['ms_per_step']) if 'value' in d else json.dumps(d)[:300])" | tee -a gpurun_out/r6z11_c3_subline.txt
done; done
TAG=r6z11_c3_stream_wgs STEPS=20 ARGS="--preset 1 --tuples 1e7 --inflight 3 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 60" VARIANTS="- --stream-wgs 3|- --stream-wgs 4|- --stream-wgs 2" ROUNDS=2 AB_TIMEOUT=150 bash scripts/gpu_ab.sh
