# round 6: C5 callers in flight (24 / 20 / 16) inside the default line's layout (the parent's 1e9-tuple graph
# resident beside the expand child's), headline and the other sub-lines off
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/r6z9_c5_inflight.txt
for r in 1; do for P in 24 20 16; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --c3-steps 0 --heavy-steps 0 --sharded-steps 0 --parity 0 --latency-batches 0 --cpu-seconds 0 --host-calls 0 --parity-roots 0 --expand-inflight $P --expand-steps $((2*P)) > gpurun_out/r6z9_one.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "P=$P rc=$rc"; tail -5 gpurun_out/r6z9_one.log; exit $rc; }
  tail -1 gpurun_out/r6z9_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['expand']; print('C5 inflight %s: device %.4g trees/s, host path %.4g, call chain %s ms' % ($P, d['value'], d['host_path']['value'], (d.get('roofline') or {}).get('call_kernel_ms')) if 'value' in d else 'C5 inflight $P: ' + json.dumps(d)[:400])" | tee -a gpurun_out/r6z9_c5_inflight.txt
done; done
# C3's kernel stats, one-batch timeline and PMC traffic at its new operating point (3 in flight)
TAG=r6z9 PARTS="c3" SK=k_stream4 bash scripts/gpu_r6_final.sh || exit 1
