# Round 3: expand largest-root walk A/B, sharded kernel profile, stream-variant A/B at the headline.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 1 0; do
  timeout -k 10 300 python bench.py --mode expand --steps 8 --warmup 4 --expand-tail $v --parity-roots 0 > gpurun_out/bench_r3e_expand_$v.log 2>&1; rc=$?; echo "expand tail=$v rc=$rc"; tail -1 gpurun_out/bench_r3e_expand_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_per_step'], d['largest_root'])"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3e_shard -o run --output-format csv -- python3 bench.py --mode sharded --steps 10 --warmup 2 > gpurun_out/prof_r3e_shard.log 2>&1; rc=$?; echo "shard prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
TAG=r3evar STEPS=60 ARGS="--parity 0 --latency-batches 0 --host-calls 0" ROUNDS=3 VARIANTS="-|- --stream 15 --stream-chunk 64|- --stream 15 --stream-chunk 32" bash scripts/gpu_ab.sh
