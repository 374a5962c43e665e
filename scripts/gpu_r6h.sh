# round 6 (second session): kernel trace of the driver's 20-step headline timed region, then an A/B of
# stats on every timed batch vs none (headline only, sub-lines off)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
HL="--steps 20 --warmup 5 --cpu-seconds 0 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0"
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/prof_r6h -o run --output-format csv -- python3 bench.py $HL --latency-batches 0 > gpurun_out/prof_r6h.log 2>&1; rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/prof_r6h.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
TAG=r6h_stats STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 60" VARIANTS="-|- --stats-every 1000" ROUNDS=3 bash scripts/gpu_ab.sh
