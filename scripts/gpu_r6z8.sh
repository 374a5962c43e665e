# round 6: C3 batches in flight (3 / 4 / 6) at the final code, same-box alternating 20-step lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6z8_c3_inflight STEPS=20 ARGS="--preset 1 --tuples 1e7 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 60" VARIANTS="- --inflight 6|- --inflight 4|- --inflight 3" ROUNDS=3 AB_TIMEOUT=150 bash scripts/gpu_ab.sh
