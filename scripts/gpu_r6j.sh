# round 6: batches in flight (4 / 6 / 8) and stats on a subset of the timed batches, the headline alone as
# the driver runs it (20 steps, warm-up 5)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6j_inflight STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 60" VARIANTS="- --stats-every 5|- --stats-every 5 --inflight 6|- --stats-every 5 --inflight 8|- --stats-every 1000 --inflight 8|- --stats-every 5 --inflight 8 --hw-queues 32" ROUNDS=3 bash scripts/gpu_ab.sh
