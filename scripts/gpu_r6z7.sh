# round 6: batches in flight on the headline at the final code (k_stream4 now 25.5 KB of LDS per workgroup:
# more of the in-flight batches' stream workgroups fit per CU), 4 / 5 / 6, same-box alternating 20-step lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6z7_inflight STEPS=20 ARGS="--warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 120" VARIANTS="- --inflight 4|- --inflight 5|- --inflight 6" ROUNDS=3 bash scripts/gpu_ab.sh
