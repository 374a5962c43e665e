# round 6: C5's kernel stats and PMC traffic at its new operating point (20 calls in flight), then the headline at
# 3 vs 4 batches in flight (C3's best point moved to 3), same-box alternating 20-step lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6z10 PARTS="expand" SK=k_stream4 bash scripts/gpu_r6_final.sh || exit 1
TAG=r6z10_c2_inflight STEPS=20 ARGS="--warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 0 --latency-batches 120" VARIANTS="- --inflight 4|- --inflight 3" ROUNDS=3 bash scripts/gpu_ab.sh
