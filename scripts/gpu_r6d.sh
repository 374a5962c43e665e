# round 6: C3 tier-knob A/B (same box, alternating): stream edge budget, backward budget, grid occupancy
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6d_c3 VARIANTS="-|- --stream-ecap 1024|- --stream-ecap 2048|- --back-edges 16384|- --back-wgs 2|- --grid-wgs 2" ROUNDS=2 STEPS=20 ARGS="--preset 1 --tuples 1e7 --inflight 6 --expand-steps 0 --c3-steps 0 --sharded-steps 0 --heavy-steps 0 --host-calls 0 --parity 0 --latency-batches 60" AB_TIMEOUT=150 bash scripts/gpu_ab.sh
