# round 6: 1024-edge grid tiles (keto_amd/lib/ab/grid4.so, -DKG_GRID_EPT=4) vs 512, C3 and the headline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r6s_grid4_c3 STEPS=20 ARGS="--preset 1 --tuples 1e7 --inflight 6 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 100000 --parity-canonical 10000 --latency-batches 60" VARIANTS="grid4.so|-" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
TAG=r6s_grid4 STEPS=20 ARGS="--warmup 5 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 200000 --parity-canonical 20000 --latency-batches 60" VARIANTS="grid4.so|-" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
