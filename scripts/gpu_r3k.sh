# Round 3: the heavy-tail point's MS-BFS grid tier -- mask words per group and the mask budget per
# workspace (rounds per batch), then kernel stats of the default.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r3kheavy STEPS=6 ARGS="--heavy-tail --batch 250000 --warmup 2 --parity 0 --latency-batches 0 --host-calls 0" ROUNDS=1 VARIANTS="- --grid-ms-words 8|- --grid-ms-words 16|- --grid-ms-words 8 --grid-ms-bytes 8e9|- --grid-ms-words 16 --grid-ms-bytes 8e9|- --grid-ms-words 16 --grid-ms-bytes 16e9" bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3k -o run --output-format csv -- python3 bench.py --heavy-tail --batch 250000 --steps 4 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 > gpurun_out/prof_r3k.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_r3k -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r3k_heavy_kernel_stats.csv; head -15 gpurun_out/r3k_heavy_kernel_stats.csv | cut -c1-200
