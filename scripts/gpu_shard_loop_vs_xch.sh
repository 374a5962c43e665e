# k_shard_level per record: the one-rank device loop (per-XCD bucket counters) vs the forced exchange
# (one counter per destination), kernel stats of each.  usage: gpurun -- 'TAG=r5i bash scripts/gpu_shard_loop_vs_xch.sh'
set -u
TAG=${TAG:-r5i}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lvx_${TAG}_loop -o run --output-format csv -- python3 tools/shard_ab.py --rounds 1 --local shard_local=0 > gpurun_out/lvx_${TAG}_loop.log 2>&1; rc=$?; echo "loop rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lvx_${TAG}_xch -o run --output-format csv -- python3 tools/shard_ab.py --rounds 1 - > gpurun_out/lvx_${TAG}_xch.log 2>&1; rc=$?; echo "xch rc=$rc"
rm -f gpurun_out/lvx_${TAG}_*/run_kernel_trace.csv
exit $rc
