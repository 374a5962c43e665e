# level-kernel occupancy variants (forced exchange) and packed local records (one-rank device loop)
set -u
TAG=${TAG:-r5k}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/shard_ab.py - shard_level_occ=6 shard_level_occ=8 > gpurun_out/shard_ab_${TAG}_occ.jsonl 2> gpurun_out/shard_ab_${TAG}_occ.err; rc=$?; echo "occ rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/shard_ab.py --local shard_local=0 shard_local=0,shard_pack=1 shard_local=0,shard_level_occ=8 > gpurun_out/shard_ab_${TAG}_loop.jsonl 2> gpurun_out/shard_ab_${TAG}_loop.err; rc=$?; echo "loop rc=$rc"
exit $rc
