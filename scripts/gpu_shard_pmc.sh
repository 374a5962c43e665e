# PMC passes over the sharded exchange protocol (tools/shard_ab.py, one configuration, one rank, forced
# exchange): fabric requests / L2 hits and wave waits of k_shard_level and k_shard_heavy.
# usage: gpurun -- 'TAG=r5c bash scripts/gpu_shard_pmc.sh'  env: CFG (default "-"), ABARGS
set -u
TAG=${TAG:-r5c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="python3 tools/shard_ab.py --rounds 1 --steps 3 --warmup 1 ${ABARGS:-} ${CFG:--}"
KRX="k_shard_level|k_shard_heavy|k_shard_seed"
PASSES=${PASSES:-TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY}
IFS='|' read -ra PS <<< "$PASSES"
i=0
for P in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "$KRX" --pmc $P -d gpurun_out/spmc_${TAG}_$i -o run --output-format csv -- $B > gpurun_out/spmc_${TAG}_$i.log 2>&1; rc=$?; echo "pmc$i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
