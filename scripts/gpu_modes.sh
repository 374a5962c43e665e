# The other bench modes on one GPU: C3 (OPL rewrites), C5 expand, world-1 sharded (RCCL), the heavy-tail point,
# the host boundary, incremental snapshot refresh (refresh: 1e7 tuples, refresh1b: 1e9).
# usage: gpurun -- 'TAG=r2x bash scripts/gpu_modes.sh'     env: MODES (default "expand sharded heavy host")
set -u
TAG=${TAG:-r2x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for M in ${MODES:-expand sharded heavy host}; do
  case $M in
    c3)      ARGS="--preset 1 --inflight 6 --steps 30 --warmup 6 --cpu-seconds 0" ;;
    expand)  ARGS="--mode expand --steps 10 --warmup 2 --cpu-seconds 0" ;;
    sharded) ARGS="--mode sharded --steps 20 --warmup 3 --cpu-seconds 0" ;;
    heavy)   ARGS="--heavy-tail --steps 20 --warmup 3 --batch 250000 --cpu-seconds 0" ;;
    host)    ARGS="--mode host --steps 10 --warmup 2 --cpu-seconds 0" ;;
    refresh) ARGS="--mode refresh --steps 20 --cpu-seconds 0" ;;
    refresh1b) ARGS="--mode refresh --steps 5 --tuples 1e9 --cpu-seconds 0" ;;
  esac
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/mode_${M}_${TAG}.log 2>&1; rc=$?; echo "$M rc=$rc"; tail -1 gpurun_out/mode_${M}_${TAG}.log | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
done
