# Heavy-tail point (P(k) ~ k^-1.5, bench.py --heavy-tail: 62.5 k checks x 2 in flight) with adjx in node
# order vs hot-first, alternating.  usage: gpurun -- 'TAG=r5r bash scripts/gpu_heavy_hot_ab.sh'
set -u
TAG=${TAG:-r5r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--heavy-tail --steps 200 --warmup 10 --cpu-seconds 0 --parity 50000 --parity-canonical 0 --latency-batches 100 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
for R in 1 2; do
  for O in 0 1; do
    KG_ADJX_ORDER=$O timeout -k 10 300 python3 bench.py $B > gpurun_out/hh_${TAG}_o${O}_r$R.json 2> gpurun_out/hh_${TAG}_o${O}_r$R.err; rc=$?
    echo "order=$O round=$R rc=$rc"; tail -1 gpurun_out/hh_${TAG}_o${O}_r$R.json | cut -c1-120
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
