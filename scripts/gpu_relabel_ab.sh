# Upper bound of an in-degree relabelling: the headline with the generator's popularity permutation
# off (KG_SYNTH_IDENTITY=1: hot groups / users at the front of their id ranges) vs on, alternating,
# then TCC requests of the hot kernels with it off.  usage: gpurun -- 'TAG=r5f bash scripts/gpu_relabel_ab.sh'
set -u
TAG=${TAG:-r5f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps 40 --warmup 6 --cpu-seconds 0 --parity 200000 --parity-canonical 0 --latency-batches 200 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
for R in 1 2; do
  for I in 0 1; do
    KG_SYNTH_IDENTITY=$I timeout -k 10 300 python3 bench.py $B > gpurun_out/relabel_${TAG}_i${I}_r$R.json 2> gpurun_out/relabel_${TAG}_i${I}_r$R.err; rc=$?
    echo "identity=$I round=$R rc=$rc"; tail -1 gpurun_out/relabel_${TAG}_i${I}_r$R.json | cut -c1-160
    [ $rc -eq 0 ] || exit $rc
  done
done
P="python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0"
KG_SYNTH_IDENTITY=1 timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_stream4|k_resolve|k_back" --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/relabel_pmc_${TAG} -o run --output-format csv -- $P > gpurun_out/relabel_pmc_${TAG}.log 2>&1; rc=$?; echo "pmc rc=$rc"
exit $rc
