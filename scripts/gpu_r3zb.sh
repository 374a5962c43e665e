# Round-3 closing evidence, part B: C3 with kernel stats + PMC, C5 expand, C4 / C3 hash-sharded, the
# heavy-tail point, the host boundary, incremental refresh.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r3zc3 PRESET=1 INFLIGHT=6 CPU=8 bash scripts/gpu_profile.sh || exit $?
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_${tag}.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/bench_${tag}.log | cut -c1-260; return $rc; }
run r3z_expand --mode expand --cpu-seconds 6 || exit $?
run r3z_sharded --mode sharded --steps 40 --warmup 6 --cpu-seconds 0 || exit $?
run r3z_sharded_c3 --mode sharded --preset 1 --steps 20 --warmup 4 --cpu-seconds 0 || exit $?
run r3z_heavy --heavy-tail --batch 250000 --steps 8 --warmup 2 --cpu-seconds 6 --host-calls 0 --parity-canonical 0 || exit $?
run r3z_host --mode host || exit $?
run r3z_refresh --mode refresh || exit $?
