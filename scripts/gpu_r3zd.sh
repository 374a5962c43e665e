# Round-3 closing evidence, part D: the heavy-tail point, the host boundary, incremental refresh, and
# the C3 hash-sharded line (records-left diagnosis after the overflow-first check).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_${tag}.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/bench_${tag}.log | cut -c1-260; return $rc; }
run r3z_heavy --heavy-tail --batch 250000 --steps 8 --warmup 2 --cpu-seconds 6 --host-calls 0 --parity-canonical 0 || exit $?
run r3z_host --mode host || exit $?
run r3z_refresh --mode refresh || exit $?
run r3z_sharded_c3s --mode sharded --preset 1 --tuples 1e8 --steps 10 --warmup 2 --cpu-seconds 0
run r3z_sharded_c3 --mode sharded --preset 1 --steps 20 --warmup 4 --cpu-seconds 0
exit 0
