# Secondary bench lines: C3 (rewrites, preset 1), C5 (expand), hash-sharded mode at world 1
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --preset 1 --cpu-seconds 0 > gpurun_out/r1w_c3.log 2>&1; rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/r1w_c3.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --mode expand --cpu-seconds 0 > gpurun_out/r1w_c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/r1w_c5.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --mode sharded --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/r1w_sharded.log 2>&1; rc=$?; echo "sharded rc=$rc"; tail -1 gpurun_out/r1w_sharded.log | cut -c1-400
exit $rc
