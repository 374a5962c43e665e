# Debug the C3 sharded leftover records; refresh bench at round 2's step count.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/dbg/sharded_c3_left.py 1e8 > gpurun_out/dbg_c3left.log 2>&1; rc=$?; echo "dbg rc=$rc"; grep -v "^\[W\|amdgpu.ids" gpurun_out/dbg_c3left.log | tail -12
timeout -k 10 300 python bench.py --mode refresh --steps 20 > gpurun_out/bench_r3z_refresh20.log 2>&1; rc=$?; echo "refresh rc=$rc"; tail -1 gpurun_out/bench_r3z_refresh20.log | cut -c1-400
