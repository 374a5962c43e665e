# round 6: C5 expand line (parity on) at HEAD, then the round's profiles (scripts/gpu_r6_prof.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode expand --inflight 8 --steps 6 --warmup 2 --cpu-seconds 0 > gpurun_out/expand_r6f.log 2>&1; rc=$?; echo "expand rc=$rc"; tail -1 gpurun_out/expand_r6f.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
TAG=r6f bash scripts/gpu_r6_prof.sh
