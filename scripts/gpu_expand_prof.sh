# C5 evidence: the expand bench line and a rocprofv3 kernel-stats profile of the same command.
set -u
TAG=${TAG:-r2x2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --mode expand --steps 10 --warmup 2 > gpurun_out/expand_${TAG}.json 2> gpurun_out/expand_${TAG}.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --mode expand --steps 6 --warmup 2 > gpurun_out/prof_${TAG}.log 2>&1; rc=$?; echo "prof rc=$rc"
rm -f gpurun_out/prof_${TAG}/run_kernel_trace.csv
exit $rc
