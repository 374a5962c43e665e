# Kernel-trace profile of the default bench (1B tuples) -> gpurun_out/prof_<tag>
set -u
TAG=${1:-cur}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/prof_$TAG.log 2>&1; rc=$?; echo "prof rc=$rc"
tail -1 gpurun_out/prof_$TAG.log
exit $rc
