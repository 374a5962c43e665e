set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 400 python -m pytest tests -m gpu -q -rs -x > gpurun_out/pytest11.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for w in 1 0; do
timeout -k 10 200 python bench.py --wide $w --tuples 1e9 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_1b_k_w$w.log 2>&1; rc=$?; echo "bench1b wide=$w rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
