# Closing validation at the final code: the whole GPU suite, smoke, the default bench line (what the driver runs).
# usage: gpurun -- 'TAG=r6zz bash scripts/gpu_validate.sh'
TAG=${TAG:-r6zz}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 180 --timeout-method thread --durations 15 > gpurun_out/pytest_${TAG}.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${TAG}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.log 2>&1; rc=$?; echo "bench rc=$rc"
tail -1 gpurun_out/bench_${TAG}.log > gpurun_out/${TAG}_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('%.4g' % d['value'], d['roofline']['frac'], {k: (d[k].get('value') if isinstance(d[k], dict) else None) for k in ('c3','heavy','expand','sharded') if k in d})"
exit $rc
