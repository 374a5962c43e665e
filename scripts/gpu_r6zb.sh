# round 6 closing line at the final code (C3 sub-line at 6 in flight, C5 at 20): the default bench line, twice
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 700 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6zb$r.log 2>&1; rc=$?; echo "bench $r rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/bench_r6zb$r.log > gpurun_out/r6zb${r}_bench.json
  python3 -c "import json; d=json.load(open('gpurun_out/r6zb${r}_bench.json')); print('%.4g' % d['value'], '%.4g' % d['steady']['value'], d['roofline']['frac'], {k: (d[k].get('value') if isinstance(d[k], dict) else None) for k in ('c3','heavy','expand','sharded') if k in d})"
done
