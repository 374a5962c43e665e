# GPU parity (all tiers incl. the 32-slot k_stream variants and the edge budget) + A/B of k_stream variants
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in "--stream 1" "--stream 3" "--stream 4" "--stream 1 --stream-ecap 256" "--stream 3 --grid-wgs 2"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 10 --warmup 3 $v > gpurun_out/ab_$i.log 2>&1; rc=$?
  echo "[$v] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$i.log; exit $rc; fi
  python - gpurun_out/ab_$i.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(" value=%.3e ms=%.3f k_stream_ms=%.3f tiers=%s diag=%s" % (d["value"], d["ms_per_step"], d["roofline"]["launch_ms"], d["tiers"], d["stream_diag"]))
PY
done
