# k_stream step time vs graph size (TLB / cache reach vs instruction latency), k_back 4 edges per thread
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 4
timeout -k 10 300 python -u -m pytest tests/test_gpu_check.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in "--stream 5" "--stream 4"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 10 --warmup 3 $v > gpurun_out/ab_$i.log 2>&1; rc=$?
  echo "[$v] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$i.log; exit $rc; fi
  python - gpurun_out/ab_$i.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g=d["stream_diag"]
print(" value=%.3e ms=%.3f k_stream_ms=%.3f us/step=%.2f diag=%s tiers=%s work=%s" % (d["value"], d["ms_per_step"], d["roofline"]["launch_ms"], g["mean_wave_us"]/max(g["steps_per_wave"],1e-9), g, d["tiers"], d["work_per_batch"]))
PY
done
