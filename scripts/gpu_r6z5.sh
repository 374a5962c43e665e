# round 6 closing (k_stream4 with a 256-key visited cache: 5 workgroups per CU): the check-path GPU tests and smoke,
# a same-box A/B against the 512-key build (keto_amd/lib/ab/vt9.so) on C3 and the heavy-tail point, the closing
# profiles (kernel stats, timelines, PMC traffic of C2 / C3 / heavy; scripts/gpu_r6_final.sh), then the default
# bench line reading the new PMC summaries
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_check.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6z5.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r6z5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6z5.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=r6z5_vt_c3 STEPS=20 ARGS="--preset 1 --tuples 1e7 --inflight 6 --warmup 6 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 100000 --parity-canonical 10000 --latency-batches 60" VARIANTS="vt9.so|-" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
TAG=r6z5_vt_heavy STEPS=20 ARGS="--heavy-tail --warmup 4 --c3-steps 0 --heavy-steps 0 --expand-steps 0 --sharded-steps 0 --host-calls 0 --parity 20000 --parity-canonical 5000 --latency-batches 60" VARIANTS="vt9.so|-" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
TAG=r6z5 PARTS="c2 c3 heavy" SK=k_stream4 bash scripts/gpu_r6_final.sh || exit 1
cp gpurun_out/pmc_k_*_p0.json gpurun_out/pmc_k_*_p1.json gpurun_out/pmc_k_*_p0h.json profiles/ 2>/dev/null
timeout -k 10 900 python bench.py > gpurun_out/bench_r6z5.log 2>&1; rc=$?; echo "bench rc=$rc"
tail -1 gpurun_out/bench_r6z5.log > gpurun_out/r6z5_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/r6z5_bench.json')); print('%.4g' % d['value'], d['roofline']['frac'], {k: (d[k].get('value') if isinstance(d[k], dict) else None) for k in ('c3','heavy','expand','sharded') if k in d})"
exit $rc
