# Round 3: sharded GPU tests after the pruning rule (no done bitmap when a node can error), then the
# one-batch kernel timeline of the C4 sharded batch with the flat hub kernel at threshold 64.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3q.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3q.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3q -o run --output-format csv -- python3 bench.py --mode sharded --steps 6 --warmup 2 --inflight 1 > gpurun_out/prof_r3q.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
t=$(find gpurun_out/prof_r3q -name '*kernel_trace.csv' | head -1); python3 - "$t" > gpurun_out/r3q_sharded_level_timeline.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
k = [r for r in rows if 'shard' in r.get('Kernel_Name', '')]
k.sort(key=lambda r: int(r['Start_Timestamp']))
seeds = [i for i, r in enumerate(k) if 'k_shard_seed' in r['Kernel_Name']]
last = k[seeds[-1]:]
t0 = int(last[0]['Start_Timestamp'])
print("one C4 sharded batch at world 1, one batch in flight (rocprofv3 --kernel-trace of bench.py --mode sharded --inflight 1)")
for r in last:
    print('%-28s start %8.1f us  dur %8.1f us' % (r['Kernel_Name'].split('(')[0][-28:], (int(r['Start_Timestamp']) - t0) / 1e3,
                                                (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
PY
cat gpurun_out/r3q_sharded_level_timeline.txt; tail -1 gpurun_out/prof_r3q.log | cut -c1-200
