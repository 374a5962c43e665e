# Round 3: where the one-rank sharded batch spends its time -- hub-row threshold A/B (rows expanded
# grid-wide vs by their workgroup) and a kernel trace at one batch in flight.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab_r3nshard.jsonl
for r in 1 2; do
  for H in 4096 16384 1024; do
    timeout -k 10 200 python bench.py --mode sharded --steps 20 --warmup 4 --shard-heavy $H > gpurun_out/ab_one.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "H=$H rc=$rc"; tail -5 gpurun_out/ab_one.log; exit $rc; }
    tail -1 gpurun_out/ab_one.log >> gpurun_out/ab_r3nshard.jsonl
    tail -1 gpurun_out/ab_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('heavy', d['shard_heavy'], '%.4g' % d['value'], d['ms_per_step'], d['p99_batch_ms'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3n -o run --output-format csv -- python3 bench.py --mode sharded --steps 6 --warmup 2 --inflight 1 > gpurun_out/prof_r3n.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_r3n -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r3n_sharded_kernel_stats.csv; head -14 gpurun_out/r3n_sharded_kernel_stats.csv | cut -c1-160
t=$(find gpurun_out/prof_r3n -name '*kernel_trace.csv' | head -1); python3 - "$t" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
k = [r for r in rows if 'shard' in r.get('Kernel_Name', '')]
k.sort(key=lambda r: int(r['Start_Timestamp']))
# the last batch: from the last k_shard_seed on
seeds = [i for i, r in enumerate(k) if 'k_shard_seed' in r['Kernel_Name']]
last = k[seeds[-1]:] if seeds else k
t0 = int(last[0]['Start_Timestamp'])
for r in last:
    print('%-28s start %8.1f us  dur %8.1f us' % (r['Kernel_Name'].split('(')[0][-28:], (int(r['Start_Timestamp']) - t0) / 1e3,
                                                (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
PY
