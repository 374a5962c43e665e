"""Per-batch kernel timeline from a rocprofv3 kernel trace (gaps included): python scripts/timeline.py run_kernel_trace.csv"""
import csv
import os
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "")).replace("kg::", "").replace("void ", "")[:40]
# batches start at k_resolve (ANCHOR: another kernel, e.g. k_shard_seed); show the last complete one
anchor = os.environ.get("ANCHOR", "k_resolve")
starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
b0, b1 = starts[-2], starts[-1]
t0 = int(rows[b0]["Start_Timestamp"])
agg = {}
prev_end = t0
gap = 0
for r in rows[b0:b1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap += max(0, s - prev_end)
    prev_end = max(prev_end, e)
    k = short(r["Kernel_Name"])
    a = agg.setdefault(k, [0, 0])
    a[0] += 1
    a[1] += e - s
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:42s} {c:4d} {t/1e3:9.1f} us")
print(f"{'gaps':42s}      {gap/1e3:9.1f} us")
print(f"{'batch span':42s}      {(prev_end - t0)/1e3:9.1f} us")
if len(sys.argv) > 2:  # per-call durations of kernels matching argv[2] in that batch
    for r in rows[b0:b1]:
        if sys.argv[2] in r["Kernel_Name"]:
            print(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
if len(sys.argv) > 2 and sys.argv[2] == "gaps":
    prev = t0
    for r in rows[b0:b1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  +{(s - t0)/1e3:8.1f} gap {(s - prev)/1e3:7.1f}  {short(r['Kernel_Name']):40s} {(e - s)/1e3:7.1f} us")
        prev = max(prev, e)
