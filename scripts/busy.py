"""Per-kernel device time and concurrency over a window of a rocprofv3 kernel trace (overlapping streams):
python scripts/busy.py run_kernel_trace.csv [name-regex-of-window-kernels] [--last-seconds S]

For each kernel name: launches, summed duration, mean duration; then the window's wall span, the time
at least one kernel ran and the mean number of kernels running (summed durations / busy time)."""
import csv
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
last = 0.0
if "--last-seconds" in sys.argv:
    last = float(sys.argv[sys.argv.index("--last-seconds") + 1])
    args = [a for a in args if a != sys.argv[sys.argv.index("--last-seconds") + 1]]
rows = list(csv.DictReader(open(args[0])))
pat = re.compile(args[1]) if len(args) > 1 else None
short = lambda n: re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "")).replace("kg::", "").replace("void ", "")[:44]
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
ev.sort()
if pat:
    ev = [e for e in ev if pat.search(e[2])]
if last and ev:
    t_end = max(e[1] for e in ev)
    ev = [e for e in ev if e[0] >= t_end - last * 1e9]
agg = {}
for s, e, k in ev:
    a = agg.setdefault(k, [0, 0])
    a[0] += 1
    a[1] += e - s
tot = sum(a[1] for a in agg.values())
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:46s} {c:6d} {t / 1e6:10.2f} ms  mean {t / c / 1e3:9.1f} us  {100 * t / max(tot, 1):5.1f} %")
busy, cur_end = 0, None
t0 = ev[0][0] if ev else 0
for s, e, _ in ev:
    if cur_end is None or s > cur_end:
        if cur_end is not None:
            busy += cur_end - seg_start
        seg_start, cur_end = s, e
    else:
        cur_end = max(cur_end, e)
if cur_end is not None:
    busy += cur_end - seg_start
span = (max(e[1] for e in ev) - t0) if ev else 0
print(f"span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, mean concurrency {tot / max(busy, 1):.2f}")
