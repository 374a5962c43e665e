"""Per-kernel mean of every counter in rocprofv3 --pmc output dirs (skips the first dispatch of
each kernel = warmup).  usage: python scripts/pmc_table.py DIR [DIR ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("kg::", "").replace("void ", "")
            disp = (f, r.get("Dispatch_Id"))
            c = vals[k][r["Counter_Name"]]
            c[disp] = c.get(disp, 0.0) + float(r["Counter_Value"])
for k, cs in vals.items():
    print(k)
    for c, dv in sorted(cs.items()):
        v = list(dv.values())
        v = v[1:] if len(v) > 2 else v
        print(f"   {c:24s} {sum(v) / len(v):16.1f}   (n={len(v)})")
