"""Calibrate rocprofv3's FETCH_SIZE for random gathers (MI355X_MICROARCH.md: "other access widths are
uncalibrated: calibrate on a known byte count in your own access pattern").  Reads the counter
passes of tools/randprobe's k_gather dispatches (a known number of independent random 16-B or 64-B
loads over a table far larger than the 256 MiB Infinity Cache) and prints the counter value per load.

usage: python scripts/pmc_calib.py --dir DIR --counter FETCH_SIZE --cus 256 --waves 8 --bytes 16
"""
import argparse
import csv
import glob
import json
import os


def dispatches(d: str, counter: str):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_gather" not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
                    continue
                key = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                name, v = r["Kernel_Name"], float(r["Counter_Value"])
                rows[key] = (name, rows.get(key, (name, 0.0))[1] + v)
    return [rows[k] for k in sorted(rows)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--counter", default="FETCH_SIZE")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--waves", type=int, default=8)
    ap.add_argument("--bytes", type=int, default=16)
    a = ap.parse_args()
    blocks = a.cus * max(1, a.waves // 4)
    ks = [1, 4] if a.bytes == 64 else [1, 4, 8]
    out = []
    ds = dispatches(a.dir, a.counter)
    # randprobe runs each variant twice: a 4-round warm-up, then 64 rounds
    for j, (name, v) in enumerate(ds):
        k = ks[min(j // 2, len(ks) - 1)]
        rounds = 4 if j % 2 == 0 else 64
        loads = blocks * 256 * rounds * k
        per = v * (1024.0 if a.counter.endswith("_SIZE") else 1.0) / loads
        out.append({"kernel": name[:40], "loads": loads, a.counter: v, "per_load": per})
    print(json.dumps({"counter": a.counter, "bytes_per_load_requested": a.bytes,
                      "unit": "bytes per load (FETCH_SIZE KiB x 1024)" if a.counter.endswith("_SIZE") else "counts per load",
                      "dispatches": out}))


if __name__ == "__main__":
    main()
