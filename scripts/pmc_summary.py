"""Summarise rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE, one pass each) for one kernel into
profiles/pmc_<kernel>.json, which bench.py reads for roofline.traffic.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (both in KiB as rocprofv3 derives them).  The
factor 2 is the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE tallies 128-byte memory-side read requests at 64 bytes.  Our reads are random 16..64-byte
gathers, a width the guide leaves uncalibrated; the same correction is applied and the raw values
are kept next to the corrected figure.

usage: python scripts/pmc_summary.py --kernel k_stream4 --fetch DIR1 --write DIR2 --tuples T --batch B
       [--preset P --inflight I] [--out profiles/pmc_k_stream4_p0.json]
"""
import argparse
import csv
import glob
import json
import os


def per_dispatch(d: str, kernel: str, counter: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
                    continue
                key = (f, r.get("Dispatch_Id", r.get("Correlation_Id")))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="k_stream")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--tuples", type=float, required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--preset", type=int, default=0)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--skip", type=int, default=1, help="leading (warmup) dispatches to drop")
    ap.add_argument("--anchor", default="",
                    help="a kernel chain: bytes of every dispatch matching --kernel, per dispatch of this kernel "
                         "(one per call), e.g. --kernel k_expand --anchor k_expand_lds (no dispatch skipped)")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.anchor:
        fetch = per_dispatch(a.fetch, a.kernel, "FETCH_SIZE")
        write = per_dispatch(a.write, a.kernel, "WRITE_SIZE")
        calls_f = len(per_dispatch(a.fetch, a.anchor, "FETCH_SIZE"))
        calls_w = len(per_dispatch(a.write, a.anchor, "WRITE_SIZE"))
        if not calls_f or not calls_w:
            raise SystemExit(f"no {a.anchor} dispatches under {a.fetch} / {a.write}")
        f_kib = sum(fetch) / calls_f
        w_kib = sum(write) / calls_w
    else:
        fetch = per_dispatch(a.fetch, a.kernel, "FETCH_SIZE")[a.skip:]
        write = per_dispatch(a.write, a.kernel, "WRITE_SIZE")[a.skip:]
        if not fetch or not write:
            raise SystemExit(f"no {a.kernel} dispatches with FETCH_SIZE/WRITE_SIZE under {a.fetch} / {a.write}")
        f_kib = sum(fetch) / len(fetch)
        w_kib = sum(write) / len(write)
    out = {
        "kernel": a.kernel, "tuples": int(a.tuples), "batch": a.batch, "preset": a.preset,
        "inflight": a.inflight,
        "dispatches": {"fetch": len(fetch), "write": len(write)}, "anchor": a.anchor or None,
        "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
        "hbm_bytes_per_launch": (2 * f_kib + w_kib) * 1024.0,
        "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section, gfx950)",
    }
    path = a.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                 f"pmc_{a.kernel}_p{a.preset}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
