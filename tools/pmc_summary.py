#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM
bytes per kernel (median of the last N launches of each kernel).

FETCH_SIZE and WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts half
the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), so it is doubled.

usage: pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [--last N] [--source TEXT]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            name = name.replace("kwok::", "")
            per.setdefault(name, []).append((int(row["Dispatch_Id"]), float(row["Counter_Value"]) * 1024.0))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--source", default="")
    ap.add_argument("--kernels", default="", help="kernel source whose sha256 ties the figures to a build")
    a = ap.parse_args()
    fe, wr = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    ks = {}
    for k in sorted(set(fe) & set(wr)):
        f = statistics.median(v for _, v in sorted(fe[k])[-a.last:])
        w = statistics.median(v for _, v in sorted(wr[k])[-a.last:])
        ks[k] = {"fetch_size_bytes": f, "write_size_bytes": w, "fetch_bytes_corrected": 2 * f,
                 "hbm_bytes": 2 * f + w, "launches": len(fe[k])}
    import hashlib
    out = {"source": a.source,
           "kernels_sha256": hashlib.sha256(open(a.kernels, "rb").read()).hexdigest() if a.kernels else None,
           "units": "bytes per launch (median of the last %d launches); counters reported in KiB, x1024" % a.last,
           "note": "FETCH_SIZE on gfx950 under-reports wide coalesced reads by 2x (MI355X_MICROARCH.md HBM); "
                   "reported raw and doubled in fetch_bytes_corrected; hbm_bytes = corrected fetch + write",
           "kernels": ks}
    json.dump(out, open(a.out, "w"), indent=1)
    for k, v in ks.items():
        print("%-28s fetch %12.0f  write %12.0f  hbm %12.0f" % (k, v["fetch_bytes_corrected"], v["write_size_bytes"], v["hbm_bytes"]))


if __name__ == "__main__":
    main()
