#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc SQ passes per kernel: the median of the last N
launches of each counter, and the ratios that say where a kernel's waves spend
their cycles (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES,
MI355X_MICROARCH.md PMC table) and how wide its stores are (write bytes per
SQ_INSTS_VMEM_WR, the bytes from a FETCH/WRITE summary of the same build).

usage: sq_summary.py OUT.txt DIR [DIR ...] [--last N] [--pmc PMC.json] [--kernel SUBSTR ...]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def load(dirs):
    per = {}  # kernel -> counter -> [(dispatch, value)]
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("kwok::", "")
                per.setdefault(name, {}).setdefault(row["Counter_Name"], []).append(
                    (int(row["Dispatch_Id"]), float(row["Counter_Value"])))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--pmc", default="", help="FETCH/WRITE summary (tools/pmc_summary.py) of the same build")
    ap.add_argument("--kernel", action="append", default=[], help="only kernels whose name holds this")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    per = load(a.dirs)
    pmc = json.load(open(a.pmc))["kernels"] if a.pmc else {}
    lines = ["# " + a.title] if a.title else []
    for k in sorted(per):
        if a.kernel and not any(s in k for s in a.kernel):
            continue
        c = {n: statistics.median(v for _, v in sorted(vs)[-a.last:]) for n, vs in per[k].items()}
        n = max(len(vs) for vs in per[k].values())
        lines.append("%s  (%d launches; medians of the last %d)" % (k, n, min(n, a.last)))
        for name in sorted(c):
            lines.append("  %-22s %16.0f" % (name, c[name]))
        waves = c.get("SQ_WAVES")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for part in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if part in c:
                    lines.append("  %-22s %15.1f%% of SQ_WAVE_CYCLES" % (part, 100.0 * c[part] / wc))
        if waves:
            for part in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if part in c:
                    lines.append("  %-22s %16.1f per wave" % (part, c[part] / waves))
        if k in pmc and c.get("SQ_INSTS_VMEM_WR"):
            wb = pmc[k]["write_size_bytes"]
            lines.append("  write bytes / VMEM_WR %16.1f (bytes per wave store instruction; 1024 = 16 B x 64 lanes)"
                         % (wb / c["SQ_INSTS_VMEM_WR"]))
        if k in pmc and c.get("SQ_INSTS_VMEM_RD"):
            rb = pmc[k]["fetch_bytes_corrected"]
            lines.append("  fetch bytes / VMEM_RD %16.1f" % (rb / c["SQ_INSTS_VMEM_RD"]))
    open(a.out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
