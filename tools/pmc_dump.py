#!/usr/bin/env python3
"""Per-kernel values of every counter in a rocprofv3 --pmc output directory:
the first dispatch and the median over dispatches of each kernel.

usage: pmc_dump.py DIR [--kernel SUBSTR]
"""
import argparse
import csv
import glob
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    per = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("kwok::", "")
            if a.kernel not in k:
                continue
            per.setdefault((k, r["Counter_Name"]), {}).setdefault(int(r["Dispatch_Id"]), 0.0)
            per[(k, r["Counter_Name"])][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, c), d in sorted(per.items()):
        v = [d[i] for i in sorted(d)]
        print("%-14s %-28s n=%-4d first=%-16.4g median=%-16.4g" % (k, c, len(v), v[0], statistics.median(v)))


if __name__ == "__main__":
    main()
