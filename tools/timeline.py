"""The last dispatches of a rocprofv3 kernel trace as a timeline: start offset
from the first of them, duration, gap to the previous end (microseconds).

usage: timeline.py run_kernel_trace.csv [--last N] [--copies run_memory_copy_trace.csv]
(--copies: the copies that start inside the window, merged in as "copy <direction> <bytes>")"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--copies")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))[-a.last:]
    t0 = int(rows[0]["Start_Timestamp"])
    if a.copies:
        for r in csv.DictReader(open(a.copies)):
            if int(r["Start_Timestamp"]) >= t0:
                size = r.get("Bytes") or r.get("Size") or r.get("Copy_Bytes") or "?"
                r["Kernel_Name"] = "copy %s %s" % (r.get("Direction", r.get("Kind", "")), size)
                rows.append(r)
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev = t0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("kwok::", "")[:40]
        print("%10.1f %9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, n))
        prev = e


if __name__ == "__main__":
    main()
