"""Summarise a rocprofv3 kernel trace: per-kernel medians over the last N
calls and one steady-state tick timeline."""
import csv
import statistics as st
import sys

path = sys.argv[1]
rows = [r for r in csv.DictReader(open(path)) if "kwok" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0].replace("kwok::", "") for r in rows]
by = {}
for r, n in zip(rows, names):
    by.setdefault(n, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for n, v in by.items():
    print("%-18s calls=%3d median(last40)=%7.1f us" % (n, len(v), st.median(v[-40:]) / 1e3))
firsts = [i for i, n in enumerate(names) if n == "k_classify"]
if len(firsts) > 6:
    i0, i1 = firsts[-5], firsts[-4]
    t0 = int(rows[i0]["Start_Timestamp"])
    print("tick timeline:")
    for r, n in zip(rows[i0:i1], names[i0:i1]):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("  %-16s start=%7.1f us  dur=%6.1f us  queue=%s" % (n, (s - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"]))
    print("tick period: %.1f us" % ((int(rows[i1]["Start_Timestamp"]) - t0) / 1e3))
