"""Summarise a rocprofv3 kernel trace (run_kernel_trace.csv) of a bench.py run:
per-kernel count / mean / max duration over ALL dispatches, and mean / median /
min / max over the steady-state dispatches (the last N of each kernel: the
timed bench steps, after the warmup ticks and the initial bulk tick).

usage: trace_summary.py run_kernel_trace.csv [--last N] [--out FILE]
"""
import argparse
import csv
import statistics as st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if "kwok" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in rows:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("kwok::", "")
        n = n.replace("rocprim::ROCPRIM_400200_NS::detail::", "rocprim::")[:48]
        by.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = ["source: %s" % a.trace,
             "durations in us; 'steady' = the last %d dispatches of each kernel (timed bench steps)" % a.last,
             "%-18s %6s %10s %10s | %6s %10s %10s %10s %10s" % ("kernel", "calls", "mean", "max", "steady", "mean",
                                                                "median", "min", "max")]
    for n, v in by.items():
        s = v[-a.last:]
        lines.append("%-18s %6d %10.1f %10.1f | %6d %10.2f %10.2f %10.2f %10.2f" % (
            n, len(v), st.mean(v), max(v), len(s), st.mean(s), st.median(s), min(s), max(s)))
    text = "\n".join(lines)
    print(text)
    if a.out:
        open(a.out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
