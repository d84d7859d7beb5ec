"""k_pod_jobs per-wave timeline from KWOK_JOBS_TRACE (diagnostics).

usage: jobs_trace.py FILE [bytes_per_job]
Each wave slot: entry / emission start / exit (s_memrealtime, 10 ns) and
HW_ID[15:0] | XCC_ID << 28 | jobs << 32.  Prints the kernel span, the phase
length distributions, and per 20 us bin: waves resident, waves emitting, and
the store rate if each wave's jobs were written evenly over its emission.
"""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], np.uint64).reshape(-1, 4)
bpj = float(sys.argv[2]) if len(sys.argv) > 2 else 575.0
ent = a[:, 0] != 0
t0 = a[ent, 0].min()
us = lambda x: (x.astype(np.int64) - int(t0)) * 0.01
work = ent & (a[:, 1] != 0) & (a[:, 2] != 0)
e0, e1, e2 = us(a[work, 0]), us(a[work, 1]), us(a[work, 2])
jobs = (a[work, 3] >> np.uint64(32)).astype(np.float64)
hw = (a[work, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
xcc = (hw >> 28) & 15
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
print(f"waves entered {ent.sum()}, emitting {work.sum()}, jobs {jobs.sum():.0f}")
idle = ent & (a[:, 2] == 0)
print(f"early-exit waves {idle.sum()}; span first entry -> last exit {e2.max():.1f} us; last entry {us(a[ent, 0]).max():.1f} us")
pct = lambda v: " ".join(f"{np.percentile(v, q):7.1f}" for q in (0, 10, 50, 90, 100))
print("percentiles 0/10/50/90/100 (us)")
print("  entry        ", pct(e0))
print("  classify     ", pct(e1 - e0))
print("  emit         ", pct(e2 - e1))
print("  jobs         ", pct(jobs))
print("  emit GB/s/wave", pct(jobs * bpj / np.maximum(e2 - e1, 1e-3) / 1e3))
for x in sorted(set(xcc.tolist())):
    m = xcc == x
    print(f"  xcc {x}: waves {m.sum():5d} last exit {e2[m].max():7.1f} us, mean emit {np.mean(e2[m] - e1[m]):6.1f} us")
B = 20.0
nb = int(e2.max() // B) + 1
print(f"{'bin_us':>7} {'resident':>8} {'emitting':>8} {'TB/s':>6}")
for b in range(nb):
    lo, hi = b * B, (b + 1) * B
    res = np.sum((e0 < hi) & (e2 > lo))
    emi = np.sum((e1 < hi) & (e2 > lo))
    ov = np.clip(np.minimum(e2, hi) - np.maximum(e1, lo), 0, None)
    rate = np.sum(jobs * bpj * ov / np.maximum(e2 - e1, 1e-3)) / (B * 1e-6) / 1e12
    print(f"{lo:7.0f} {res:8d} {emi:8d} {rate:6.2f}")
