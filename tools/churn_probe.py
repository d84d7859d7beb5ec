#!/usr/bin/env python3
"""C4 churn probe: 1M-node fleet, n churn ticks, ingest vs tick wall time for
one ingest thread count (KWOK_INGEST_THREADS, read at engine create).
Usage: churn_probe.py THREADS [TICKS] [NODES]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.set_device(0)
from kwok_amd import engine as keng, workload  # noqa: E402

th = int(sys.argv[1])
ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 4
nodes = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
os.environ["KWOK_INGEST_THREADS"] = str(th)
e, fl, ph = workload.build_engine_fleet(keng.Engine, nodes)
n_handles = workload.BUCKETS * fl.cp
now = workload.S0 + 30
e.tick(now, read=False)
ch = workload.Churn(ph, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_handles, nodes, seed=3)
dump = lambda: e.dump_pods(0, n_handles)  # noqa: E731
ing, tck = [], []
for k in range(ticks):
    now += 30
    ev, ar = ch.batch(dump, now)
    t0 = time.perf_counter()
    hs, st, _ = e.ingest_pods_raw(ev, ar)
    t1 = time.perf_counter()
    e.tick(now, read=False)
    t2 = time.perf_counter()
    ch.applied(hs, st)
    ing.append((t1 - t0) * 1e3)
    tck.append((t2 - t1) * 1e3)
print("threads %2d: ingest ms %s | tick ms %s" % (th, " ".join("%.1f" % x for x in ing), " ".join("%.1f" % x for x in tck)),
      flush=True)
e.close()
