#!/usr/bin/env python3
"""C4 on a full engine, then (engine closed) C4 on a heartbeat-once engine in the same
process, as bench.py runs its legs: does the second engine's ingest lose time?
(KWOK_INGEST_PROF=1 shows whether the create handles took the mapped path.)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kwok_amd import engine as keng, workload  # noqa: E402

for once in (False, True, False, True):
    e, fl, pods = workload.build_engine_fleet(keng.Engine, 1_000_000, heartbeat_once=once)
    now = workload.S0 + 30
    e.tick(now, read=False)
    now += 30
    _, _, c = bench.churn_leg(e, fl, pods, now, 4, 1_000_000)
    e.close()
    print("once" if once else "full", json.dumps({k: c[k] for k in ("ms_per_step", "ingest_ms", "tick_ms")}), flush=True)
