#!/usr/bin/env python3
"""Heartbeat-once steady tick at the metric size (1M nodes x 10M pods), for
kernel A/B work: queued steps (as bench.py's heartbeat_once leg), then blocking
ticks with HIP-event kernel times.  With KWOK_TICK_TRACE=1 in the environment
the blocking ticks also collect per-block phase stamps (printed by the engine
at destroy).  Usage: once_probe.py [steps] [label]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process, as bench.py)

from kwok_amd import engine as keng  # noqa: E402
from kwok_amd import workload  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
label = sys.argv[2] if len(sys.argv) > 2 else ""
trace = bool(os.environ.get("KWOK_TICK_TRACE"))
e, fl, _ = workload.build_engine_fleet(keng.Engine, 1_000_000, heartbeat_once=True)
now = workload.S0 + 30
e.tick(now, read=False)
for _ in range(5):
    now += 30
    e.tick(now, read=False)
q = None
if not trace:
    # warm the queued path first (the first queued submit allocates the second tick slot)
    for _ in range(3):
        e.tick_submit(now + 30)
        e.tick_submit(now + 60)
        e.tick_collect(read=False)
        e.tick_collect(read=False)
        now += 60
    e.tick_submit(now + 30)
    now += 30
    t0 = time.perf_counter()
    for k in range(steps):
        if k + 1 < steps:
            e.tick_submit(now + 30)
            now += 30
        e.tick_collect(read=False)
    q = (time.perf_counter() - t0) / steps * 1e3
e.profile_enable(True)
for _ in range(steps):
    now += 30
    e.tick(now, read=False)
ph, nt = e.profile_read()
e.profile_enable(False)
print("%s queued %s ms/step | blocking: kernel %.4f ms, classify %.4f ms (%d ticks) | %s" % (
    label, "%.4f" % q if q else "-", ph["kernel"] / nt, ph["classify"] / nt, nt, e.stats()), flush=True)
e.close()
