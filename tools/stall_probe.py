#!/usr/bin/env python3
"""C4 stall probe: the bench's packed churn steps (page-locked batches) on the
1M x 10M fleet; per step the ingest / tick wall times beside the cgroup's CPU
throttling (cpu.stat throttled_usec) and this process's involuntary context
switches, to tell a host-side stall (CPU quota) from a device-side one.
Usage: stall_probe.py [STEPS]"""
import os
import resource
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.set_device(0)
from kwok_amd import engine as keng, workload  # noqa: E402


def throttled():
    for p in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            d = dict(line.split() for line in open(p))
            return int(d.get("throttled_usec", int(d.get("throttled_time", 0)) // 1000)), int(d.get("nr_throttled", 0))
        except OSError:
            continue
    return -1, -1


steps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
    try:
        print(p, open(p).read().strip(), flush=True)
    except OSError:
        pass
e, fl, ph = workload.build_engine_fleet(keng.Engine, 1_000_000)
n_handles = workload.BUCKETS * fl.cp
now = workload.S0 + 30
e.tick(now, read=False)
n = 1_000_000
ch = workload.Churn(ph, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_handles, n, seed=7, alloc=keng.host_array)
ch.packed, ch.bufs = True, None
outs = (keng.host_array((2 * n,), np.int32), keng.host_array((2 * n,), np.int8), None)
dump = lambda: e.dump_pods(0, n_handles)  # noqa: E731
for k in range(steps):
    now += 30
    ev, _ = ch.batch(dump, now)
    torch.cuda.synchronize()
    th0, nt0 = throttled()
    r0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    hs, st, _ = e.ingest_pods_packed(ev, out=outs)
    t1 = time.perf_counter()
    e.tick(now, read=False)
    t2 = time.perf_counter()
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    th1, nt1 = throttled()
    ch.applied(hs.copy(), st)
    print("step %2d: ingest %6.3f ms tick %6.3f ms | throttled %+8d us (%+d periods) | nivcsw %+d nvcsw %+d" %
          (k, (t1 - t0) * 1e3, (t2 - t1) * 1e3, th1 - th0, nt1 - nt0, r1.ru_nivcsw - r0.ru_nivcsw,
           r1.ru_nvcsw - r0.ru_nvcsw), flush=True)
e.close()
