"""Times the dirty ticks of C2: the initial tick (100k node inits, 1M
Pending->Running with IPs) and churn ticks (delete + re-create a fraction of
the pods), with the kernel's phase split.  Diagnostics only."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: F401,E402  (one HIP runtime per process, as in bench.py)

from kwok_amd import abi, workload  # noqa: E402
from kwok_amd.engine import Engine, load_engine_lib  # noqa: E402

load_engine_lib()
nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
e, fl, ph = workload.build_engine_fleet(Engine, nodes)
e.profile_enable(True)
now = workload.S0 + 30


def tick(label):
    global now
    e.profile_host(reset=True)
    t0 = time.perf_counter()
    r = e.tick(now, read=False)
    dt = time.perf_counter() - t0
    hm, _ = e.profile_host(reset=True)
    now += 30
    phases, n = e.profile_read()
    e.profile_enable(True)
    c = dict(zip(abi.COUNTERS, r.counters))
    print("%-10s wall %8.3f ms  kernel %8.3f ms  pp %8d del %8d init %7d alloc %8d rel %8d" % (
        label, dt * 1e3, phases["kernel"], c["pod_patch"], c["delete"], c["node_init"], c["alloc"], c["release"]),
        {k: round(v, 3) for k, v in phases.items() if v}, "host", {k: round(v, 3) for k, v in hm.items()})


tick("initial")
if len(sys.argv) > 3 and sys.argv[3] == "initial":
    e.close()
    sys.exit(0)
tick("steady")
rng = np.random.default_rng(1)
for k in range(3):
    # churn: mark a fraction of the live pods deleting (half with a finalizer), create as many new ones
    sel = rng.choice(len(ph), int(len(ph) * frac), replace=False)
    ev = np.zeros(len(sel), abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = ph[sel]
    ev["phase"] = abi.PHASE_RUNNING
    ev["flags"] = abi.POD_DELETING | abi.POD_CONFORMS | abi.POD_STATUS_NONEMPTY | np.where(
        rng.random(len(sel)) < 0.5, abi.POD_HAS_FINALIZERS, 0).astype(ev["flags"].dtype)
    ev["spec_id"] = 0
    ev["creation_unix"] = workload.S0 - 60
    t0 = time.perf_counter()
    hs, st, _ = e.ingest_pods_raw(ev, b"")
    print("ingest of %d deleting pods: %.3f ms" % (len(ev), (time.perf_counter() - t0) * 1e3))
    tick("churn-del")
    ph = np.delete(ph, sel)
