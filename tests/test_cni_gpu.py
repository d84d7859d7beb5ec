"""GPU parity of EnableCNI mode (pod_controller.go:377-389 configurePod's
cni.Setup, :337-342 cni.Remove): the HIP engine and the CPU oracle driven with
the same churn trace (creates with and without status, deletionTimestamp
deletes, external Deleted events, node flaps), the same pending lists from
kwok_cni_pending and the same IPs from a fake host-local IPAM through
kwok_cni_assign; one tick per round leaves some pods without an IP (a failed
cni.Setup).  Compared on every output and on the full pod state."""
import ipaddress

import numpy as np
import pytest

from gpu_common import Driver, external_deletes, mark_deleting, new_pods
from kwok_amd import abi

pytestmark = pytest.mark.gpu

CNI_BASE = int(ipaddress.IPv4Address("172.20.0.2"))


def test_cni_engine_matches_oracle():
    kw = dict(cidr="10.0.0.1/16", node_ip="196.168.0.1", buckets=256, node_slots_per_bucket=16,
              pod_slots_per_bucket=256, enable_cni=True)
    d = Driver(kw, 21)
    rng = d.rng
    names = ["node-%07d" % i for i in range(1000)]
    nh, st = d.nodes(names, managed=(rng.random(1000) < 0.9).astype(np.uint8),
                     lockable=(rng.random(1000) < 0.95).astype(np.uint8))
    assert (st == 0).all()
    next_ip = CNI_BASE
    for t in range(6):
        if t:
            idx, _, _, _ = d.live()
            dels = rng.choice(idx, min(len(idx), 1500), replace=False)
            ev, ar = mark_deleting(rng, d, np.sort(dels[:1000]).astype(np.int32))
            d.pods(ev, ar)
            ev, ar = external_deletes(d, np.sort(dels[1000:]).astype(np.int32))
            _, _, rel = d.pods(ev, ar)
            assert (rel == 0).all()  # cni.Remove, not ipPool.Put
            if t % 2 == 0:
                fl = list(rng.choice(names, 20, replace=False))
                d.nodes(fl, managed=1, lockable=1, op=abi.OP_DELETE)
                d.nodes(fl, managed=1, lockable=1)
        ev, ar = new_pods(rng, nh, 20_000 if t == 0 else 2000, d.spec)
        d.pods(ev, ar)
        pe, po = d.e.cni_pending(), d.o.cni_pending()
        assert (pe == po).all(), "tick %d: pending lists differ" % t
        take = pe if t != 3 else pe[: len(pe) // 2]  # tick 3: half the cni.Setup calls fail
        ips = np.arange(next_ip, next_ip + len(take), dtype=np.uint32)
        next_ip += len(take)
        assert (d.e.cni_assign(take, ips) == d.o.cni_assign(take, ips)).all()
        out = d.tick("cni tick %d" % t)
        assert out.counters["alloc"] == 0 and out.counters["release"] == 0
    d.e.close()
    d.o.close()
