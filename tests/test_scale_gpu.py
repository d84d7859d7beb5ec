"""GPU parity at scale: the HIP engine vs the CPU oracle on the same seeded
event traces, compared tick by tick on every output (handles, patch bytes,
deletes, counters) and on the full pod state, plus size-independent
properties of the C2 workload (BASELINE configs[1]: 100k nodes x 1M pods).
The oracle finishes C2 in seconds, so C2 is compared exhaustively."""
import ipaddress

import numpy as np
import pytest

from gpu_common import Driver, compare, compare_state, external_deletes, mark_deleting, new_pods
from kwok_amd import abi, workload
from kwok_amd.engine import Engine, make_config
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def test_c2_full_parity_and_properties():
    """C2 at full size: initial tick (100k node inits, 1M Pending->Running with
    IPs) and steady ticks, byte-exact against the oracle; IPs are exactly the
    first 1M addresses of 10.0.0.1/8 in canonical (bucket, slot) order.  Ticks
    0 and 1 are queued back to back (kwok_tick_submit x2, then collect), tick 2
    is a plain kwok_tick."""
    e, fl, ph = workload.build_engine_fleet(Engine, 100_000)
    o, _, ph2 = workload.build_engine_fleet(Oracle, 100_000)
    assert (ph == ph2).all()
    n_slots = workload.BUCKETS * fl.cp
    e.tick_submit(workload.S0 + 30)
    e.tick_submit(workload.S0 + 60)
    for t in range(3):
        now = workload.S0 + 30 * (t + 1)
        eo = e.tick_collect() if t < 2 else e.tick(now)
        oo = o.tick(now)
        compare(eo, oo, "c2 tick %d" % t)
        if t == 0:
            assert eo.counters["pod_patch"] == 1_000_000 and eo.counters["node_init"] == 100_000
            # size-independent properties of the allocation
            used, phase, hip, pip = e.dump_pods(0, n_slots)
            ips = pip[used.astype(bool)]
            base = int(ipaddress.IPv4Address("10.0.0.1"))
            assert len(np.unique(ips)) == 1_000_000
            order = np.argsort(np.nonzero(used)[0])
            assert (np.sort(ips) == base + np.arange(1_000_000, dtype=np.uint32)).all()
            assert (ips[order] == base + np.arange(1_000_000, dtype=np.uint32)).all()  # canonical order
        else:
            assert eo.counters["pod_patch"] == 0 and eo.counters["heartbeat"] == 100_000
    compare_state(e, o, n_slots, "c2")
    e.close()
    o.close()


@pytest.mark.parametrize("seed,cidr", [(1, "10.0.0.1/16"), (2, "10.0.0.1/20"), (3, "172.16.3.9/22")])
def test_churn_parity(seed, cidr):
    """C4-style churn at reduced size: creates, deletionTimestamp deletes with
    and without finalizers, external Deleted events (ingest-time release),
    pre-existing / duplicate IPs (Use), CIDR exhaustion (out-of-CIDR fresh IPs
    for the /22 case), node flaps."""
    kw = dict(cidr=cidr, node_ip="196.168.0.1", buckets=256, node_slots_per_bucket=16, pod_slots_per_bucket=256)
    d = Driver(kw, seed)
    rng = d.rng
    names = ["node-%07d" % i for i in range(1000)]
    nh, st = d.nodes(names, managed=(rng.random(1000) < 0.9).astype(np.uint8),
                     lockable=(rng.random(1000) < 0.95).astype(np.uint8))
    assert (st == 0).all()
    net = ipaddress.IPv4Network(cidr, strict=False)
    ip_range = (int(net.network_address), int(net.network_address) + min(net.num_addresses, 4096))
    ev, ar = new_pods(rng, nh, 20_000, d.spec, 0.02, ip_range)
    d.pods(ev, ar)
    d.tick("churn seed %d tick 0" % seed)
    for t in range(1, 7):
        idx, _, _, _ = d.live()
        dels = rng.choice(idx, min(len(idx), 3000), replace=False)
        ev, ar = mark_deleting(rng, d, np.sort(dels[:2000]).astype(np.int32))
        d.pods(ev, ar)
        ev, ar = external_deletes(d, np.sort(dels[2000:]).astype(np.int32))
        d.pods(ev, ar)
        if t % 2 == 0:  # flap 2% of the nodes
            fl = list(rng.choice(names, 20, replace=False))
            d.nodes(fl, managed=1, lockable=1, op=abi.OP_DELETE)
            d.nodes(fl, managed=1, lockable=1)
        ev, ar = new_pods(rng, nh, 3000, d.spec, 0.02, ip_range)
        d.pods(ev, ar)
        if t == 6:  # deletes, releases and Gets in the first of two queued ticks
            d.tick_pair("churn seed %d tick %d" % (seed, t))
        else:
            d.tick("churn seed %d tick %d" % (seed, t))
    d.e.close()
    d.o.close()


def test_partial_management_flap_parity():
    """C5-style: ManageAllNodes=false with a selector on 50% of the nodes, a
    disregard annotation on 0.1%, and 1% of the managed nodes deleted and
    re-created per tick."""
    cn, cp = workload.slots_for(20_000, 1024, 12)
    kw = dict(cidr="10.0.0.1/12", node_ip="10.1.2.3", buckets=1024, node_slots_per_bucket=cn,
              pod_slots_per_bucket=cp)
    d = Driver(kw, 7)
    rng = d.rng
    names = ["node-%07d" % i for i in range(20_000)]
    managed = (rng.random(len(names)) < 0.5).astype(np.uint8)
    lockable = (rng.random(len(names)) >= 0.001).astype(np.uint8)
    nh, st = d.nodes(names, managed, lockable)
    assert (st == 0).all()
    ev, ar = new_pods(rng, nh, 100_000, d.spec)
    d.pods(ev, ar)
    d.tick("c5 tick 0")
    mnames = [n for n, m in zip(names, managed) if m]
    for t in range(1, 4):
        fl = list(rng.choice(mnames, len(mnames) // 100, replace=False))
        d.nodes(fl, managed=1, lockable=1, op=abi.OP_DELETE)
        d.nodes(fl, managed=1, lockable=1)
        d.tick("c5 tick %d" % t)
    assert d.e.node_size() == d.o.node_size()
    d.e.close()
    d.o.close()


def test_domain_table_engine():
    """The engine accepts / rejects exactly the domain table the oracle does
    (tests/domain_cases.py, tests/test_domain.py): yaml.v2-typed strings, IPv4
    dotted quads as Go 1.19 parses them."""
    from test_domain import KW, check_backend
    check_backend(lambda: Engine(make_config(**KW)))


def test_domain_rejections():
    """Configurations outside the supported domain are rejected, never
    emulated: IPv6 / non-canonical CIDRs, prefixes shorter than /4, custom
    templates.  EnableCNI is accepted (kwok_cni_pending / kwok_cni_assign)."""
    for kw in (dict(cidr="fe80::1/64"), dict(cidr="10.0.0.1/3"), dict(cidr="010.0.0.1/8")):
        with pytest.raises(Exception):
            Engine(make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8, **kw))
    cfg = make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8)
    cfg.custom_templates = 1
    with pytest.raises(Exception):
        Engine(cfg)
    Engine(make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8, enable_cni=True)).close()
