"""GPU parity at scale: the HIP engine vs the CPU oracle on the same seeded
event traces, compared tick by tick on every output (handles, patch bytes,
deletes, counters) and on the full pod state, plus size-independent
properties of the C2 workload (BASELINE configs[1]: 100k nodes x 1M pods).
The oracle finishes C2 in seconds, so C2 is compared exhaustively."""
import ipaddress

import numpy as np
import pytest

from kwok_amd import abi, workload
from kwok_amd.engine import Engine, make_config
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def compare(e_out, o_out, where):
    assert list(e_out.heartbeat_nodes) == list(o_out.heartbeat_nodes), where + " heartbeat handles"
    n = len(e_out.heartbeat_nodes)
    if n:
        hb = o_out.heartbeat_body(0)
        a = np.frombuffer(e_out.arena, np.uint8)[e_out.heartbeat_off:e_out.heartbeat_off + n * e_out.heartbeat_stride]
        a = a.reshape(n, e_out.heartbeat_stride)[:, :e_out.heartbeat_len]
        assert (a == np.frombuffer(hb, np.uint8)[None, :]).all(), where + " heartbeat bytes"
        ob = np.frombuffer(o_out.arena, np.uint8)[o_out.heartbeat_off:o_out.heartbeat_off + n * len(hb)]
        assert (ob.reshape(n, len(hb)) == np.frombuffer(hb, np.uint8)[None, :]).all()
    assert [h for h, _ in e_out.node_inits] == [h for h, _ in o_out.node_inits], where + " node-init handles"
    assert [b for _, b in e_out.node_inits] == [b for _, b in o_out.node_inits], where + " node-init bytes"
    assert [h for h, _ in e_out.pod_patches] == [h for h, _ in o_out.pod_patches], where + " pod-patch handles"
    bad = [h for (h, b), (_, c) in zip(e_out.pod_patches, o_out.pod_patches) if b != c]
    assert not bad, where + " pod-patch bytes differ for %d pods, first %d" % (len(bad), bad[0])
    assert e_out.deletes == o_out.deletes, where + " deletes"
    assert e_out.counters == o_out.counters, where + " counters"


def compare_state(e, o, n_slots, where):
    eu, ep, eh, ei = e.dump_pods(0, n_slots)
    ou, op, oh, oi = o.dump_pods(0, n_slots)
    assert (eu == ou).all(), where + " pod slots"
    assert (ep == op).all(), where + " phases"
    assert (eh == oh).all(), where + " hostIPs"
    assert (ei == oi).all(), where + " podIPs"


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


class Driver:
    """Applies the same random event batches to engine and oracle."""

    def __init__(self, cfg_kw, seed):
        self.e = Engine(make_config(**cfg_kw))
        self.o = Oracle(make_config(**cfg_kw))
        self.rng = np.random.default_rng(seed)
        self.cfg = cfg_kw
        self.spec = [self.e.register_pod_spec([("fake-pod", "fake")]),
                     self.e.register_pod_spec([("a", "img-a"), ("b", "img/b:v2")], [("init", "busybox")], ["g.io/x"])]
        assert self.spec == [self.o.register_pod_spec([("fake-pod", "fake")]),
                             self.o.register_pod_spec([("a", "img-a"), ("b", "img/b:v2")], [("init", "busybox")],
                                                      ["g.io/x"])]
        self.n_slots = cfg_kw["buckets"] * cfg_kw["pod_slots_per_bucket"]
        self.spec_of = np.zeros(self.n_slots, np.int32)   # immutable pod fields, by handle
        self.ctime_of = np.zeros(self.n_slots, np.int64)
        self.now = 1704067230

    def nodes(self, names, managed, lockable, op=abi.OP_UPSERT, phase=abi.PHASE_NONE):
        ar = abi.Arena()
        ev = np.zeros(len(names), abi.NODE_EVENT_DTYPE)
        ev["op"] = op
        ev["managed"] = managed
        ev["lockable"] = lockable
        ev["phase"] = phase
        for i, n in enumerate(names):
            ev[i]["name"] = ar.ref(n)
        a = bytes(ar.buf)
        h1, s1 = self.e.ingest_nodes_raw(ev, a)
        h2, s2 = self.o.ingest_nodes_raw(ev, a)
        assert (h1 == h2).all() and (s1 == s2).all()
        return h1, s1

    def pods(self, ev, arena=b""):
        h1, s1, r1 = self.e.ingest_pods_raw(ev, arena)
        h2, s2, r2 = self.o.ingest_pods_raw(ev, arena)
        assert (h1 == h2).all() and (s1 == s2).all() and (r1 == r2).all()
        new = (ev["op"] == abi.OP_UPSERT) & (ev["handle"] < 0) & (s1 == 0)
        self.spec_of[h1[new]] = ev["spec_id"][new]
        self.ctime_of[h1[new]] = ev["creation_unix"][new]
        return h1, s1, r1

    def tick(self, where):
        eo, oo = self.e.tick(self.now), self.o.tick(self.now)
        self.now += 30
        compare(eo, oo, where)
        compare_state(self.e, self.o, self.n_slots, where)
        return eo

    def tick_pair(self, where):
        """two ticks queued back to back on the engine, one after the other on the oracle"""
        self.e.tick_submit(self.now)
        self.e.tick_submit(self.now + 30)
        for k in range(2):
            eo, oo = self.e.tick_collect(), self.o.tick(self.now)
            self.now += 30
            compare(eo, oo, "%s (queued %d)" % (where, k))
        compare_state(self.e, self.o, self.n_slots, where)

    def live(self):
        used, phase, hip, pip = self.o.dump_pods(0, self.n_slots)
        idx = np.nonzero(used)[0]
        return idx, phase[idx], hip[idx], pip[idx]


def new_pods(rng, node_handles, n, spec_ids, with_ip_frac=0.0, ip_range=None):
    ev = np.zeros(n, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = -1
    ev["node_handle"] = rng.choice(node_handles, n)
    ev["spec_id"] = rng.choice(spec_ids, n)
    ev["creation_unix"] = 1704067200 - rng.integers(0, 10 ** 6, n)
    ph = rng.choice([abi.PHASE_PENDING, abi.PHASE_PENDING, abi.PHASE_NONE], n)
    ev["phase"] = ph
    fl = np.where(ph == abi.PHASE_PENDING, abi.POD_STATUS_NONEMPTY, 0)
    fl |= np.where(rng.random(n) < 0.3, abi.POD_HAS_FINALIZERS, 0)
    fl |= np.where(rng.random(n) < 0.03, abi.POD_DISREGARD, 0)
    ev["flags"] = fl
    arena = b""
    if with_ip_frac and ip_range:
        ar = abi.Arena()
        lo, hi = ip_range
        for i in np.nonzero(rng.random(n) < with_ip_frac)[0]:
            ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(rng.integers(lo, hi))))
            ev[i]["flags"] |= abi.POD_STATUS_NONEMPTY
        arena = bytes(ar.buf)
    return ev, arena


def mark_deleting(rng, d, handles):
    """Modified events with a deletionTimestamp for existing pods (state kept)."""
    idx, phase, hip, pip = d.live()
    pos = np.searchsorted(idx, handles)
    ar = abi.Arena()
    ev = np.zeros(len(handles), abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = handles
    ev["node_handle"] = -1
    ev["spec_id"] = d.spec_of[handles]
    ev["phase"] = phase[pos]
    ev["creation_unix"] = d.ctime_of[handles]
    fl = abi.POD_DELETING | np.where(rng.random(len(handles)) < 0.5, abi.POD_HAS_FINALIZERS, 0)
    fl |= np.where(phase[pos] == abi.PHASE_RUNNING, abi.POD_CONFORMS | abi.POD_STATUS_NONEMPTY, 0)
    ev["flags"] = fl
    for i in range(len(handles)):
        if hip[pos[i]]:
            ev[i]["host_ip"] = ar.ref(abi.ip4s(int(hip[pos[i]])))
        if pip[pos[i]]:
            ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(pip[pos[i]])))
    return ev, bytes(ar.buf)


def external_deletes(d, handles):
    idx, phase, hip, pip = d.live()
    pos = np.searchsorted(idx, handles)
    ar = abi.Arena()
    ev = np.zeros(len(handles), abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_DELETE
    ev["handle"] = handles
    for i in range(len(handles)):
        if pip[pos[i]]:
            ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(pip[pos[i]])))
    return ev, bytes(ar.buf)


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


def test_domain_rejections():
    """Values outside the supported domain are rejected, never emulated:
    YAML-typed strings (yaml.v2 would turn `y` / `1.5` / `null` into bool /
    float / null), IPv6 / non-canonical IPs, custom templates, EnableCNI."""
    e = Engine(make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8))
    for bad in ("y", "on", "null", "1.5", "0x1F", "-x", "a b", ""):
        with pytest.raises(Exception):
            e.register_pod_spec([("c", bad)])
    e.register_pod_spec([("c", "nginx:1.25")])
    ar = abi.Arena()
    ev = np.zeros(2, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = -1
    ev["node_handle"] = -1
    ev[0]["node_name"] = ar.ref("n")
    ev[1]["node_name"] = ar.ref("n")
    ev[0]["pod_ip"] = ar.ref("010.0.0.1")
    ev[1]["pod_ip"] = ar.ref("fe80::1")
    _, st, _ = e.ingest_pods_raw(ev, bytes(ar.buf))
    assert list(st) == [abi.EDOMAIN, abi.EDOMAIN]
    e.close()
    for kw in (dict(cidr="fe80::1/64"), dict(cidr="10.0.0.1/4")):
        with pytest.raises(Exception):
            Engine(make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8, **kw))
    cfg = make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8)
    cfg.custom_templates = 1
    with pytest.raises(Exception):
        Engine(cfg)
