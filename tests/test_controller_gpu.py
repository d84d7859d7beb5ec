"""GPU parity of the drop-in's call sequence (integration/go/.../gpu_controller.go,
restated in kwok_amd/controller.py): the controller over the HIP engine
against the same controller over the CPU oracle, each on its own fake
clientset driven with the same cluster events, compared call by call (verb,
object, body); the reference's unit tests through the drop-in on the engine;
and, at the metric's size, the shim's ingest sequence on a heartbeat-once
engine (KWOK_CFG_HEARTBEAT_ONCE, as engine_cgo.go creates it) against the
oracle: flushPods' per-UID runs with Added + Modified and Added + Deleted in
one batch, and a batch of echoes of the engine's own patches that must change
nothing."""
import numpy as np
import pytest

import test_controller_cpu as T
from fake_clientset import FakeClientset
from gpu_common import shim_read_check
from kwok_amd import abi, workload
from kwok_amd.controller import ingest_pod_runs, NOT_SENT
from kwok_amd.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _pair(deliver, geometry=T.SMALL, **kw):
    out = []
    for backend in (Engine, Oracle):
        cs = FakeClientset(deliver=deliver)
        out.append((cs, T.controller(cs, backend=backend, geometry=geometry, **kw)))
    return out


@pytest.mark.parametrize("deliver", ["sync", "queued"])
def test_drop_in_engine_equals_oracle(deliver):
    """200 nodes (a fifth unmanaged), 2000 pods created / modified / deleted
    over 6 ticks, an external node status change: every write the controller
    makes - PatchStatus of heartbeats and init patches, pod status patches,
    finalizer patches, deletes - is the same, body for body, on the engine and
    on the oracle, and so are the echo counts."""
    (ce, e), (co, o) = _pair(deliver, manage_nodes_with_annotation_selector=T.MANAGE, cidr="10.0.0.1/24")
    a = T.scenario(ce, e, ticks=6, nodes=200, pods_per_node=10, seed=11)
    b = T.scenario(co, o, ticks=6, nodes=200, pods_per_node=10, seed=11)
    for t, (x, y) in enumerate(zip(a, b)):
        assert x == y, "tick %d" % t
    assert sum(len(x) for x in a) > 2000
    assert (e.stats.echoes_on_arrival, e.stats.echoes_at_flush) == (o.stats.echoes_on_arrival, o.stats.echoes_at_flush)
    assert ce.store == co.store
    e.close()
    o.close()


@pytest.mark.parametrize("deliver", ["sync", "queued"])
def test_empty_status_same_interval_engine_vs_oracle(deliver):
    """the drop-in's step 6 (controller.py: an IP-less pod patch re-enters and
    the engine ticks again at the same clock) on the engine and on the oracle:
    every pod write equal, body for body, and both IPs in the first step"""
    (ce, e), (co, o) = _pair(deliver, manage_nodes_with_annotation_selector=T.MANAGE, node_ip="10.0.0.254",
                             cidr="10.0.0.1/24")
    a = T.empty_status_scenario(ce, e)
    b = T.empty_status_scenario(co, o)
    assert a == b and len(a[0]) == 5 and a[1] == a[2] == []
    assert e.stats.reentered == o.stats.reentered == 2
    assert ce.store == co.store
    e.close()
    o.close()


@pytest.mark.parametrize("name", ["test_reference_node_controller", "test_reference_pod_controller"])
def test_reference_tests_through_the_engine(name, monkeypatch):
    """node_controller_test.go / pod_controller_test.go, restated through the
    drop-in (tests/test_controller_cpu.py), with the HIP engine as the backend"""
    monkeypatch.setattr(T, "BACKEND", Engine)
    getattr(T, name)()


def test_c1_through_the_drop_in_engine_vs_oracle():
    """BASELINE configs[0]'s shape (1k nodes x 10k pods) through the drop-in:
    three ticks, every write equal on engine and oracle"""
    geo = dict(buckets=256, node_slots_per_bucket=32, pod_slots_per_bucket=128, pod_handle_stride=0,
               max_pod_specs=16)
    pair = _pair("queued", geometry=geo, manage_all_nodes=True, cidr="10.0.0.1/8")
    calls = []
    for cs, c in pair:
        for i in range(1000):
            cs.create(T.node("node-%07d" % i))
        for j in range(10000):
            cs.create(T.pod("pod-%08d" % j, "node-%07d" % (j // 10), containers=(("fake-pod", "fake"),),
                            status={"phase": "Pending"}))
        per = []
        for t in range(3):
            n0 = len(cs.calls)
            c.step(T.S0 + 30 * (t + 1))
            cs.pump()
            per.append(cs.calls[n0:])
        calls.append(per)
        c.close()
    assert [len(x) for x in calls[0]] == [0, 12000, 1000]  # the creates are delivered after tick 0
    assert calls[0] == calls[1]


NODES = 1_000_000


@pytest.mark.timeout(900)
def test_shim_ingest_sequence_1m_10m_heartbeat_once():
    shim_ingest_sequence(Engine, NODES)


def shim_ingest_sequence(engine_cls, nodes):
    """The metric's fleet on a heartbeat-once engine (engine_cgo.go's flags)
    and on the oracle.  After the initial tick, one batch in the order the shim
    hands it over: 20k new pods (Added), of which 5k are Modified and 3k Deleted
    later in the same batch (flushPods' runs); 1M echoes of the initial tick's
    pod patches (Modified, Running, conforming, with the patched IPs) - what the
    shim would ingest without dropping them; 10k deletion marks of existing
    pods.  Per-record handles / statuses, the tick's lists, its one heartbeat
    body and every patch (the shim's read sequence), counters and pod state
    equal the oracle's; the echoes change nothing (no echoed pod is patched or
    moved), and a steady tick after equals the oracle too."""
    NODES = nodes
    e, fl, ph = workload.build_engine_fleet(engine_cls, NODES, heartbeat_once=True)
    o, _, ph2 = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=0), NODES)
    assert (ph == ph2).all()
    n_slots = workload.BUCKETS * fl.cp
    now = workload.S0 + 30
    r0 = e.tick(now, read=False)
    o.tick(now, read=False)
    assert r0.n_heartbeat == NODES and (r0.heartbeat_stride == 0 or engine_cls is not Engine)
    O = o.read_arrays()
    shim_read_check(e, O, r0)
    assert list(r0.counters) == [O["counters"][k] for k in abi.COUNTERS]

    rng = np.random.default_rng(42)
    used, phase, hip, pip = e.dump_pods(0, n_slots)
    spec = 0
    # event list, in watch order: uid per record (existing pods: their handle; new: -1 - k)
    n_new, n_mod, n_del, n_echo, n_mark = (np.array([20_000, 5_000, 3_000, 1_000_000, 10_000]) * NODES
                                           // 1_000_000).tolist()
    echo_h = rng.choice(ph, n_echo, replace=False)
    mark_h = rng.choice(np.setdiff1d(ph, echo_h), n_mark, replace=False)
    new_nodes = rng.choice(fl.node_handles, n_new)
    nip = workload.NODE_IP.encode()
    ip_buf, ip_off, ip_len = workload.ip_strings(pip[echo_h], base=len(nip))
    ip_buf2, ip_off2, ip_len2 = workload.ip_strings(pip[mark_h], base=len(nip) + ip_buf.size)
    arena = nip + ip_buf.tobytes() + ip_buf2.tobytes()

    def new_rec(k):
        r = np.zeros(len(k), abi.POD_EVENT_DTYPE)
        r["spec_id"] = spec
        r["node_handle"] = new_nodes[k]
        r["phase"] = abi.PHASE_PENDING
        r["flags"] = abi.POD_STATUS_NONEMPTY
        r["creation_unix"] = now + 10
        return r

    parts, uids, dels = [], [], []

    def add(r, u, d=False):
        parts.append(r)
        uids.extend(u)
        dels.extend([d] * len(u))

    half = n_new // 2
    add(new_rec(np.arange(half)), [-1 - k for k in range(half)])              # Added (first half)
    e_rec = np.zeros(n_echo, abi.POD_EVENT_DTYPE)                            # echoes of tick 0's patches
    e_rec["spec_id"] = spec
    e_rec["node_handle"] = -1
    e_rec["phase"] = abi.PHASE_RUNNING
    e_rec["flags"] = abi.POD_STATUS_NONEMPTY | abi.POD_CONFORMS
    e_rec["creation_unix"] = workload.S0 - 60
    e_rec["host_ip"]["off"], e_rec["host_ip"]["len"] = 0, len(nip)
    e_rec["pod_ip"]["off"], e_rec["pod_ip"]["len"] = ip_off, ip_len
    add(e_rec[: n_echo // 2], echo_h[: n_echo // 2].tolist())
    mod = rng.choice(half, n_mod, replace=False)                             # Added + Modified
    add(new_rec(mod), [-1 - int(k) for k in mod])
    add(new_rec(np.arange(half, n_new)), [-1 - k for k in range(half, n_new)])  # Added (second half)
    m_rec = np.zeros(n_mark, abi.POD_EVENT_DTYPE)                            # deletionTimestamp set
    m_rec["spec_id"] = spec
    m_rec["node_handle"] = -1
    m_rec["phase"] = abi.PHASE_RUNNING
    m_rec["flags"] = abi.POD_STATUS_NONEMPTY | abi.POD_CONFORMS | abi.POD_DELETING | \
        np.where(rng.random(n_mark) < 0.5, abi.POD_HAS_FINALIZERS, 0)
    m_rec["creation_unix"] = workload.S0 - 60
    m_rec["host_ip"]["off"], m_rec["host_ip"]["len"] = 0, len(nip)
    m_rec["pod_ip"]["off"], m_rec["pod_ip"]["len"] = ip_off2, ip_len2
    add(m_rec, mark_h.tolist())
    add(e_rec[n_echo // 2:], echo_h[n_echo // 2:].tolist())
    gone = rng.choice(n_new, n_del, replace=False)                           # Added + Deleted
    add(np.zeros(n_del, abi.POD_EVENT_DTYPE), [-1 - int(k) for k in gone], True)
    recs = np.concatenate(parts)
    known = {int(h): int(h) for h in np.concatenate([echo_h, mark_h])}

    res = []
    for b in (e, o):
        r = recs.copy()
        res.append(ingest_pod_runs(b, dict(known), r, uids, dels, arena))
    (h1, s1, runs1), (h2, s2, runs2) = res
    assert runs1 == runs2 >= 3
    assert (h1 == h2).all() and (s1 == s2).all()
    assert (s1[np.asarray(dels)] == abi.OK).all() and ((s1 == abi.OK) | (s1 == NOT_SENT)).all()

    now += 30
    r1 = e.tick(now, read=False)
    o.tick(now, read=False)
    O = o.read_arrays()
    shim_read_check(e, O, r1)
    c = dict(zip(abi.COUNTERS, list(r1.counters)))
    assert c == O["counters"]
    # the echoes changed nothing: the patches are exactly the surviving new pods
    assert c["pod_patch"] == n_new - n_del and c["delete"] == n_mark and c["alloc"] == n_new - n_del
    assert c["release"] == n_mark and c["heartbeat"] == NODES
    u2, p2, hi2, pi2 = e.dump_pods(0, n_slots)
    assert (pi2[echo_h] == pip[echo_h]).all() and (p2[echo_h] == phase[echo_h]).all()
    ou, op, oh, oi = o.dump_pods(0, n_slots)
    assert (ou == u2).all() and (op == p2).all() and (oh == hi2).all() and (oi == pi2).all()
    # deletes reused the released addresses lowest first, in the same tick
    now += 30
    r2 = e.tick(now, read=False)
    o.tick(now, read=False)
    O = o.read_arrays()
    shim_read_check(e, O, r2)
    c = dict(zip(abi.COUNTERS, list(r2.counters)))
    assert c == O["counters"] and c["pod_patch"] == 0 and c["heartbeat"] == NODES
    e.close()
    o.close()
