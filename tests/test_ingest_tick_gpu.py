"""GPU: kwok_ingest_pods_packed12_tick - a batch of kwok_pod_rec12 records with its
tick queued behind the batch's apply passes (engine.cpp ingest_pods_impl, tick
mode: the tick's kernels run while the per-record results travel back) - against
the oracle fed the same records and then ticked, call for call: handles,
statuses, every tick's outputs and the pod state.  Includes a batch whose creates
overflow a bucket (the tick's launches skip on the device, the call grows the
buckets, applies the chunk and queues the tick again), in one chunk and in
several (KWOK_INGEST_CHUNK), and the checks made before the batch is touched.
Reference: pod_controller.go:301-343 (the watch events), :377-439 (the tick's
patches), utils.go:83-108 (the pool)."""
import numpy as np
import pytest

from gpu_common import Driver, compare, compare_state, external_deletes, mark_deleting, new_pods
from kwok_amd import abi
from kwok_amd.engine import KwokError

pytestmark = pytest.mark.gpu

NODE_IP = "196.168.0.1"


def packed12(d, ev):
    """ev (kwok_pod_event rows) as kwok_pod_rec12, the IPs from the live pods"""
    hip = np.zeros(len(ev), np.uint32)
    pip = np.zeros(len(ev), np.uint32)
    old = ev["handle"] >= 0
    if old.any():
        idx, _, h, p = d.live()
        pos = np.searchsorted(idx, ev["handle"][old])
        hip[old] = np.where(ev["op"][old] == abi.OP_UPSERT, h[pos], 0)
        pip[old] = p[pos]
    return abi.pack12(abi.pack_pod_events(ev, hip, pip), abi.ip4(NODE_IP))


def step(d, ev, arena, where):
    """the engine: ev as kwok_pod_rec12 with its tick behind it; the oracle: ev, then a tick"""
    recs = packed12(d, ev)
    nh, s1, _ = d.e.ingest_pods_packed12(recs, tick_now=d.now)
    h2, s2, _ = d.o.ingest_pods_raw(ev, arena)
    assert (s1 == s2).all(), where + " statuses"
    new = (ev["op"] == abi.OP_UPSERT) & (ev["handle"] < 0)
    assert (nh == h2[new]).all(), where + " create handles"
    ok = new & (s2 == 0)
    d.spec_of[h2[ok]] = ev["spec_id"][ok]
    d.ctime_of[h2[ok]] = ev["creation_unix"][ok]
    eo = d.e.tick_collect()
    oo = d.o.tick(d.now)
    d.now += 30
    compare(eo, oo, where)
    compare_state(d.e, d.o, d.n_slots, where)
    return h2


def test_ingest_then_tick_equals_the_two_calls():
    """creates, deletion marks (half with finalizers) and external deletes in
    mixed batches, each with its tick behind it"""
    kw = dict(cidr="10.0.0.1/16", node_ip=NODE_IP, buckets=64, node_slots_per_bucket=16, pod_slots_per_bucket=256)
    d = Driver(kw, 21, specs=[Driver.DEFAULT_SPECS[0]])
    nh, st = d.nodes(["node-%07d" % i for i in range(300)], managed=1, lockable=1)
    assert (st == 0).all()
    ev, ar = new_pods(d.rng, nh, 3000, d.spec)
    step(d, ev, ar, "creates")
    for t in range(4):
        idx, _, _, _ = d.live()
        pick = np.sort(d.rng.choice(idx, 600, replace=False)).astype(np.int32)
        dm, _ = mark_deleting(d.rng, d, pick[:400])
        xd, _ = external_deletes(d, pick[400:])
        cr, _ = new_pods(d.rng, nh, 700, d.spec)
        # (the oracle reads the IPs from the strings: give it the same batch as events)
        batch = np.concatenate([dm, xd, cr])
        arena = _ip_arena(d, batch)
        step(d, batch, arena, "churn %d" % t)
    d.e.close()
    d.o.close()


def _ip_arena(d, ev):
    """the batch's IPs as strings for the oracle's kwok_pod_event form"""
    ar = abi.Arena()
    old = np.nonzero(ev["handle"] >= 0)[0]
    if len(old):
        idx, _, h, p = d.live()
        pos = np.searchsorted(idx, ev["handle"][old])
        for i, q in zip(old, pos):
            ev[i]["host_ip"] = ar.ref(abi.ip4s(int(h[q]))) if h[q] and ev[i]["op"] == abi.OP_UPSERT else (0, 0)
            ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(p[q]))) if p[q] else (0, 0)
    return bytes(ar.buf)


@pytest.mark.parametrize("chunk", [None, "300"])
def test_ingest_then_tick_grows_the_buckets(chunk, monkeypatch):
    """1000 creates on one node in buckets of 16 pod slots: the tick queued behind
    the batch skips on the device until the call has grown the buckets and applied
    the chunk, then runs (one chunk, and chunks of 300 records: the growth in the
    batch's first chunk, the others applied with the host in the loop)"""
    if chunk:
        monkeypatch.setenv("KWOK_INGEST_CHUNK", chunk)
    kw = dict(cidr="10.0.0.1/16", node_ip=NODE_IP, buckets=64, node_slots_per_bucket=8, pod_slots_per_bucket=16,
              pod_handle_stride=8192)
    d = Driver(kw, 5, specs=[Driver.DEFAULT_SPECS[0]])
    nh, _ = d.nodes(["node-%07d" % i for i in range(40)], managed=1, lockable=1)
    ev = np.zeros(1000, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = -1
    ev["node_handle"] = nh[3]
    ev["spec_id"] = d.spec[0]
    ev["phase"] = abi.PHASE_PENDING
    ev["flags"] = abi.POD_STATUS_NONEMPTY
    ev["creation_unix"] = 1704067140
    h = step(d, ev, b"", "grown")
    assert (h >= 0).all()
    more, ar = new_pods(d.rng, nh, 500, d.spec)
    step(d, more, ar, "after the growth")
    d.e.close()
    d.o.close()


def test_ingest_then_tick_checks_first():
    """two ticks outstanding: the call fails with KWOK_EBUSY before the batch is
    touched (the oracle, which never saw it, still equals the engine)"""
    kw = dict(cidr="10.0.0.1/16", node_ip=NODE_IP, buckets=16, node_slots_per_bucket=8, pod_slots_per_bucket=64)
    d = Driver(kw, 9, specs=[Driver.DEFAULT_SPECS[0]])
    nh, _ = d.nodes(["node-%07d" % i for i in range(20)], managed=1, lockable=1)
    d.e.tick_submit(d.now)
    d.e.tick_submit(d.now + 30)
    ev, _ = new_pods(d.rng, nh, 50, d.spec)
    with pytest.raises(KwokError, match="outstanding"):
        d.e.ingest_pods_packed12(packed12(d, ev), tick_now=d.now + 60)
    for k in range(2):
        eo, oo = d.e.tick_collect(), d.o.tick(d.now)
        d.now += 30
        compare(eo, oo, "queued tick %d" % k)
    compare_state(d.e, d.o, d.n_slots, "after the refused batch")
    d.e.close()
    d.o.close()


def test_ingest_then_tick_edges():
    """an empty batch (the tick alone), and a batch with more creates than
    out_new_handles holds: the call reports KWOK_EINVAL once the batch is applied
    (the engine stays usable) and the tick behind it is the oracle's"""
    kw = dict(cidr="10.0.0.1/16", node_ip=NODE_IP, buckets=16, node_slots_per_bucket=8, pod_slots_per_bucket=64)
    d = Driver(kw, 13, specs=[Driver.DEFAULT_SPECS[0]])
    nh, _ = d.nodes(["node-%07d" % i for i in range(20)], managed=1, lockable=1)
    ev, ar = new_pods(d.rng, nh, 100, d.spec)
    step(d, ev, ar, "first batch")
    # the tick alone
    d.e.ingest_pods_packed12(np.zeros(0, abi.POD_REC12_DTYPE), tick_now=d.now)
    eo, oo = d.e.tick_collect(), d.o.tick(d.now)
    d.now += 30
    compare(eo, oo, "empty batch")
    # room for 10 of 40 create handles
    ev, ar = new_pods(d.rng, nh, 40, d.spec)
    with pytest.raises(KwokError, match="out_new_handles"):
        d.e.ingest_pods_packed12(packed12(d, ev), new_cap=10, tick_now=d.now)
    h2, s2, _ = d.o.ingest_pods_raw(ev, ar)
    ok = s2 == 0
    d.spec_of[h2[ok]] = ev["spec_id"][ok]
    d.ctime_of[h2[ok]] = ev["creation_unix"][ok]
    eo, oo = d.e.tick_collect(), d.o.tick(d.now)
    d.now += 30
    compare(eo, oo, "batch past new_cap")
    compare_state(d.e, d.o, d.n_slots, "batch past new_cap")
    d.e.close()
    d.o.close()
