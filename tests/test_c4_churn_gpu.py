"""GPU parity of the C4 pod churn storm (BASELINE configs[3]: create/delete
churn exercising ipPool release/reuse and deletion finalizers) against the CPU
oracle, tick by tick on every output and on the full pod state:
  * at reduced size with batches above the engine's threaded-ingest threshold
    (the partitioned host ingest, engine.cpp kwok_ingest_pods), for several
    ingest thread counts;
  * at the metric's size: 1M nodes x 10M pods, 1M deletion-marked pods (half
    with finalizers) + 1M creates per tick (2M create/delete per tick).
Reference: pod_controller.go:155-202 (DeletePod), :301-343 (WatchPods
routing), utils.go:83-108 (ipPool Get/Put)."""
import os

import numpy as np
import pytest

from gpu_common import compare_state, compare_tick
from kwok_amd import workload
from kwok_amd.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def run_churn(nodes, n_churn, ticks, buckets=workload.BUCKETS, threads=None, full_state=True, alloc=None,
              packed=False, once=False, shim=False, together=False):
    """packed: the engine ingests the compact wire form (kwok_ingest_pods_packed;
    packed=12: kwok_pod_rec12 through kwok_ingest_pods_packed12, which returns the
    creates' handles only), the oracle the same events as kwok_pod_event with
    dotted quads.  once: heartbeat-once engines (the drop-in's).  shim: every churn
    tick is also read back as the Go drop-in reads it (gpu_common.shim_read_check:
    lists, one heartbeat body, every patch byte in 64 MiB pieces) and compared with
    the oracle byte for byte.  together: kwok_ingest_pods_packed12_tick (the tick
    queued behind the batch's apply passes), the oracle's two calls beside it"""
    from gpu_common import shim_read_check
    if threads is not None:
        os.environ["KWOK_INGEST_THREADS"] = str(threads)
    try:
        e, fl, ph = workload.build_engine_fleet(Engine, nodes, buckets=buckets, heartbeat_once=once)
    finally:
        os.environ.pop("KWOK_INGEST_THREADS", None)
    o, _, ph2 = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=0), nodes, buckets=buckets)
    assert (ph == ph2).all()
    n_handles = buckets * fl.cp
    now = workload.S0 + 30
    e.tick(now, read=False)
    o.tick(now, read=False)
    compare_tick(e, o, "churn initial tick", once)
    ch = workload.Churn(ph, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_handles, n_churn, seed=11,
                        alloc=alloc)
    chp = workload.Churn(ph, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_handles, n_churn, seed=11,
                         alloc=alloc, packed=packed) if packed else None
    dump = lambda: o.dump_pods(0, n_handles)  # noqa: E731
    for t in range(ticks):
        now += 30
        ev, ar = ch.batch(dump, now)
        if packed == 12:
            recs, _ = chp.batch(dump, now)
            assert recs.dtype.itemsize == 12
            nh, s1, r1 = e.ingest_pods_packed12(recs, tick_now=now if together else None)
            assert len(nh) == n_churn
            chp.applied(nh.copy(), s1, new_only=True)
            # every other record's handle is its target
            h1 = np.concatenate([recs["target"][:len(recs) - len(nh)], nh])
        elif packed:
            recs, _ = chp.batch(dump, now)
            h1, s1, r1 = e.ingest_pods_packed(recs)
            chp.applied(h1.copy(), s1)
        else:
            h1, s1, r1 = e.ingest_pods_raw(ev, ar)
        h2, s2, r2 = o.ingest_pods_raw(ev, ar)
        assert (h1 == h2).all() and (s1 == s2).all() and (r1 == r2).all(), "churn tick %d ingest" % t
        ch.applied(h1, s1)
        res = e.tick_collect(read=False) if together else e.tick(now, read=False)
        o.tick(now, read=False)
        if shim:
            pieces, nbytes = shim_read_check(e, o.read_arrays(), res)
            assert nbytes > 0.5e9 or nodes < 1_000_000, nbytes
        c = compare_tick(e, o, "churn tick %d" % t, once)
        assert (c["delete"], c["release"], c["pod_patch"], c["alloc"]) == (n_churn,) * 4, c
        if full_state or t == ticks - 1:
            compare_state(e, o, n_handles, "churn tick %d" % t)
    e.close()
    o.close()


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_churn_threaded_ingest_parity(threads):
    """20k nodes x 200k pods, 40k deletes + 40k creates per tick (80k records:
    above the threaded-ingest threshold)"""
    run_churn(20_000, 40_000, 3, threads=threads)


@pytest.mark.timeout(900)
def test_c4_churn_metric_size():
    """1M nodes x 10M pods, 1M deletes (50% finalizers) + 1M creates per tick"""
    run_churn(1_000_000, 1_000_000, 2, full_state=False)


@pytest.mark.timeout(900)
def test_c4_churn_metric_size_packed():
    """the same churn storm with the engine fed the compact wire form (20 B per
    record, kwok_ingest_pods_packed, page-locked and read in place), the
    oracle the full kwok_pod_event records: equal per record and per tick"""
    from kwok_amd.engine import host_array
    run_churn(1_000_000, 1_000_000, 2, full_state=False, packed=True, alloc=host_array)


def test_churn_packed_parity():
    """20k nodes x 200k pods, 40k + 40k per tick, compact records in pageable memory"""
    run_churn(20_000, 40_000, 3, packed=True)


@pytest.mark.timeout(900)
def test_c4_churn_metric_size_packed12():
    """the metric-size storm through kwok_pod_rec12 (12 B per record: hostIP as
    a flag, the marked pods' creation times kept by the engine; the creates'
    handles only back; page-locked and read in place): equal to the oracle per
    record and per tick"""
    from kwok_amd.engine import host_array
    run_churn(1_000_000, 1_000_000, 2, full_state=False, packed=12, alloc=host_array)


@pytest.mark.timeout(900)
def test_c4_churn_metric_size_ingest_then_tick():
    """kwok_ingest_pods_packed12_tick at 1M nodes x 10M pods (the tick's kernels
    queued behind the batch, running while the results travel), heartbeat-once
    engines, every churn tick read back as the drop-in reads it"""
    from kwok_amd.engine import host_array
    run_churn(1_000_000, 1_000_000, 2, full_state=False, packed=12, alloc=host_array, once=True, shim=True,
              together=True)


def test_churn_ingest_then_tick_parity():
    """20k nodes x 200k pods, 40k + 40k per tick, the full state every tick"""
    run_churn(20_000, 40_000, 3, packed=12, together=True)


@pytest.mark.timeout(900)
def test_c4_churn_metric_size_drop_in_read_back():
    """the drop-in's C4: heartbeat-once engines, kwok_pod_rec12, and every churn
    tick read back as engine_cgo.go reads it (0.58 GB of patches per tick in 64 MiB
    pieces), byte for byte against the oracle at 1M nodes x 10M pods"""
    from kwok_amd.engine import host_array
    run_churn(1_000_000, 1_000_000, 2, full_state=False, packed=12, alloc=host_array, once=True, shim=True)


@pytest.mark.parametrize("buckets", [1024, 8192, 16384])
def test_churn_bucket_counts(buckets):
    """the bucket sort's three forms (ingest.hip bucket_sort): 8 scatter waves per
    tile up to 4607 local buckets, 4 waves up to 8447, rocPRIM's radix sort past
    that - 20k nodes x 200k pods, 40k + 40k per tick in kwok_pod_rec12"""
    run_churn(20_000, 40_000, 2, buckets=buckets, packed=12)


@pytest.mark.parametrize("chunk", [None, "70000"])
def test_churn_packed12_parity(chunk, monkeypatch):
    """20k nodes x 200k pods, 40k + 40k per tick as kwok_pod_rec12 in pageable
    memory; chunk: KWOK_INGEST_CHUNK small enough that every batch runs in two
    chunks (the creates' ordinals cross the chunk boundary)"""
    if chunk:
        monkeypatch.setenv("KWOK_INGEST_CHUNK", chunk)
    run_churn(20_000, 40_000, 3, packed=12)


def test_packed12_edges():
    """kwok_ingest_pods_packed12 on a small engine against kwok_ingest_pods_packed
    on a twin: rejected creates (a node handle the engine does not hold, a bad
    spec) get -1 at their create ordinal; a hostIP flag stands for the node IP; an
    update keeps the pod's creation time; a create count above new_cap fails
    after the batch is applied (the engine stays usable); an empty batch"""
    from kwok_amd import abi
    e1, fl, ph = workload.build_engine_fleet(Engine, 2_000)
    e2, _, _ = workload.build_engine_fleet(Engine, 2_000)
    now = workload.S0 + 30
    e1.tick(now, read=False)
    e2.tick(now, read=False)
    node_ip = abi.ip4(workload.NODE_IP)
    n = 64
    r = np.zeros(n, abi.POD_REC_DTYPE)
    r["op"] = abi.OP_UPSERT | abi.REC_NEW
    r["target"] = np.resize(fl.node_handles, n)
    r["flags"] = abi.POD_STATUS_NONEMPTY | (abi.PHASE_PENDING << abi.REC_PHASE_SHIFT)
    r["creation"] = now
    r["target"][5] = 1 << 30      # a node handle nobody holds
    r["spec_id"][9] = 4000        # no such spec
    r["host_ip"][11] = node_ip    # a create that already holds the node IP
    r[20]["op"] = abi.OP_UPSERT   # a modify of an existing pod (its creation time: the fleet's)
    r[20]["target"] = ph[0]
    r[20]["host_ip"] = node_ip
    r[20]["creation"] = workload.S0 - 60
    r[20]["flags"] = abi.POD_STATUS_NONEMPTY | abi.POD_CONFORMS | (abi.PHASE_RUNNING << abi.REC_PHASE_SHIFT)
    r12 = abi.pack12(r, node_ip)
    h2, s2, rel2 = e2.ingest_pods_packed(r)
    nh, s1, rel1 = e1.ingest_pods_packed12(r12)
    new = (r["op"] & abi.REC_NEW) != 0
    assert (s1 == s2).all() and (rel1 == rel2).all()
    assert (nh == h2[new]).all() and nh[5] == -1 and nh[9] == -1 and (s1[[5, 9]] != 0).all()
    now += 30
    t1, t2 = e1.tick(now), e2.tick(now)
    assert list(t1.counters) == list(t2.counters)
    with pytest.raises(ValueError):  # another hostIP: not expressible
        abi.pack12(np.array([(abi.OP_UPSERT, 0, 0, ph[1], now, node_ip + 1, 0)], abi.POD_REC_DTYPE), node_ip)
    # new_cap below the creates: the batch applies, the call fails, the engine carries on
    r2 = r12[:8].copy()
    r2["target"][5] = fl.node_handles[0]
    with pytest.raises(RuntimeError):
        e1.ingest_pods_packed12(r2, new_cap=4)
    e1.ingest_pods_packed12(r12[:0])
    now += 30
    e1.tick(now)
    e1.close()
    e2.close()
