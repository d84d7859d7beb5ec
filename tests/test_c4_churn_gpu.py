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
              packed=False):
    """packed: the engine ingests the compact wire form (kwok_ingest_pods_packed),
    the oracle the same events as kwok_pod_event with dotted quads"""
    if threads is not None:
        os.environ["KWOK_INGEST_THREADS"] = str(threads)
    try:
        e, fl, ph = workload.build_engine_fleet(Engine, nodes, buckets=buckets)
    finally:
        os.environ.pop("KWOK_INGEST_THREADS", None)
    o, _, ph2 = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=0), nodes, buckets=buckets)
    assert (ph == ph2).all()
    n_handles = buckets * fl.cp
    now = workload.S0 + 30
    e.tick(now, read=False)
    o.tick(now, read=False)
    compare_tick(e, o, "churn initial tick")
    ch = workload.Churn(ph, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_handles, n_churn, seed=11,
                        alloc=alloc)
    chp = workload.Churn(ph, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_handles, n_churn, seed=11,
                         alloc=alloc, packed=True) if packed else None
    dump = lambda: o.dump_pods(0, n_handles)  # noqa: E731
    for t in range(ticks):
        now += 30
        ev, ar = ch.batch(dump, now)
        if packed:
            recs, _ = chp.batch(dump, now)
            h1, s1, r1 = e.ingest_pods_packed(recs)
            chp.applied(h1.copy(), s1)
        else:
            h1, s1, r1 = e.ingest_pods_raw(ev, ar)
        h2, s2, r2 = o.ingest_pods_raw(ev, ar)
        assert (h1 == h2).all() and (s1 == s2).all() and (r1 == r2).all(), "churn tick %d ingest" % t
        ch.applied(h1, s1)
        e.tick(now, read=False)
        o.tick(now, read=False)
        c = compare_tick(e, o, "churn tick %d" % t)
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
