"""GPU parity of pod-capacity growth: buckets start small (pod_slots_per_bucket)
and grow up to the handle stride when a batch of creates would fill one, so a
skewed fleet - the reference benchmark's 1000 pods on one node
(test/kwokctl/kwokctl_benchmark_test.sh:119-124,159-160) - never hits
KWOK_EFULL below the stride.  Handles (bucket * stride + index), canonical
order and IP order do not change with the capacity; the oracle holds every
bucket at the stride from the start, so equality with it checks exactly that."""
import numpy as np
import pytest

from gpu_common import Driver, external_deletes, mark_deleting, new_pods
from kwok_amd import abi

pytestmark = pytest.mark.gpu


def pods_on(d, node_handle, n, spec):
    ev = np.zeros(n, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = -1
    ev["node_handle"] = node_handle
    ev["spec_id"] = spec
    ev["phase"] = abi.PHASE_PENDING
    ev["flags"] = abi.POD_STATUS_NONEMPTY
    ev["creation_unix"] = 1704067140
    return d.pods(ev)


@pytest.mark.parametrize("threads", [None, "1"])
def test_1000_pods_on_one_node_grow(threads, monkeypatch):
    if threads:
        monkeypatch.setenv("KWOK_INGEST_THREADS", threads)
    kw = dict(cidr="10.0.0.1/16", node_ip="196.168.0.1", buckets=64, node_slots_per_bucket=8,
              pod_slots_per_bucket=16, pod_handle_stride=8192)
    d = Driver(kw, 3)
    names = ["node-%07d" % i for i in range(40)]
    nh, st = d.nodes(names, managed=1, lockable=1)
    assert (st == 0).all()
    h, s, _ = pods_on(d, nh[0], 1000, d.spec[0])  # 16 -> 1000+ slots in one batch
    assert (s == 0).all()
    ev, ar = new_pods(d.rng, nh, 400, d.spec)
    d.pods(ev, ar)
    d.tick("skew tick 0")
    # handles from before the growth stay valid: delete half the big node's pods
    ev, ar = mark_deleting(d.rng, d, np.sort(h[::2]).astype(np.int32))
    d.pods(ev, ar)
    ev, ar = external_deletes(d, np.sort(h[1:200:2]).astype(np.int32))
    d.pods(ev, ar)
    d.tick("skew tick 1")
    # a second hot node in another bucket, in a batch above the threaded-ingest
    # threshold (40000 more pods spread over the fleet), past 2x the capacity
    hot = np.zeros(5000, abi.POD_EVENT_DTYPE)
    hot["op"] = abi.OP_UPSERT
    hot["handle"] = -1
    hot["node_handle"] = nh[7]
    hot["spec_id"] = d.spec[1]
    hot["phase"] = abi.PHASE_PENDING
    hot["flags"] = abi.POD_STATUS_NONEMPTY
    hot["creation_unix"] = 1704067140
    ev, ar = new_pods(d.rng, nh, 40_000, d.spec)
    _, s2, _ = d.pods(np.concatenate([hot, ev]), ar)
    assert (s2 == 0).all()
    d.tick("skew tick 2")
    d.tick_pair("skew tick 3")
    assert d.e.node_size() == d.o.node_size()
    d.e.close()
    d.o.close()


def test_efull_at_the_stride():
    kw = dict(cidr="10.0.0.1/16", node_ip="196.168.0.1", buckets=16, node_slots_per_bucket=4,
              pod_slots_per_bucket=8, pod_handle_stride=64)
    d = Driver(kw, 4)
    nh, _ = d.nodes(["n0", "n1"], managed=1, lockable=1)
    h, s, _ = pods_on(d, nh[0], 100, d.spec[0])  # compared with the oracle inside Driver.pods
    assert (s[:64] == abi.OK).all() and (s[64:] == abi.EFULL).all()
    d.tick("efull tick")
    d.e.close()
    d.o.close()
