"""The compact wire form of pod events (kwok_pod_rec, kwok_ingest_pods_packed):
20 bytes per record, the strings parsed by the caller (IPv4 integers, the node
by handle).  CPU side: kwok_pack_pod_events against the vectorised packing the
churn generator uses, its rejections, and every golden trace replayed on the
oracle with the pods in the compact form wherever it can carry them (the rest
in kwok_pod_event calls, in event order) - the same handles, statuses, patch
bytes and state as the fixtures (pod_controller.go:301-343)."""
import numpy as np
import pytest

import harness
from kwok_amd import abi
from kwok_amd.engine import pack_pod_events
from oracle.oracle import Oracle


def test_record_is_20_bytes():
    assert abi.POD_REC_DTYPE.itemsize == 20


def test_pack_matches_vectorised_packing():
    rng = np.random.default_rng(1)
    n = 500
    ev = np.zeros(n, abi.POD_EVENT_DTYPE)
    ev["op"] = rng.choice([abi.OP_UPSERT, abi.OP_DELETE], n)
    ev["handle"] = np.where(rng.random(n) < 0.5, -1, rng.integers(0, 1 << 20, n))
    ev["handle"] = np.where(ev["op"] == abi.OP_DELETE, rng.integers(0, 1 << 20, n), ev["handle"])
    ev["node_handle"] = rng.integers(0, 1 << 16, n)
    ev["spec_id"] = rng.integers(0, 7, n)
    ev["phase"] = rng.integers(0, 6, n)
    ev["flags"] = rng.integers(0, 32, n)
    ev["creation_unix"] = rng.integers(0, 1 << 32, n)
    hip = np.where(rng.random(n) < 0.5, rng.integers(1, 1 << 32, n), 0).astype(np.uint32)
    pip = np.where(rng.random(n) < 0.5, rng.integers(1, 1 << 32, n), 0).astype(np.uint32)
    ar = abi.Arena()
    for i in range(n):
        ev[i]["host_ip"] = ar.ref(abi.ip4s(int(hip[i])))
        ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(pip[i])))
    got, st = pack_pod_events(ev, bytes(ar.buf))
    assert (st == abi.OK).all()
    want = abi.pack_pod_events(ev, hip, pip)
    assert got.tobytes() == want.tobytes()


def test_pack_rejections():
    ar = abi.Arena()
    ev = np.zeros(7, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = -1
    ev["node_handle"] = 3
    ev[0]["node_handle"] = -1                    # a create by spec.nodeName: the full form only
    ev[0]["node_name"] = ar.ref("node-a")
    ev[1]["pod_ip"] = ar.ref("10.0.0.01")        # not canonical
    ev[2]["host_ip"] = ar.ref("0.0.0.0")         # the zero address
    ev[3]["creation_unix"] = -5                  # before 1970
    ev[4]["op"] = 7                              # no such op
    ev[5]["pod_ip"] = ar.ref("10.0.0.7")         # fine
    ev[6]["phase"] = abi.PHASE_OTHER             # a node phase, not a pod's (kwok_ingest_pods rejects it too)
    out, st = pack_pod_events(ev, bytes(ar.buf))
    assert list(st) == [abi.EINVAL, abi.EDOMAIN, abi.EDOMAIN, abi.EDOMAIN, abi.EINVAL, abi.OK, abi.EINVAL]
    assert out[5]["pod_ip"] == abi.ip4("10.0.0.7") and out[5]["op"] == abi.OP_UPSERT | abi.REC_NEW
    assert out[5]["target"] == 3


@pytest.mark.parametrize("name", harness.TRACES)
def test_oracle_trace_packed(name):
    fx = harness.load_trace(name)
    o = Oracle(harness.config_for(fx))
    harness.replay(fx, o, packed=True)
    o.close()


def test_packed_create_without_node_handle_is_rejected_per_record():
    fx = harness.load_trace("doc_known_answer")
    o = Oracle(harness.config_for(fx))
    recs = np.zeros(2, abi.POD_REC_DTYPE)
    recs["op"] = abi.OP_UPSERT | abi.REC_NEW
    recs["target"] = -1
    hs, st, rel = o.ingest_pods_packed(recs)
    assert list(st) == [abi.EINVAL, abi.EINVAL] and list(hs) == [-1, -1]
    o.close()
