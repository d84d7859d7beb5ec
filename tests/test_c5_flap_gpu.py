"""GPU parity of BASELINE configs[4] at full size: 1M nodes (10M pods) with
ManageAllNodes=false and an annotation selector matching 50% of the nodes, a
disregard annotation on 0.1%, and 1% of the managed nodes deleted and created
again every tick (workload.Flap), against the CPU oracle on every output and
on the pod state.  Reference: node_controller.go:206-223 (needHeartbeat /
needLockNode), :256-270 (watch routing), :356-391 (configureNode)."""
import numpy as np
import pytest

from gpu_common import compare_tick
from harness import DISREGARD, MANAGE
from kwok_amd import abi, workload
from kwok_amd.codec import Codec
from kwok_amd.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
@pytest.mark.parametrize("wire", ["records", "json"])
def test_c5_flap_partial_management_1m_nodes(wire):
    """wire=json: the engine takes each flap batch as the watch's node documents
    (kwok_ingest_nodes_json: the Deleted events carry the nodes as kwok patched
    them, the Added ones a zero status), decoded on the GPU with none left to the
    host, while the oracle takes the records; the first batch's documents are
    also decoded record for record against the host codec"""
    kw = dict(managed_frac=0.5, lockable_frac=0.999, seed=5)
    e, fl, ph = workload.build_engine_fleet(Engine, 1_000_000, **kw)
    o, _, ph2 = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=0), 1_000_000, **kw)
    assert (ph == ph2).all()
    managed = int(fl.node_events["managed"].sum())
    now = workload.S0 + 30
    e.tick(now, read=False)
    o.tick(now, read=False)
    c = compare_tick(e, o, "c5 tick 0")
    assert c["heartbeat"] == managed and c["pod_patch"] == 10 * managed
    f = workload.Flap(fl, 0.01, seed=6)
    codec = Codec(manage_all_nodes=False, manage_nodes_with_annotation_selector=MANAGE,
                  disregard_status_with_annotation_selector=DISREGARD)
    for t in range(1, 3):
        now += 30
        if wire == "json":
            arena, offs, lens, ops, ev = f.batch_json()
            ar = fl.arena
            if t == 1:
                gev, gst, gnh, _ = e.decode_nodes_gpu(codec, arena=arena, offs=offs, lens=lens)
                b = codec.decode_nodes([arena[int(a):int(a) + int(n)] for a, n in zip(offs, lens)], strict=False,
                                       threads=16)
                assert (gst == 0).all() and list(b.status) == [0] * len(offs) and gnh == f.k  # (deleted: blobs)
                hb = np.frombuffer(b"".join(bytes(x) for x in b.nodes), abi.NODE_EVENT_DTYPE)
                assert gev.tobytes() == hb.tobytes()  # record for record
            h1, s1, nh = e.ingest_nodes_json(codec, arena, offs, lens, ops)
            assert nh == 0  # (deleted nodes' statuses are not read; the added ones are empty)
        else:
            ev, ar = f.batch()
            h1, s1 = e.ingest_nodes_raw(ev, ar)
        h2, s2 = o.ingest_nodes_raw(ev, ar)
        assert (h1 == h2).all() and (s1 == s2).all() and (s1 == 0).all()
        assert e.node_size() == o.node_size() == managed
        e.tick(now, read=False)
        o.tick(now, read=False)
        c = compare_tick(e, o, "c5 tick %d" % t)
        assert c["heartbeat"] == managed and c["node_init"] > 0.99 * f.k and c["pod_patch"] == 0
    n = workload.BUCKETS * fl.cp
    eu, ep, eh, ei = e.dump_pods(0, n)
    ou, op, oh, oi = o.dump_pods(0, n)
    assert (eu == ou).all() and (ep == op).all() and (eh == oh).all() and (ei == oi).all()
    assert int(np.count_nonzero(eu)) == 10_000_000
    e.close()
    o.close()
