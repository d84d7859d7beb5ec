"""GPU parity: the HIP engine, driven through the C-ABI, reproduces the golden
traces (reference templates + tick contract) and the CPU oracle bit for bit."""
import numpy as np
import pytest

import harness
from kwok_amd import abi
from kwok_amd.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", harness.TRACES)
def test_engine_golden_trace(name):
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    harness.replay(fx, e)
    e.close()


@pytest.mark.parametrize("name", harness.TRACES)
def test_engine_golden_trace_packed(name):
    """Pods in the compact wire form (kwok_ingest_pods_packed) wherever it can
    carry them, read in place from page-locked memory when the batch is one
    chunk: same goldens"""
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    harness.replay(fx, e, packed=True)
    e.close()


@pytest.mark.parametrize("name", harness.TRACES)
def test_engine_golden_trace_via_json(name):
    """Events as Kubernetes JSON objects through the host codec
    (kwok_decode_node / kwok_decode_pod) into the HIP engine: same goldens."""
    from kwok_amd.codec import Codec
    fx = harness.load_trace(name)
    codec = Codec(manage_all_nodes=False, manage_nodes_with_annotation_selector=harness.MANAGE,
                  disregard_status_with_annotation_selector=harness.DISREGARD)
    e = Engine(harness.config_for(fx))
    harness.replay(fx, e, codec=codec)
    e.close()


@pytest.mark.parametrize("name", harness.TRACES)
def test_engine_golden_trace_queued(name):
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    harness.replay_queued(fx, e)
    e.close()


@pytest.mark.parametrize("name", harness.TRACES)
@pytest.mark.parametrize("queued", [False, True], ids=["blocking", "queued"])
def test_engine_golden_trace_heartbeat_once(name, queued):
    """KWOK_CFG_HEARTBEAT_ONCE: the tick materialises ONE heartbeat body for
    every handle (heartbeat_stride 0); handles, body, node-init / pod patches,
    deletes, counters and state are the goldens' (node_controller.go:393-401:
    the body is the same for every node)"""
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx, heartbeat_once=True))
    (harness.replay_queued if queued else harness.replay)(fx, e)
    assert e.last.heartbeat_stride == 0
    e.close()


@pytest.mark.parametrize("name", ["specs", "churn"])
def test_engine_compact_readout(name):
    """KWOK_READ_HEARTBEAT_ONCE on the engine: one heartbeat body plus the patch
    region, byte-identical patches to the full arena copy; the heartbeat epoch
    moves only when the managed set changes"""
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    epochs = []

    def check(ti, t, out):
        once = e.read_outputs(heartbeat_once=True)
        assert once.node_inits == out.node_inits and once.pod_patches == out.pod_patches, ti
        if len(out.heartbeat_nodes):
            assert once.heartbeat_body(0) == out.heartbeat_body(0)
        epochs.append((e.last.heartbeat_epoch, tuple(out.heartbeat_nodes)))

    harness.replay(fx, e, on_tick=check)
    for (e0, h0), (e1, h1) in zip(epochs, epochs[1:]):
        if e0 == e1:
            assert h0 == h1
    e.close()


def test_failed_tick_poisons_engine(monkeypatch):
    """A tick that fails on the device (here a forced heartbeat-layout mismatch,
    KWOK_DEBUG_LAYOUT_FAULT_TICK) is reported by collect, and every later call
    fails with KWOK_EDEVICE instead of running on host mirrors that no longer
    match the device (destroy / recreate is the recovery)."""
    from kwok_amd.engine import KwokError
    fx = harness.load_trace("churn")
    monkeypatch.setenv("KWOK_DEBUG_LAYOUT_FAULT_TICK", "2")
    e = Engine(harness.config_for(fx))
    monkeypatch.delenv("KWOK_DEBUG_LAYOUT_FAULT_TICK")
    specs = harness.SpecCache(e)
    t = fx["ticks"]
    recs, ar = harness.node_batch(t[0]["node_events"])
    e.ingest_nodes_raw(recs, ar)
    recs, ar = harness.pod_batch(t[0]["pod_events"], specs)
    e.ingest_pods_raw(recs, ar)
    e.tick(t[0]["now"])
    with pytest.raises(KwokError) as ex:
        e.tick(t[1]["now"])
    assert ex.value.code == abi.EDEVICE
    for call in (lambda: e.tick(t[1]["now"] + 30), lambda: e.ingest_nodes_raw(*harness.node_batch(t[0]["node_events"])),
                 lambda: e.dump_pods(0, 8)):
        with pytest.raises(KwokError) as ex:
            call()
        assert ex.value.code == abi.EDEVICE and "recreate" in str(ex.value)
    e.close()
    e = Engine(harness.config_for(fx))  # a fresh engine replays the trace
    harness.replay(fx, e)
    e.close()
