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
