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
def test_engine_golden_trace_queued(name):
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    harness.replay_queued(fx, e)
    e.close()
