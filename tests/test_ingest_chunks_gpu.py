"""GPU parity of chunked pod ingest.  kwok_ingest_pods runs a batch of more than
KWOK_INGEST_CHUNK records (default 1048576) in chunks: the copy engine moves chunk
k+1's records to HBM and k_ing_prep prepares them on a second stream while chunk
k is applied, and chunk k's results go back on a third (engine.cpp ingest_chunk).  Applying the chunks one after the other
must equal applying the batch at once, since every record is applied in event
order (pod_controller.go:301-343).  Tiny chunks put chunk boundaries everywhere:
between by-name creates and the deletes that free their node entries (REC_HARD),
inside growth batches, and across the churn generator's deletes and creates,
for page-locked and pageable batches."""
import pytest

import harness
from kwok_amd.engine import Engine, host_array
from test_c4_churn_gpu import run_churn
import test_growth_gpu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chunk", ["1", "3"])
@pytest.mark.parametrize("name", harness.TRACES)
def test_golden_trace_chunked(name, chunk, monkeypatch):
    monkeypatch.setenv("KWOK_INGEST_CHUNK", chunk)
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    harness.replay(fx, e)
    e.close()


def test_growth_chunked(monkeypatch):
    monkeypatch.setenv("KWOK_INGEST_CHUNK", "97")
    test_growth_gpu.test_1000_pods_on_one_node_grow(None, monkeypatch)


@pytest.mark.parametrize("packed", [False, True], ids=["events", "packed"])
@pytest.mark.parametrize("pinned", [True, False], ids=["pinned", "pageable"])
def test_churn_chunked(pinned, packed, monkeypatch):
    """20k nodes x 200k pods, 40k deletes + 40k creates per tick in chunks of
    ~7001: batches in page-locked memory (DMA) and in pageable memory (staged),
    as kwok_pod_event and in the compact form"""
    monkeypatch.setenv("KWOK_INGEST_CHUNK", "7001")
    run_churn(20_000, 40_000, 3, alloc=host_array if pinned else None, packed=packed)


@pytest.mark.parametrize("chunk", ["1", "3"])
@pytest.mark.parametrize("name", harness.TRACES)
def test_golden_trace_packed_chunked(name, chunk, monkeypatch):
    """the golden traces with the pods in the compact form where it carries
    them (harness.ingest_pods_mixed), in tiny chunks"""
    monkeypatch.setenv("KWOK_INGEST_CHUNK", chunk)
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    harness.replay(fx, e, packed=True)
    e.close()


def test_failed_chunk_after_an_applied_one_poisons(monkeypatch):
    """A pod batch that fails after one of its chunks was applied is partly in
    the state: the engine is poisoned (every later call fails; destroy /
    recreate is the recovery).  A failure in the first chunk leaves the state
    as a one-chunk batch failing there would (kwok_engine.h)."""
    from kwok_amd import abi
    from kwok_amd.engine import KwokError
    fx = harness.load_trace("churn")
    t = fx["ticks"]
    for fail_chunk, poisoned in ((2, True), (1, False)):
        monkeypatch.setenv("KWOK_INGEST_CHUNK", "3")
        monkeypatch.setenv("KWOK_DEBUG_INGEST_FAIL_CHUNK", str(fail_chunk))
        e = Engine(harness.config_for(fx))
        monkeypatch.delenv("KWOK_DEBUG_INGEST_FAIL_CHUNK")
        specs = harness.SpecCache(e)
        e.ingest_nodes_raw(*harness.node_batch(t[0]["node_events"]))
        recs, ar = harness.pod_batch(t[0]["pod_events"], specs)
        assert len(recs) > 6
        with pytest.raises(KwokError) as ex:
            e.ingest_pods_raw(recs, ar)
        assert ex.value.code == abi.EDEVICE
        if poisoned:
            with pytest.raises(KwokError) as ex:
                e.tick(t[0]["now"])
            assert ex.value.code == abi.EDEVICE and "recreate" in str(ex.value)
        else:
            e.tick(t[0]["now"])  # nothing of the batch applied; the engine goes on
        e.close()


@pytest.mark.parametrize("chunk", ["3", "1000000"], ids=["chunked", "one-chunk"])
def test_failure_after_an_apply_pass_poisons(chunk, monkeypatch):
    """A batch that fails after its (first) chunk's apply pass ran is partly in
    the state - pod slots, node references and the pool changed - even when no
    chunk completed: the engine is poisoned, for one-chunk batches too, so that
    a caller's retry cannot apply the creates twice."""
    from kwok_amd import abi
    from kwok_amd.engine import KwokError
    fx = harness.load_trace("churn")
    t = fx["ticks"]
    monkeypatch.setenv("KWOK_INGEST_CHUNK", chunk)
    monkeypatch.setenv("KWOK_DEBUG_INGEST_FAIL_APPLY", "1")
    e = Engine(harness.config_for(fx))
    monkeypatch.delenv("KWOK_DEBUG_INGEST_FAIL_APPLY")
    specs = harness.SpecCache(e)
    e.ingest_nodes_raw(*harness.node_batch(t[0]["node_events"]))
    recs, ar = harness.pod_batch(t[0]["pod_events"], specs)
    with pytest.raises(KwokError) as ex:
        e.ingest_pods_raw(recs, ar)
    assert ex.value.code == abi.EDEVICE and "apply pass" in str(ex.value)
    with pytest.raises(KwokError) as ex:
        e.ingest_pods_raw(recs, ar)  # the retry is refused
    assert ex.value.code == abi.EDEVICE and "recreate" in str(ex.value)
    e.close()
