"""GPU, one rank through the multi-rank tick (KWOK_FORCE_MULTI=1): the FRONT
launch, the exchange of the per-rank message (engine.cpp exchange), the BACK
launch, and for long lists the second exchange and k_pool_apply.  The exchange
runs over RCCL - ncclCommInitRank of a one-rank communicator from kwok_comm_id,
ncclAllGather on the engine stream - or over the host allgather hook.  RCCL
refuses two ranks on one GPU, so this is how the RCCL transport code runs on
the single-GPU box (tests/test_dist_gpu.py covers two ranks over the host hook).
Every tick must equal the oracle (and so the single-rank engine) exactly."""
import ctypes as C

import pytest

import dist_common as dc

pytestmark = pytest.mark.gpu

KEYS = ("hb", "hb_body", "inits", "pods", "deletes", "counters")


def _host_gather(user, send, nbytes, recv):  # one rank: the gathered array is its own message
    C.memmove(recv, send, nbytes)
    return 0


@pytest.mark.parametrize("transport", ["rccl", "host"])
@pytest.mark.parametrize("big,pair", [(False, False), (True, True)], ids=["inline-lists", "long-lists-queued"])
def test_one_rank_multi_path_matches_oracle(monkeypatch, transport, big, pair):
    from kwok_amd import engine as keng
    from oracle.oracle import Oracle
    sc = dc.scenario(big=big, ticks=4 if big else 5)
    ref = dc.run_all(dc.Runner(dc.make(Oracle, 0, 1, big=big)), sc, pair)
    monkeypatch.setenv("KWOK_FORCE_MULTI", "1")
    if transport == "rccl":
        e = dc.make(keng.Engine, 0, 1, big=big, comm_id=keng.comm_id())
    else:
        e = dc.make(keng.Engine, 0, 1, big=big, allgather=_host_gather)
    if not pair:  # (profiled ticks are not queued)
        e.profile_enable(True)
    got = dc.run_all(dc.Runner(e), sc, pair)
    if not pair:
        ms, n = e.profile_read()
        assert n > 0 and ms["exchange"] > 0.0, "the ticks did not take the FRONT / exchange / BACK path"
    e.close()
    for t, (g, r) in enumerate(zip(got, ref)):
        for k in KEYS:
            assert g[k] == r[k], "%s one-rank multi path, tick %d %s" % (transport, t, k)
    if big:  # the long-list exchange really ran: > 2048 Uses + releases in one tick
        assert max(r["counters"]["release"] for r in ref) > 2048


@pytest.mark.parametrize("pair", [False, True], ids=["blocking", "queued"])
def test_failed_exchange_poisons_engine(monkeypatch, pair):
    """A tick whose host-side exchange fails (the second allgather of long
    lists, in kwok_tick_collect's retire) is reported as KWOK_ECOMM, a tick
    queued behind it fails with it, and every later call fails with
    KWOK_EDEVICE: the device state went on without the host."""
    from kwok_amd import abi
    from kwok_amd import engine as keng
    calls = {"long": 0}

    def gather(user, send, nbytes, recv):
        # (XMsg: alloc, n_use, n_rel, seq, foreign, counters[16], ips[XINLINE])
        if nbytes != 8 * 5 + 16 * 8 + 2048 * 4:  # not the fixed-size message: the long-list exchange
            calls["long"] += 1
            return 1
        C.memmove(recv, send, nbytes)
        return 0

    monkeypatch.setenv("KWOK_FORCE_MULTI", "1")
    e = dc.make(keng.Engine, 0, 1, big=True, allgather=gather)
    run = dc.Runner(e)
    with pytest.raises(keng.KwokError) as ex:
        for n, p in dc.scenario(big=True, ticks=4):
            run.run_tick(n, p, pair=pair)
    assert calls["long"] == 1, calls
    if pair:
        # multi rank: the second submit first finishes the previous tick on the host,
        # which fails; the submit refuses, and collect reports the failed tick
        assert ex.value.code == abi.EDEVICE and "recreate" in str(ex.value), ex.value
        with pytest.raises(keng.KwokError) as ex:
            e.tick_collect(read=False)
    assert ex.value.code == abi.ECOMM, ex.value
    for call in (lambda: e.tick(1704070000, read=False), lambda: e.dump_pods(0, 8)):
        with pytest.raises(keng.KwokError) as ex:
            call()
        assert ex.value.code == abi.EDEVICE and "recreate" in str(ex.value)
    e.close()
