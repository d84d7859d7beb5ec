"""GPU, world_size 2 on one MI355X: two engine processes (each owning half the
buckets) exchange per-tick pool/counter data through the host allgather hook
(gloo) and must reproduce the single-rank engine and the oracle exactly.  This
covers every multi-rank code path of the engine except the RCCL transport call
itself (RCCL refuses two ranks on one GPU); the 8-GPU scaling bench runs that."""
import os
import pickle
import tempfile

import pytest
import torch.multiprocessing as mp

import dist_common as dc
from test_dist_cpu import merge

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, outdir, big=False, pair=False, foreign_from=0):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    # two engines share one GPU: each persistent tick grid must fit beside the other
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KWOK_TICK_BLOCKS_PER_CU="1")
    if os.environ.get("KWOK_TEST_TRACE"):  # a stuck rank shows where
        import faulthandler
        faulthandler.dump_traceback_later(60, exit=True)
    import torch.distributed as dist
    import dist_common as dc2
    from kwok_amd.engine import Engine
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange_puts(mine):
        objs = [None] * world
        dist.all_gather_object(objs, mine)
        return [ip for r, l in enumerate(objs) if r != rank for ip in l]

    e = dc2.make(Engine, rank, world, allgather=dc2.gloo_allgather_fn(), big=big)
    run = dc2.Runner(e, world, rank, exchange_puts)
    res = dc2.run_all(run, dc2.scenario(big=big, ticks=4 if big else 5, foreign_from=foreign_from), pair)
    with open(os.path.join(outdir, "r%d.pkl" % rank), "wb") as f:
        pickle.dump(res, f)
    e.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("big,pair,foreign_from", [(False, False, 0), (True, False, 0), (True, True, 0),
                                                   (False, False, 3), (False, True, 3)],
                         ids=["inline-lists", "long-lists", "long-lists-queued", "quiet-then-foreign",
                              "quiet-then-foreign-queued"])
def test_two_rank_engine_matches_single_and_oracle(big, pair, foreign_from):
    """queued: every step is two ticks submitted back to back, so a tick queues
    behind one whose lists are not inline (it skips on the device and is
    launched again after the host finishes the first).  quiet-then-foreign: no
    pod brings an address of its own before tick 3, so the ranks skip the Use
    checks of pods without events (every rank's foreign-IP flag travels in the
    exchange message); from tick 3 on, foreign addresses end that on every rank."""
    from kwok_amd.engine import Engine
    from oracle.oracle import Oracle
    sc = dc.scenario(big=big, ticks=4 if big else 5, foreign_from=foreign_from)
    single_o = dc.Runner(dc.make(Oracle, 0, 1, big=big))
    ref = dc.run_all(single_o, sc, pair)
    single_e = dc.Runner(dc.make(Engine, 0, 1, big=big))
    eng = dc.run_all(single_e, sc, pair)
    for t, (g, r) in enumerate(zip(eng, ref)):
        for k in ("hb", "hb_body", "inits", "pods", "deletes", "counters"):
            assert g[k] == r[k], "single-rank engine tick %d %s" % (t, k)
    single_e.b.close()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, dc.free_port(), d, big, pair, foreign_from), nprocs=2, start_method="spawn",
                           join=True)
        parts = [pickle.load(open(os.path.join(d, "r%d.pkl" % r), "rb")) for r in range(2)]
    got = merge(parts)
    for t, (g, r) in enumerate(zip(got, ref)):
        for k in ("hb", "hb_body", "inits", "pods", "deletes", "counters"):
            assert g[k] == r[k], "2-rank engine tick %d %s" % (t, k)
    if big:  # the long-list exchange really ran: > 2 x 2048 releases in one tick
        assert max(r["counters"]["release"] for r in ref) > 2 * 2048
