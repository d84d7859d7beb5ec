"""CPU, world_size 2 over gloo: two oracle shards (contiguous bucket ranges,
per-tick allgather of pool/counter data, ingest-time releases replicated)
reproduce the single-rank oracle exactly - the same sharding and exchange
protocol the engine runs over RCCL (DESIGN.md "Multi-GPU")."""
import os
import pickle
import tempfile

import pytest
import torch.multiprocessing as mp

import dist_common as dc


def _worker(rank, world, port, outdir, big=False):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import dist_common as dc2
    from oracle.oracle import Oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange_puts(mine):
        objs = [None] * world
        dist.all_gather_object(objs, mine)
        return [ip for r, l in enumerate(objs) if r != rank for ip in l]

    o = dc2.make(Oracle, rank, world, allgather=dc2.gloo_allgather_fn(), big=big)
    run = dc2.Runner(o, world, rank, exchange_puts)
    res = [dc2.summarize(run.run_tick(n, p)) for n, p in dc2.scenario(big=big, ticks=4 if big else 5)]
    with open(os.path.join(outdir, "r%d.pkl" % rank), "wb") as f:
        pickle.dump(res, f)
    o.close()
    dist.destroy_process_group()


def merge(parts):
    out = []
    for ticks in zip(*parts):
        m = dict(hb=[], inits=[], pods=[], deletes=[], hb_body=b"", counters=ticks[0]["counters"])
        for t in ticks:
            for k in ("hb", "inits", "pods", "deletes"):
                m[k] += t[k]
            m["hb_body"] = m["hb_body"] or t["hb_body"]
            assert t["counters"] == m["counters"]  # fleet counters agree on every rank
        out.append(m)
    return out


@pytest.mark.parametrize("world,big", [(2, False), (4, False), (2, True)])
def test_sharded_oracle_matches_single(world, big):
    from oracle.oracle import Oracle
    single = dc.Runner(dc.make(Oracle, 0, 1, big=big))
    ref = [dc.summarize(single.run_tick(n, p)) for n, p in dc.scenario(big=big, ticks=4 if big else 5)]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, dc.free_port(), d, big), nprocs=world, start_method="spawn", join=True)
        parts = [pickle.load(open(os.path.join(d, "r%d.pkl" % r), "rb")) for r in range(world)]
    got = merge(parts)
    assert len(got) == len(ref)
    for t, (g, r) in enumerate(zip(got, ref)):
        for k in ("hb", "hb_body", "inits", "pods", "deletes", "counters"):
            assert g[k] == r[k], "tick %d %s" % (t, k)
    assert sum(len(r["pods"]) for r in ref) > 3000 and sum(len(r["deletes"]) for r in ref) > 500


def test_eight_oracle_shards_c3_churn():
    """W = 8 oracle shards over gloo on the C3 protocol (tests/c3_common.py):
    20k nodes x 200k pods, then 20k deletes + 20k creates in one tick, so every
    shard's release list (~2.5k) is longer than the inline exchange message"""
    from c3_common import run_c3
    run_c3(8, 20_000, 20_000, "oracle")
