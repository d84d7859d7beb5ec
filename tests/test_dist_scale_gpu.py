"""GPU, world_size 2 on one MI355X at size (BASELINE configs[2], C3-shaped:
global pod-IP allocation across ranks): a fleet of 2 x 250k nodes x 10 pods
hashed into 4096 buckets, each engine process owning half the buckets and
exchanging through the host allgather hook.  The initial tick (500k node
inits, 5M Pending->Running patches with IPs) and a steady tick must give the
single-rank oracle's pod state (phases, hostIPs, and IPs in the global
canonical (bucket, slot) order), and fleet counters, exactly.
Reference: utils.go:68-98 (ipPool new / Get), pod_controller.go:377-439."""
import os
import pickle
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import dist_common as dc

pytestmark = pytest.mark.gpu

NODES_PER_RANK = 250_000


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KWOK_TICK_BLOCKS_PER_CU="1")
    import torch.distributed as dist
    import dist_common as dc2
    from kwok_amd import workload
    from kwok_amd.engine import Engine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e, fl, ph = workload.build_engine_fleet(Engine, NODES_PER_RANK, rank=rank, world=world,
                                            allgather=dc2.gloo_allgather_fn())
    out = {"counters": []}
    for t in range(2):
        r = e.tick(workload.S0 + 30 * (t + 1), read=False)
        out["counters"].append(list(r.counters))
    lo = rank * workload.BUCKETS // world
    hi = (rank + 1) * workload.BUCKETS // world
    out["first"] = lo * fl.cp
    out["dump"] = e.dump_pods(lo * fl.cp, (hi - lo) * fl.cp)
    with open(os.path.join(outdir, "r%d.pkl" % rank), "wb") as f:
        pickle.dump(out, f)
    e.close()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_two_rank_c3_initial_tick_at_size():
    from kwok_amd import workload
    from oracle.oracle import Oracle
    o, fl, ph = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=0), 2 * NODES_PER_RANK)
    ref_counters = [list(o.tick(workload.S0 + 30 * (t + 1), read=False).counters) for t in range(2)]
    assert ref_counters[0][2] == 10 * 2 * NODES_PER_RANK  # every pod patched in tick 0
    ref = o.dump_pods(0, workload.BUCKETS * fl.cp)
    o.close()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, dc.free_port(), d), nprocs=2, start_method="spawn", join=True)
        parts = [pickle.load(open(os.path.join(d, "r%d.pkl" % r), "rb")) for r in range(2)]
    for r, p in enumerate(parts):
        assert p["counters"] == ref_counters, "rank %d fleet counters" % r
        n = len(p["dump"][0])
        for k, name in enumerate(("used", "phase", "hostIP", "podIP")):
            want = ref[k][p["first"]:p["first"] + n]
            got = p["dump"][k]
            bad = np.nonzero(got != want)[0]
            assert len(bad) == 0, "rank %d %s differs at %d handles (first %d)" % (r, name, len(bad), p["first"] + bad[0])
