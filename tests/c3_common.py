"""BASELINE configs[2] (C3) at its stated shape: a fleet sharded over W ranks,
global pod-IP allocation across ranks, checked against the single-rank CPU
oracle of the whole fleet.  Used by the GPU test (W = 8 engine processes
sharing one MI355X, 1M nodes x 10M pods; RCCL refuses two ranks on one GPU,
so the exchange runs over the host allgather hook: the same FRONT / exchange
/ BACK tick as the RCCL transport) and by the CPU test (W = 8 oracle shards
over gloo, a small fleet).  Each rank owns B/W of the buckets.  Compared:
  * the initial tick (every node init, every Pending->Running patch with its
    IP in the global canonical order): fleet counters, every rank's pod state
    (phase, hostIP, podIP), its heartbeat / init / patch / delete lists and
    every pod patch's and node-init patch's bytes (64-bit digests);
  * a C4-style churn tick (10% of the pods marked for deletion, half with
    finalizers, and as many created, so every rank's release list is longer
    than the inline exchange message: the second allgather + pool apply):
    ingest handles / status / releases, counters, state, the output lists
    and every pod patch's bytes (64-bit digests);
  * a steady tick after it (counters).
Reference: utils.go:68-108 (ipPool new / Get / Put), pod_controller.go:155-202
(DeletePod), :301-343 (WatchPods routing), :377-439 (configurePod)."""
import os
import pickle
import tempfile

import numpy as np
import torch.multiprocessing as mp

import dist_common as dc

LISTS = ("heartbeat_nodes", "node_init_nodes", "pod_patch_pods", "delete_pods", "delete_has_finalizers")


def _owner(ev, cn, hs, buckets, world):
    """rank of every pod record: its pod handle's bucket, or its node's"""
    b = np.where(ev["handle"] >= 0, ev["handle"] // hs, ev["node_handle"] // cn)
    return (b.astype(np.int64) * world) // buckets


def _backend(name):
    if name == "engine":
        from kwok_amd.engine import Engine
        return Engine
    from oracle.oracle import Oracle
    return lambda cfg: Oracle(cfg, threads=1)


def _tick(e, now, d, where):
    d["c" + where] = list(e.tick(now, read=False).counters)
    return e.read_arrays(heartbeat_once=True)


def _worker(rank, world, port, d, nodes, backend):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    # engines sharing one GPU: grids small enough to be co-resident together (a
    # dirty tick's chain blocks wait for each other), two ingest threads each
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KWOK_TICK_CHAIN_BLOCKS="16",
                      KWOK_TICK_STREAMERS="16", KWOK_INGEST_THREADS="2")
    import torch.distributed as dist
    import dist_common as dc2
    from gpu_common import patch_digests
    from kwok_amd import workload
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e, fl, ph = workload.build_engine_fleet(_backend(backend), nodes // world, rank=rank, world=world,
                                            allgather=dc2.gloo_allgather_fn())
    lo, hi = rank * workload.BUCKETS // world, (rank + 1) * workload.BUCKETS // world
    out = {"first": lo * fl.cp, "pods": ph}
    a = _tick(e, workload.S0 + 30, out, "0")
    out["l0"] = {k: a[k] for k in LISTS}
    out["dig0"] = patch_digests(a["arena"], a["pod_patch_off"], a["pod_patch_len"])
    out["dig0n"] = patch_digests(a["arena"], a["node_init_off"], a["node_init_len"])
    del a
    out["dump0"] = e.dump_pods(lo * fl.cp, (hi - lo) * fl.cp)
    ev = np.load(os.path.join(d, "ev%d.npy" % rank))
    with open(os.path.join(d, "arena.bin"), "rb") as f:
        ar = f.read()
    out["ingest"] = e.ingest_pods_raw(ev, ar)
    a = _tick(e, workload.S0 + 60, out, "1")
    out["l1"] = {k: a[k] for k in LISTS}
    out["dig1"] = patch_digests(a["arena"], a["pod_patch_off"], a["pod_patch_len"])
    out["dump1"] = e.dump_pods(lo * fl.cp, (hi - lo) * fl.cp)
    out["c2"] = list(e.tick(workload.S0 + 90, read=False).counters)
    with open(os.path.join(d, "r%d.pkl" % rank), "wb") as f:
        pickle.dump(out, f)
    e.close()
    dist.destroy_process_group()


def run_c3(world, nodes, churn, backend):
    from gpu_common import patch_digests
    from kwok_amd import workload
    from oracle.oracle import Oracle
    o, fl, ph = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=0), nodes)
    n_slots = workload.BUCKETS * fl.cp
    ref = {}
    A = _tick(o, workload.S0 + 30, ref, "0")
    ref["l0"] = {k: A[k] for k in LISTS}
    ref["dig0"] = patch_digests(A["arena"], A["pod_patch_off"], A["pod_patch_len"])
    ref["dig0n"] = patch_digests(A["arena"], A["node_init_off"], A["node_init_len"])
    del A
    ref["dump0"] = o.dump_pods(0, n_slots)
    assert ref["c0"][2] == 10 * nodes  # every pod patched in the initial tick
    ch = workload.Churn(ph, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_slots, churn, seed=3)
    ev, ar = ch.batch(lambda: o.dump_pods(0, n_slots), workload.S0 + 60)
    own = _owner(ev, fl.cn, fl.cp, workload.BUCKETS, world)
    ref["ingest"] = o.ingest_pods_raw(ev, ar)
    A = _tick(o, workload.S0 + 60, ref, "1")
    ref["l1"] = {k: A[k] for k in LISTS}
    ref["dig1"] = patch_digests(A["arena"], A["pod_patch_off"], A["pod_patch_len"])
    ref["dump1"] = o.dump_pods(0, n_slots)
    ref["c2"] = list(o.tick(workload.S0 + 90, read=False).counters)
    o.close()
    c1 = [ref["c1"][k] for k in (3, 5, 2, 4)]  # delete, release, pod_patch, alloc
    assert c1 == [churn] * 4, c1
    # every rank releases more than the inline exchange message holds (XINLINE = 2048 IPs)
    assert churn // world > 2048 or nodes < 100_000
    with tempfile.TemporaryDirectory() as d:
        for r in range(world):
            np.save(os.path.join(d, "ev%d.npy" % r), ev[own == r])
        with open(os.path.join(d, "arena.bin"), "wb") as f:
            f.write(ar)
        mp.start_processes(_worker, args=(world, dc.free_port(), d, nodes, backend), nprocs=world,
                           start_method="spawn", join=True)
        parts = [pickle.load(open(os.path.join(d, "r%d.pkl" % r), "rb")) for r in range(world)]
    # every pod of the fleet lives on exactly one rank, under the oracle's handle
    assert np.array_equal(np.sort(np.concatenate([p["pods"] for p in parts])), np.sort(ph))
    for r, p in enumerate(parts):
        for c in ("c0", "c1", "c2"):
            assert p[c] == ref[c], "rank %d fleet counters %s" % (r, c)
        n = len(p["dump0"][0])
        lo_h, hi_h = p["first"], p["first"] + n
        lo_n, hi_n = lo_h // fl.cp * fl.cn, hi_h // fl.cp * fl.cn
        for tick in ("0", "1"):
            for k, name in enumerate(("used", "phase", "hostIP", "podIP")):
                want = ref["dump" + tick][k][lo_h:hi_h]
                bad = np.nonzero(p["dump" + tick][k] != want)[0]
                assert len(bad) == 0, "rank %d tick %s %s differs at %d handles (first %d)" % (
                    r, tick, name, len(bad), lo_h + bad[0])
            R = ref["l" + tick]
            for k in LISTS:
                rv = R["delete_pods" if k == "delete_has_finalizers" else k]
                sel = (rv >= lo_n) & (rv < hi_n) if k in LISTS[:2] else (rv >= lo_h) & (rv < hi_h)
                assert np.array_equal(p["l" + tick][k], R[k][sel]), "rank %d tick %s %s" % (r, tick, k)
        pp = ref["l1"]["pod_patch_pods"]
        assert np.array_equal(p["dig1"], ref["dig1"][(pp >= lo_h) & (pp < hi_h)]), "rank %d churn patch bytes" % r
        # the initial tick's bytes too: every Pending->Running patch (its IP in the
        # global order) and every node-init patch of the rank
        pp0, ni0 = ref["l0"]["pod_patch_pods"], ref["l0"]["node_init_nodes"]
        assert np.array_equal(p["dig0"], ref["dig0"][(pp0 >= lo_h) & (pp0 < hi_h)]), "rank %d initial patch bytes" % r
        assert np.array_equal(p["dig0n"], ref["dig0n"][(ni0 >= lo_n) & (ni0 < hi_n)]), "rank %d node-init bytes" % r
        mine = np.nonzero(own == r)[0]  # the rank's ingest results are the oracle's for its records
        for k in range(3):
            assert np.array_equal(p["ingest"][k], ref["ingest"][k][mine]), "rank %d ingest output %d" % (r, k)
    return ref
