#!/usr/bin/env python3
"""Debug the first engine / oracle difference of tests/test_node_dir_gpu.py (seed argv[1])."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import test_node_dir_gpu as T  # noqa: E402
from kwok_amd import abi  # noqa: E402
from kwok_amd.engine import Engine  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 2
rng = np.random.default_rng(seed)
names = T._names(rng, 60)
B = [Engine(device=0, **T.GEOM), Oracle(**T.GEOM)]
spec = [b.register_pod_spec(containers=[("c", "img")]) for b in B][0]
live = set()
now = 1704067200 + 30
bucket = lambda nm: T.abi.fnv1a32(nm.encode()) & 3 if hasattr(T.abi, "fnv1a32") else None  # noqa: E731
for step in range(14):
    ev, ar = T._node_batch(rng, names, int(rng.integers(1, 40)))
    res = [b.ingest_nodes_raw(ev, ar) for b in B]
    print("step", step, "nodes", len(ev), "equal", list(res[0][0]) == list(res[1][0]) and list(res[0][1]) == list(res[1][1]))
    pe, par, keys = T._pod_batch(rng, names, live, spec, now, int(rng.integers(1, 30)))
    pres = [b.ingest_pods_raw(pe, par) for b in B]
    if list(pres[0][0]) != list(pres[1][0]) or list(pres[0][1]) != list(pres[1][1]):
        print("pod batch differs at step", step)
        for i in range(len(pe)):
            r = pe[i]
            nm = bytes(par[r["node_name"]["off"]:r["node_name"]["off"] + r["node_name"]["len"]]).decode() if r["node_name"]["len"] else ""
            print("  %2d op %d handle %5d name %-12s len %3d | engine %5d st %d | oracle %5d st %d %s" % (
                i, r["op"], r["handle"], nm[:12], len(nm), pres[0][0][i], pres[0][1][i], pres[1][0][i], pres[1][1][i],
                "<<" if pres[0][0][i] != pres[1][0][i] else ""))
        for bk in range(4):
            u = [b.dump_pods(bk * 64, 64)[0] for b in B]
            print("  bucket", bk, "used engine", "".join(str(int(x)) for x in u[0]))
            print("  bucket", bk, "used oracle", "".join(str(int(x)) for x in u[1]))
        break
    for i, ((kind, h), hh, st) in enumerate(zip(keys, pres[0][0], pres[0][1])):
        if kind == "new" and st == abi.OK:
            live.add(int(hh))
        elif kind == "old" and st == abi.OK and pe[i]["op"] == abi.OP_DELETE:
            live.discard(h)
    outs = [b.tick(now) for b in B]
    print("   tick equal", T._outputs(outs[0]) == T._outputs(outs[1]), "deletes", len(outs[0].deletes))
    for h, _ in outs[0].deletes:
        live.discard(int(h))
    now += 30
