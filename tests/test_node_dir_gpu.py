"""GPU parity of the device node directory (ingest.hip: k_nd_prep / k_nd_apply,
by-name pod creates resolved in k_ing_apply, k_free_zombies, k_node_lookup)
against the oracle, on a geometry small enough that every edge is hit often:
4 buckets x 8 node slots for a pool of 60 names (full buckets: EFULL), names of
1 to 253 bytes (one NAME_STRIDE slot each), Deleted nodes that pods still
reference (zombies) revived by a later Added, pods naming nodes that do not
exist (placeholder entries), deletes of zombies and of unknown names, ticks
that delete pods (the zombies' frees).  After every batch: handles, statuses,
kwok_node_has of every name and kwok_node_size; after every tick: every
output.  node_controller.go:256-270 (WatchNodes routing), pod_controller.go:
301-343 (spec.nodeName)."""
import numpy as np
import pytest

from kwok_amd import abi
from kwok_amd.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

GEOM = dict(buckets=4, node_slots_per_bucket=8, pod_slots_per_bucket=64, cidr="10.0.0.1/22")


def _names(rng, n):
    out = []
    for i in range(n):
        ln = int(rng.choice([1, 7, 12, 63, 64, 65, 128, 200, 252, 253]))
        stem = ("n%d-" % i)
        body = "".join(rng.choice(list("abcdefghijklmnopqrstuvwxyz0123456789-")) for _ in range(max(0, ln - len(stem))))
        out.append((stem + body)[:ln] if ln >= len(stem) else "n%d" % i)
    return sorted(set(out))


def _node_batch(rng, names, k):
    ar = abi.Arena()
    ev = np.zeros(k, abi.NODE_EVENT_DTYPE)
    for i in range(k):
        nm = str(rng.choice(names))
        ev[i]["op"] = abi.OP_DELETE if rng.random() < 0.35 else abi.OP_UPSERT
        ev[i]["name"] = ar.ref(nm)
        ev[i]["managed"] = 1 if rng.random() < 0.8 else 0
        ev[i]["lockable"] = 1 if rng.random() < 0.9 else 0
    return ev, bytes(ar.buf)


def _pod_batch(rng, names, live, spec, now, k):
    ar = abi.Arena()
    ev = np.zeros(k, abi.POD_EVENT_DTYPE)
    keys = []
    for i in range(k):
        r = ev[i]
        r["spec_id"] = spec
        r["creation_unix"] = now - 60
        r["node_handle"] = -1
        if live and rng.random() < 0.35:
            h = int(rng.choice(sorted(live)))
            r["op"] = abi.OP_DELETE if rng.random() < 0.5 else abi.OP_UPSERT
            r["handle"] = h
            if r["op"] == abi.OP_UPSERT:  # deletion-marked (the tick deletes it)
                r["flags"] = abi.POD_DELETING | (abi.POD_HAS_FINALIZERS if rng.random() < 0.5 else 0)
                r["phase"] = abi.PHASE_PENDING
            keys.append(("old", h))
        else:
            r["op"] = abi.OP_UPSERT
            r["handle"] = -1
            r["node_name"] = ar.ref(str(rng.choice(names)))
            r["phase"] = abi.PHASE_PENDING
            r["flags"] = abi.POD_STATUS_NONEMPTY
            keys.append(("new", None))
    return ev, bytes(ar.buf), keys


def _outputs(o):
    return (list(o.heartbeat_nodes), o.heartbeat_body(0) if len(o.heartbeat_nodes) else b"", list(o.node_inits),
            list(o.pod_patches), [tuple(d) for d in o.deletes], dict(o.counters))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_node_directory_edges_engine_equals_oracle(seed):
    rng = np.random.default_rng(seed)
    names = _names(rng, 60)
    backends = [Engine(device=0, **GEOM), Oracle(**GEOM)]
    specs = [b.register_pod_spec(containers=[("c", "img")]) for b in backends]
    assert specs[0] == specs[1]
    live = set()
    now = 1704067200 + 30
    for step in range(14):
        ev, ar = _node_batch(rng, names, int(rng.integers(1, 40)))
        res = [b.ingest_nodes_raw(ev, ar) for b in backends]
        assert list(res[0][1]) == list(res[1][1]), "step %d node statuses" % step
        assert list(res[0][0]) == list(res[1][0]), "step %d node handles" % step
        assert set(res[0][1].tolist()) <= {abi.OK, abi.ENOTFOUND, abi.EFULL}
        pe, par, keys = _pod_batch(rng, names, live, specs[0], now, int(rng.integers(1, 30)))
        pres = [b.ingest_pods_raw(pe, par) for b in backends]
        assert list(pres[0][1]) == list(pres[1][1]), "step %d pod statuses" % step
        assert list(pres[0][0]) == list(pres[1][0]), "step %d pod handles" % step
        for i, ((kind, h), hh, st) in enumerate(zip(keys, pres[0][0], pres[0][1])):
            if kind == "new" and st == abi.OK:
                live.add(int(hh))
            elif kind == "old" and st == abi.OK and pe[i]["op"] == abi.OP_DELETE:
                live.discard(h)
        for nm in names:
            assert backends[0].node_has(nm) == backends[1].node_has(nm), "step %d has(%r)" % (step, nm)
        assert backends[0].node_size() == backends[1].node_size()
        outs = [b.tick(now) for b in backends]
        assert _outputs(outs[0]) == _outputs(outs[1]), "step %d tick" % step
        for h, _ in outs[0].deletes:
            live.discard(int(h))
        now += 30
    for b in backends:
        b.close()
