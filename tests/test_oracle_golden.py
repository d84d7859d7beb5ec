"""CPU: pin the oracle against the golden fixtures (which execute the
reference's own templates; see tests/golden/make_golden.py)."""
import json
import os

import pytest

import gotmpl_path  # noqa: F401  (adds tests/golden to sys.path)
import gotmpl
import harness
from oracle.oracle import Oracle

GOLDEN = harness.GOLDEN


def test_renderer_known_answers():
    # renderer_test.go:32-67 replayed through the fixture generator's interpreter
    for c in json.load(open(os.path.join(GOLDEN, "renderer_kat.json"))):
        fns = {k: (lambda v=v: v) for k, v in c["funcs"].items()}
        assert gotmpl.render_to_json(c["tmpl"], c["data"], fns) == c["expected"], c["name"]


@pytest.mark.parametrize("name", harness.TRACES)
def test_oracle_trace(name):
    fx = harness.load_trace(name)
    o = Oracle(harness.config_for(fx))
    harness.replay(fx, o)


def _oracle_one(cfg_kw, node_events, pod_events, now):
    o = Oracle(**cfg_kw)
    if node_events:
        recs, ar = harness.node_batch(node_events)
        o.ingest_nodes_raw(recs, ar)
    specs = harness.SpecCache(o)
    if pod_events:
        recs, ar = harness.pod_batch(pod_events, specs)
        o.ingest_pods_raw(recs, ar)
    return o.tick(now)


def test_render_cases():
    """Every render case (heartbeat, node init variants, pod variants) through
    the oracle equals the reference-template rendering byte for byte."""
    cases = json.load(open(os.path.join(GOLDEN, "render_cases.json")))
    for c in cases:
        kw = dict(node_ip=c["node_ip"], buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8)
        if c["kind"] == "heartbeat":
            out = _oracle_one(dict(kw, start_time=c["start"]), [dict(op="upsert", name="node-0000000", managed=True,
                              lockable=False, phase="Running")], [], c["now"])
            assert out.heartbeat_body(0).decode() == c["expected"]
        elif c["kind"] == "node_init":
            ev = dict(c["node"], op="upsert")
            out = _oracle_one(dict(kw, start_time=c["start"]), [ev], [], c["now"])
            assert out.node_inits[0][1].decode() == c["expected"], c["label"]
        else:
            p = dict(c["pod"], op="upsert", handle=-1)
            if c["alloc"]:
                # make the pool hand out exactly c["alloc"] as its first fresh address
                kw["cidr"] = c["alloc"] + "/32"
            nodes = [dict(op="upsert", name=p["node"], managed=True, lockable=False, phase="Running")]
            out = _oracle_one(kw, nodes, [p], 1704067230)
            assert out.pod_patches[0][1].decode() == c["expected"], c["label"]


def test_ippool_cases():
    """ipPool op sequences (utils.go:52-117) incl. the doc known answer
    (10 pods -> 10.0.0.1..10.0.0.10, kwok-manage-nodes-and-pods.md:125-134)."""
    cases = json.load(open(os.path.join(GOLDEN, "ippool_cases.json")))
    assert cases[0]["results"] == ["10.0.0.%d" % i for i in range(1, 11)]
    for c in cases:
        # drive the oracle pool through pods: every 'get' is a Pending pod, 'put'
        # an external Deleted event of a pod holding the IP, 'use' a pod carrying it
        o = Oracle(cidr=c["cidr"], buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=1024)
        specs = harness.SpecCache(o)
        recs, ar = harness.node_batch([dict(op="upsert", name="n", managed=True, lockable=False, phase="Running")])
        o.ingest_nodes_raw(recs, ar)
        now = 1704067230
        got = []
        for op, want in zip(c["ops"], c["results"]):
            if op == "get":
                ev = dict(op="upsert", key="p", node="n", phase="Pending", status_nonempty=True, creation=0,
                          spec={"containers": [["c", "i"]]})
                recs, ar = harness.pod_batch([ev], specs)
                o.ingest_pods_raw(recs, ar)
                out = o.tick(now)
                now += 30
                pp = out.pod_patches[-1][1].decode()
                ip = json.loads(pp)["status"]["podIP"]
                got.append(ip)
            else:
                kind, ip = op.split(":")
                if kind == "put":
                    ev = dict(op="upsert", key="x", node="n", phase="Running", status_nonempty=True, conforms=True,
                              creation=0, hostIP="1.1.1.1", podIP=ip, spec={"containers": [["c", "i"]]})
                    recs, ar = harness.pod_batch([ev], specs)
                    hs, _, _ = o.ingest_pods_raw(recs, ar)
                    ev.update(op="delete", handle=int(hs[0]))
                    recs, ar = harness.pod_batch([ev], specs)
                    o.ingest_pods_raw(recs, ar)
                else:
                    ev = dict(op="upsert", key="u", node="n", phase="Running", status_nonempty=True, conforms=True,
                              creation=0, hostIP="1.1.1.1", podIP=ip, spec={"containers": [["c", "i"]]})
                    recs, ar = harness.pod_batch([ev], specs)
                    o.ingest_pods_raw(recs, ar)
                    o.tick(now)  # evaluation performs ipPool.Use
                    now += 30
                got.append(None)
        assert got == c["results"], c


@pytest.mark.parametrize("name", harness.TRACES)
def test_oracle_threads_golden(name):
    """the OpenMP sweeps (the all-core CPU baseline) reproduce the goldens too"""
    fx = harness.load_trace(name)
    o = Oracle(harness.config_for(fx), threads=8)
    harness.replay(fx, o)


def test_oracle_threads_match_sequential_at_scale():
    """8 threads vs 1 thread on a churning fleet (deletions with and without
    finalizers, IP release and reuse, new pods): identical outputs and state"""
    import numpy as np
    from kwok_amd import abi, workload
    outs = []
    for th in (1, 8):
        o, fl, ph = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=th), 3000, buckets=256)
        assert o.threads == th
        rng = np.random.default_rng(5)
        seq = []
        for t in range(3):
            if t:
                used, phase, hip, pip = o.dump_pods(0, 256 * fl.cp)
                idx = np.nonzero(used)[0]
                dl = np.sort(rng.choice(idx, 500, replace=False)).astype(np.int32)
                ar = abi.Arena()
                ev = np.zeros(len(dl), abi.POD_EVENT_DTYPE)
                ev["op"] = abi.OP_UPSERT
                ev["handle"] = dl
                ev["phase"] = abi.PHASE_RUNNING
                ev["creation_unix"] = workload.S0 - 60
                ev["flags"] = (abi.POD_DELETING | abi.POD_STATUS_NONEMPTY | abi.POD_CONFORMS |
                               np.where(np.arange(len(dl)) % 2, abi.POD_HAS_FINALIZERS, 0))
                for i, h in enumerate(dl):
                    ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(pip[h])))
                    ev[i]["host_ip"] = ar.ref(abi.ip4s(int(hip[h])))
                _, st, _ = o.ingest_pods_raw(ev, bytes(ar.buf))
                assert (st == 0).all()
                names = fl.names[rng.choice(len(fl.names), 700)]
                new = np.zeros(len(names), abi.POD_EVENT_DTYPE)
                new["op"] = abi.OP_UPSERT
                new["handle"] = -1
                new["node_handle"] = -1
                new["phase"] = abi.PHASE_PENDING
                new["flags"] = abi.POD_STATUS_NONEMPTY
                new["creation_unix"] = workload.S0 + t
                new["node_name"]["off"] = np.arange(len(names), dtype=np.uint32) * 12
                new["node_name"]["len"] = 12
                _, st, _ = o.ingest_pods_raw(new, names.tobytes())
                assert (st == 0).all()
            out = o.tick(workload.S0 + 30 * (t + 1))
            seq.append((list(out.heartbeat_nodes), out.node_inits, out.pod_patches, out.deletes, out.counters))
        assert seq[1][3] and seq[1][2]  # deletes and new pods' patches happened
        seq.append(o.dump_pods(0, 256 * fl.cp))
        outs.append(seq)
        o.close()
    a, b = outs
    for x, y in zip(a[:-1], b[:-1]):
        assert x == y
    for x, y in zip(a[-1], b[-1]):
        assert (x == y).all()
