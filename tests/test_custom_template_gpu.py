"""GPU: custom pod status templates (Config.PodStatusTemplate, controller.go:76;
SURVEY §8(f) rank 3).  The engine compiles the template per registered pod
spec into the kernels' A | hostIP | B | podIP | C program; every pod patch
k_emit writes must equal tests/golden/gotmpl.py's rendering of the template
(an independent Go text/template + yaml.v2 -> encoding/json interpreter) over
the pod, and the host assembly of the program (kwok_pod_template_patch).
Custom node-initialization and heartbeat bodies are likewise compared with
gotmpl.py's rendering of the templates (node_controller.go:101 appends the
heartbeat template to the node template).  Who is patched, IP allocation,
deletes and counters do not depend on the template: they must equal the
oracle's (default template) on the same events."""
import ipaddress
import json

import numpy as np
import pytest

from gpu_common import compare_state, new_pods
from kwok_amd import abi, engine
from kwok_amd.engine import Engine, make_config
from oracle.oracle import Oracle
import gotmpl_path  # noqa: F401
import gotmpl
from test_template_cpu import NODE_IP, START, expected_patch, node_doc, rfc3339, tpl


def gotmpl_node(text, hb_text, n, now):
    """configureNode's patch body, rendered by gotmpl.py (node_controller.go:101, :356-391)"""
    funcs = {"NodeIP": lambda: NODE_IP, "Now": lambda: rfc3339(now), "StartTime": lambda: rfc3339(START)}
    return ('{"status":%s}' % gotmpl.render_to_json(text + "\n" + hb_text, node_doc(n), funcs)).encode()


def gotmpl_heartbeat(text, now):
    funcs = {"NodeIP": lambda: NODE_IP, "Now": lambda: rfc3339(now), "StartTime": lambda: rfc3339(START)}
    return ('{"status":%s}' % gotmpl.render_to_json(text, {"metadata": {}, "spec": {}, "status": {}}, funcs)).encode()

pytestmark = pytest.mark.gpu

SPECS = [([("fake-pod", "fake")], [], []),
         ([("a", "img-a"), ("b", "img/b:v2")], [("init", "busybox")], ["g.io/x"]),
         ([], [("i0", "registry.k8s.io/pause:3.9"), ("i1", "busybox:1.36")], ["g.io/a", "g.io/b"])]


@pytest.mark.parametrize("name", ["pod_a.tpl", "pod_b.tpl", "pod_c.tpl"])
def test_custom_pod_template_engine(name):
    text = tpl(name)
    kw = dict(cidr="10.0.0.1/16", node_ip="196.168.0.1", buckets=256, node_slots_per_bucket=16,
              pod_slots_per_bucket=256)
    e = Engine(make_config(pod_status_template=text, **kw))
    o = Oracle(make_config(**kw))
    spec = [e.register_pod_spec(*s) for s in SPECS]
    assert spec == [o.register_pod_spec(*s) for s in SPECS]
    rng = np.random.default_rng(5)
    ar = abi.Arena()
    names = ["node-%04d" % i for i in range(300)]
    ev = np.zeros(len(names), abi.NODE_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["managed"] = 1
    ev["lockable"] = 1
    for i, n in enumerate(names):
        ev[i]["name"] = ar.ref(n)
    nh, st = e.ingest_nodes_raw(ev, bytes(ar.buf))
    assert (o.ingest_nodes_raw(ev, bytes(ar.buf))[0] == nh).all()
    n_slots = 256 * 256
    meta = {}  # handle -> (spec index, creation, original hostIP, status non-empty)
    now = 1704067230
    for t in range(3):
        pods, par = new_pods(rng, nh, 900, spec, host_ips=("10.9.8.7", "172.16.0.1"), host_ip_frac=0.3,
                             years=40)
        pods["flags"] &= np.uint8(0xFF & ~abi.POD_DISREGARD)
        h1, s1, _ = e.ingest_pods_raw(pods, par)
        h2, s2, _ = o.ingest_pods_raw(pods, par)
        assert (h1 == h2).all() and (s1 == s2).all()
        for i, h in enumerate(h1):
            hip = 0
            if pods[i]["host_ip"]["len"]:
                off = int(pods[i]["host_ip"]["off"])
                hip = int(ipaddress.IPv4Address(par[off:off + int(pods[i]["host_ip"]["len"])].decode()))
            meta[int(h)] = (spec.index(int(pods[i]["spec_id"])), int(pods[i]["creation_unix"]), hip,
                            bool(pods[i]["flags"] & abi.POD_STATUS_NONEMPTY))
        if t:  # deletions: IP release and reuse in the same tick
            live = np.array(sorted(meta), np.int32)
            dead = rng.choice(live, 200, replace=False)
            d = np.zeros(len(dead), abi.POD_EVENT_DTYPE)
            d["op"] = abi.OP_DELETE
            d["handle"] = dead
            assert (e.ingest_pods_raw(d, b"")[1] == o.ingest_pods_raw(d, b"")[1]).all()
            for h in dead:
                meta.pop(int(h))
        E, O = e.tick(now), o.tick(now)
        now += 30
        assert E.counters == O.counters, t
        assert [h for h, _ in E.pod_patches] == [h for h, _ in O.pod_patches], t
        assert E.deletes == O.deletes and list(E.heartbeat_nodes) == list(O.heartbeat_nodes)
        compare_state(e, o, n_slots, "custom template tick %d" % t)
        used, phase, hips, pips = e.dump_pods(0, n_slots)
        for k, (h, got) in enumerate(E.pod_patches):
            si, ct, hip, ne = meta[h]
            cs, ics, gates = SPECS[si]
            want = engine.pod_template_patch(text, cs, ics, gates, 1704067200, "196.168.0.1", ct, hip,
                                             int(pips[h]), ne)
            assert got == want, "tick %d pod %d" % (t, h)
            assert got == expected_patch(text, cs, ics, gates, ct, hip, int(pips[h]), ne), "gotmpl: tick %d pod %d" % (t, h)
        for h, _ in E.pod_patches:  # applied: the status is no longer empty
            si, ct, hip, _ = meta[h]
            meta[h] = (si, ct, hip, True)
    e.close()
    o.close()


def test_custom_template_rejected_at_create():
    with pytest.raises(engine.KwokError):
        Engine(make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8,
                           pod_status_template="conditions: []\nstartTime: {{ Now }}\n"))


def test_custom_node_init_template_engine():
    """node_a.tpl for the init patches (compiled per distinct node status into
    the node's blob; the heartbeat conditions spliced in by k_emit)"""
    from test_template_cpu import NODES, node_record
    text = tpl("node_a.tpl")
    kw = dict(cidr="10.0.0.1/16", node_ip="196.168.0.1", buckets=64, node_slots_per_bucket=16,
              pod_slots_per_bucket=64)
    e = Engine(make_config(node_init_template=text, pod_status_template=tpl("pod_b.tpl"), **kw))
    o = Oracle(make_config(**kw))
    recs = {}
    for i in range(300):
        ev, ar = node_record(NODES[i % len(NODES)], "node-%04d" % i)
        h1, s1 = e.ingest_nodes_raw(ev, ar)
        h2, s2 = o.ingest_nodes_raw(ev, ar)
        assert s1[0] == 0 and h1[0] == h2[0]
        recs[int(h1[0])] = (ev, ar, i % len(NODES))
    now = 1704067230
    for t in range(2):
        E, O = e.tick(now), o.tick(now)
        assert list(E.heartbeat_nodes) == list(O.heartbeat_nodes)
        assert E.heartbeat_body(0) == O.heartbeat_body(0)
        if t == 0:
            assert sorted(h for h, _ in E.node_inits) == sorted(recs)  # every node is initialised once
        else:
            assert E.node_inits == []  # the engine applied its patches: the nodes conform now
        # the default heartbeat's conditions as a template of our own (the oracle's body
        # with its Now / StartTime values as the funcs): node_controller.go:101 appends
        # the heartbeat template to the node template
        conds = json.dumps(json.loads(O.heartbeat_body(0))["status"]["conditions"], separators=(",", ":"))
        hb_tpl = "conditions: " + conds.replace(rfc3339(now), "{{ Now }}").replace(rfc3339(START), "{{ StartTime }}")
        want = {k: gotmpl_node(text, hb_tpl, n, now) for k, n in enumerate(NODES)}
        for h, got in E.node_inits:
            ev, ar, k = recs[h]
            assert got == engine.node_template_patch(text, ev[0], ar, 1704067200, "196.168.0.1", now), h
            assert got == want[k], "gotmpl: node %d" % h
        now += 30
    e.close()
    o.close()


@pytest.mark.parametrize("hb", ["heartbeat_a.tpl", "heartbeat_b.tpl"])
def test_custom_heartbeat_template_engine(hb):
    """a custom heartbeat (1254 B: 79 units per slot, near the 80-unit limit; and
    a short 165 B one): the stream writes the compiled body for every managed
    node through the general group walk, node inits splice its conditions"""
    from test_template_cpu import NODES, node_record
    htext, ntext = tpl(hb), tpl("node_a.tpl")
    kw = dict(cidr="10.0.0.1/16", node_ip="196.168.0.1", buckets=256, node_slots_per_bucket=64,
              pod_slots_per_bucket=64)
    e = Engine(make_config(node_heartbeat_template=htext, node_init_template=ntext, **kw))
    o = Oracle(make_config(**kw))
    recs = {}
    for i in range(5003):  # not a multiple of the 4-slot stream group
        ev, ar = node_record(NODES[i % len(NODES)], "node-%05d" % i)
        h1, s1 = e.ingest_nodes_raw(ev, ar)
        h2, _ = o.ingest_nodes_raw(ev, ar)
        assert s1[0] == 0 and h1[0] == h2[0]
        recs[int(h1[0])] = (ev, ar, i % len(NODES))
    now = 1704067230
    for t in range(3):
        E, O = e.tick(now), o.tick(now)
        assert list(E.heartbeat_nodes) == list(O.heartbeat_nodes)
        body = engine.heartbeat_template_patch(htext, 1704067200, "196.168.0.1", now)
        assert body == gotmpl_heartbeat(htext, now)
        want = {k: gotmpl_node(ntext, htext, n, now) for k, n in enumerate(NODES)}
        n = len(E.heartbeat_nodes)
        assert E.heartbeat_len == len(body) and E.heartbeat_stride == (len(body) + 15) // 16 * 16
        a = np.frombuffer(E.arena, np.uint8)[E.heartbeat_off:E.heartbeat_off + n * E.heartbeat_stride]
        a = a.reshape(n, E.heartbeat_stride)[:, :E.heartbeat_len]
        assert (a == np.frombuffer(body, np.uint8)[None, :]).all(), "tick %d heartbeat bodies" % t
        assert len(E.node_inits) == (len(recs) if t == 0 else 0)
        for h, got in E.node_inits:
            ev, ar, k = recs[h]
            assert got == engine.node_template_patch(ntext, ev[0], ar, 1704067200, "196.168.0.1", now,
                                                     heartbeat_tpl=htext), h
            assert got == want[k], "gotmpl: node %d" % h
        out = e.read_outputs(heartbeat_once=True)  # the compact hand-off carries one body
        assert out.heartbeat_body(0) == body
        now += 30
    e.close()
    o.close()
