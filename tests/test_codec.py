"""CPU: the host watch-event codec (kwok_decode_node / kwok_decode_pod,
kwok_amd/csrc/codec.cpp) against the golden traces and the reference's tests.

- every node / pod event of every golden trace, written as the Kubernetes JSON
  object a watch would carry (whitespace and key order scrambled), decodes to
  exactly the record fields the trace feeds the engine;
- the apiserver echo: every init / pod patch a golden trace expects, applied
  to its object, decodes to a node / pod the reference's LockNode /
  computePatchData would leave alone (conforms, Running, the patched IPs), and
  the echoed node blobs come back byte-identical to the patch's JSON;
- label-selector semantics of k8s.io/apimachinery labels.Parse / Matches
  (equality, set, existence terms) and the reference tests' selectors
  (pod_controller_test.go:76,129-131: DisregardStatusWithAnnotationSelector "fake=custom").
"""
import glob
import json
import os
import random

import pytest

from kwok_amd import abi
from kwok_amd.codec import Codec, selector_matches
from kwok_amd.engine import KwokError
from harness import MANAGE, DISREGARD, node_doc, pod_doc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TRACES = sorted(glob.glob(os.path.join(GOLDEN, "trace_*.json")))


def scramble(obj, rng):
    """Same JSON value, different bytes: shuffled keys and random indentation."""
    def shuf(v):
        if isinstance(v, dict):
            items = list(v.items())
            rng.shuffle(items)
            return {k: shuf(x) for k, x in items}
        if isinstance(v, list):
            return [shuf(x) for x in v]
        return v
    return json.dumps(shuf(obj), indent=rng.choice([None, 1, 2])).encode()


def expected_pod_flags(ev):
    return ((abi.POD_DISREGARD if ev["disregard"] else 0) | (abi.POD_DELETING if ev["deleting"] else 0) |
            (abi.POD_STATUS_NONEMPTY if (ev["status_nonempty"] or ev["phase"] or ev["hostIP"] or ev["podIP"]) else 0) |
            (abi.POD_CONFORMS if ev["conforms"] else 0) | (abi.POD_HAS_FINALIZERS if ev["finalizers"] else 0))


def check_pod(b, i, ev):
    d = b.pods[i]
    assert b.status[i] == 0
    assert b.text(d.name) == ev["key"]
    assert d.ev.op == abi.OP_UPSERT and d.ev.handle == -1 and d.ev.spec_id == -1
    assert d.ev.phase == abi.POD_PHASES[ev["phase"]]
    assert d.ev.flags == expected_pod_flags(ev), (ev, d.ev.flags)
    assert d.ev.creation_unix == ev["creation"]
    assert b.text(d.ev.node_name) == ev["node"]
    assert b.text(d.ev.host_ip) == ev["hostIP"] and b.text(d.ev.pod_ip) == ev["podIP"]
    spec = ev["spec"]
    assert [(b.text(c.name), b.text(c.image)) for c in d.containers[:d.n_containers]] == [tuple(x) for x in spec["containers"]]
    assert [(b.text(c.name), b.text(c.image)) for c in d.init_containers[:d.n_init_containers]] == [tuple(x) for x in spec["init"]]
    assert [b.text(g) for g in d.readiness_gates[:d.n_readiness_gates]] == list(spec["gates"])


def cjson(v):
    """json.Marshal of the YAML round-tripped value: compact, keys sorted."""
    return json.dumps(v, separators=(",", ":"), sort_keys=True) if v else ""


def check_node(b, i, ev):
    n = b.nodes[i]
    assert b.status[i] == 0
    assert b.text(n.name) == ev["name"]
    assert (n.managed, n.lockable) == (int(ev["managed"]), int(ev["lockable"]))
    assert n.phase == {"": abi.PHASE_NONE, "Running": abi.PHASE_RUNNING}.get(ev["phase"], abi.PHASE_OTHER)
    for k in ("addresses", "allocatable", "capacity"):
        assert b.text(getattr(n, k)) == cjson(ev[k]), k  # canonical bytes, whatever the source layout
    for j, k in enumerate(abi.NODEINFO_KEYS):
        assert b.text(n.node_info[j]) == ev["nodeInfo"].get(k, "")


@pytest.mark.parametrize("path", TRACES, ids=lambda p: os.path.basename(p)[6:-5])
def test_golden_events_roundtrip_through_json(path):
    fx = json.load(open(path))
    rng = random.Random(7)
    codec = Codec(manage_all_nodes=False, manage_nodes_with_annotation_selector=MANAGE,
                  disregard_status_with_annotation_selector=DISREGARD)
    pods = [e for t in fx["ticks"] for e in t.get("pod_events", []) if e["op"] == "upsert"]
    nodes = [e for t in fx["ticks"] for e in t.get("node_events", []) if e["op"] == "upsert"]
    b = codec.decode_pods([scramble(pod_doc(e), rng) for e in pods])
    for i, e in enumerate(pods):
        check_pod(b, i, e)
    b = codec.decode_nodes([scramble(node_doc(e), rng) for e in nodes])
    for i, e in enumerate(nodes):
        check_node(b, i, e)


@pytest.mark.parametrize("path", TRACES, ids=lambda p: os.path.basename(p)[6:-5])
def test_apiserver_echo_of_expected_patches_conforms(path):
    """Apply each expected patch to its object (as the apiserver would) and
    decode it again: the reference's no-op tests must now hold."""
    fx = json.load(open(path))
    codec = Codec(manage_all_nodes=True)
    pod_by_handle, node_by_handle = {}, {}
    pod_docs, pod_evs, node_docs, want_nodes = [], [], [], []
    for t in fx["ticks"]:
        for e in t.get("node_events", []):
            if e["op"] == "upsert":
                node_by_handle[e["expect_handle"]] = e
        for e in t.get("pod_events", []):
            if e["op"] == "upsert":
                pod_by_handle[e["expect_handle"] if e["handle"] == -1 else e["handle"]] = e
        for h, patch in t["expect"].get("pod_patches", []):
            ev = pod_by_handle[h]
            doc = pod_doc(ev)
            doc["status"].update(json.loads(patch)["status"])  # merge of the top-level status keys
            pod_docs.append(json.dumps(doc, indent=1).encode())
            pod_evs.append((ev, json.loads(patch)["status"]))
        for h, patch in t["expect"].get("node_inits", []):
            doc = node_doc(node_by_handle[h])
            doc["status"].update(json.loads(patch)["status"])
            node_docs.append(json.dumps(doc, indent=2).encode())
            want_nodes.append(patch.encode())
    if not pod_docs and not node_docs:
        pytest.skip("trace emits no patches")
    b = codec.decode_pods(pod_docs)
    for i, (ev, st) in enumerate(pod_evs):
        d = b.pods[i].ev
        assert d.flags & abi.POD_CONFORMS, (ev["key"], st)
        assert d.phase == abi.PHASE_RUNNING
        assert b.text(d.pod_ip) == st.get("podIP", ev["podIP"])
        assert b.text(d.host_ip) == st.get("hostIP", ev["hostIP"])
    b = codec.decode_nodes(node_docs)
    for i, patch in enumerate(want_nodes):
        n = b.nodes[i]
        assert n.phase == abi.PHASE_RUNNING
        for k in ("addresses", "allocatable", "capacity"):  # the echo is byte-identical
            frag = b'"%s":%s' % (k.encode(), b.text(getattr(n, k)).encode())
            assert frag in patch, k
        st = json.loads(patch)["status"]["nodeInfo"]
        for j, k in enumerate(abi.NODEINFO_KEYS):
            assert b.text(n.node_info[j]) == st[k]


SELECTOR_CASES = [
    ("fake=custom", {"fake": "custom"}, True), ("fake=custom", {"fake": "x"}, False),
    ("fake=custom", {}, False), ("fake==custom", {"fake": "custom", "a": "b"}, True),
    ("fake!=custom", {}, True), ("fake!=custom", {"fake": "custom"}, False), ("fake!=custom", {"fake": "y"}, True),
    ("fake", {"fake": ""}, True), ("fake", {"x": "y"}, False), ("!fake", {}, True), ("!fake", {"fake": "1"}, False),
    ("env in (prod, dev)", {"env": "dev"}, True), ("env in (prod,dev)", {"env": "qa"}, False),
    ("env in (prod)", {}, False), ("env notin (prod,dev)", {}, True), ("env notin (prod,dev)", {"env": "prod"}, False),
    ("a=1,b=2", {"a": "1", "b": "2"}, True), ("a=1, b=2", {"a": "1"}, False),
    ("kwok.x-k8s.io/node=fake", {"kwok.x-k8s.io/node": "fake"}, True),
    ("", {"a": "b"}, False),  # labelsParse("") = nil selector (utils.go:205-210): disregard never applies
]


@pytest.mark.parametrize("sel,labels,want", SELECTOR_CASES)
def test_selector_semantics(sel, labels, want):
    assert selector_matches(sel, labels) is want


@pytest.mark.parametrize("sel", ["a>1", "a in (x", "a notin", "=x", "a b=c"])
def test_selector_rejections(sel):
    with pytest.raises(KwokError):
        selector_matches(sel, {})


def test_reference_pod_test_objects():
    """pod_controller_test.go:76-193: the disregard-annotated pod1 is not locked,
    the pod with a deletionTimestamp is routed to deletion."""
    codec = Codec(manage_all_nodes=True, disregard_status_with_annotation_selector="fake=custom")
    base = {"metadata": {"name": "pod1", "namespace": "default", "creationTimestamp": "2024-01-01T00:00:00Z"},
            "spec": {"nodeName": "node0", "containers": [{"name": "test-container", "image": "test-image"}]},
            "status": {}}
    p1 = json.loads(json.dumps(base))
    p1["metadata"]["annotations"] = {"fake": "custom"}
    p1["status"]["reason"] = "custom"
    p2 = json.loads(json.dumps(base))
    p2["metadata"]["deletionTimestamp"] = "2024-01-01T00:01:00Z"
    p3 = json.loads(json.dumps(base))
    p3["metadata"]["annotations"] = {}  # empty maps never match (pod_controller.go:258)
    b = codec.decode_pods([p1, p2, p3, base])
    assert b.pods[0].ev.flags == abi.POD_DISREGARD | abi.POD_STATUS_NONEMPTY
    assert b.pods[1].ev.flags == abi.POD_DELETING
    assert b.pods[2].ev.flags == 0 and b.pods[3].ev.flags == 0
    assert b.pods[3].ev.creation_unix == 1704067200


def test_node_selection_modes():
    node = {"metadata": {"name": "n0", "annotations": {"kwok.x-k8s.io/node": "fake"}, "labels": {"type": "kwok"}},
            "status": {}}
    other = {"metadata": {"name": "n1"}, "status": {}}
    for kw, want in [(dict(manage_all_nodes=True), (1, 1)),
                     (dict(manage_all_nodes=False, manage_nodes_with_annotation_selector=MANAGE), (1, 0)),
                     (dict(manage_all_nodes=False, manage_nodes_with_label_selector="type=kwok"), (1, 0))]:
        b = Codec(**kw).decode_nodes([node, other])
        assert (b.nodes[0].managed, b.nodes[1].managed) == want, kw
    with pytest.raises(KwokError):
        Codec(manage_all_nodes=False)  # controller.go:99-100 "no nodes are managed"
    # disregard on nodes (needLockNode, node_controller.go:210-223)
    b = Codec(disregard_status_with_label_selector="type=kwok").decode_nodes([node, other])
    assert (b.nodes[0].lockable, b.nodes[1].lockable) == (0, 1)


def test_conforms_is_strict_per_field():
    ev = dict(key="p", node="n", disregard=False, deleting=False, finalizers=0, creation=1704067140,
              phase="Running", status_nonempty=True, conforms=True, hostIP="196.168.0.1", podIP="10.0.0.9",
              spec={"containers": [["c", "img"]], "init": [], "gates": ["g1"]})
    codec = Codec()
    good = pod_doc(ev)
    bad = []
    for mut in ("cond_status", "missing_gate", "started", "image", "restart", "extra_container", "init", "start_time"):
        d = json.loads(json.dumps(good))
        st = d["status"]
        if mut == "cond_status":
            st["conditions"][1]["status"] = "False"
        elif mut == "missing_gate":
            st["conditions"].pop()
        elif mut == "started":
            st["containerStatuses"][0]["state"]["running"]["startedAt"] = "2024-01-01T00:00:01Z"
        elif mut == "image":
            st["containerStatuses"][0]["image"] = "other"
        elif mut == "restart":
            st["containerStatuses"][0]["restartCount"] = 1
        elif mut == "extra_container":
            st["containerStatuses"].append(dict(st["containerStatuses"][0], name="x"))
        elif mut == "init":
            st["initContainerStatuses"] = [{"name": "i", "image": "i", "ready": True}]
        elif mut == "start_time":
            del st["startTime"]
        bad.append(d)
    # extra fields on conditions are kept by the merge: still a no-op
    ok2 = json.loads(json.dumps(good))
    ok2["status"]["conditions"][0]["reason"] = "whatever"
    ok2["status"]["conditions"].append({"type": "PodScheduled", "status": "True"})
    b = codec.decode_pods([good, ok2] + bad)
    assert b.pods[0].ev.flags & abi.POD_CONFORMS and b.pods[1].ev.flags & abi.POD_CONFORMS
    for i in range(2, len(b.pods)):
        assert not b.pods[i].ev.flags & abi.POD_CONFORMS, i


def test_domain_rejections():
    codec = Codec()
    base = {"metadata": {"name": "p", "creationTimestamp": "2024-01-01T00:00:00Z"},
            "spec": {"nodeName": "n", "containers": [{"name": "c", "image": "i"}]}}
    cases = []
    d = json.loads(json.dumps(base)); d["metadata"]["creationTimestamp"] = "2024-01-01T00:00:00.5Z"; cases.append(d)
    d = json.loads(json.dumps(base)); d["spec"]["nodeName"] = "né"; cases.append(json.dumps(d).encode())  # escape
    d = json.loads(json.dumps(base)); d["spec"]["containers"] *= 33; cases.append(d)
    cases.append(b'{"metadata": {"name": "p"}')
    b = codec.decode_pods(cases, strict=False)
    assert all(s == abi.EDOMAIN for s in b.status), b.status
    nb = codec.decode_nodes([{"metadata": {"name": "n"}, "status": {"capacity": {"cpu": 1.5}}}], strict=False)
    assert nb.status == [abi.EDOMAIN]


@pytest.mark.parametrize("name", __import__("harness").TRACES)
def test_trace_via_json_codec_matches_golden_on_oracle(name):
    """Whole ingest path on CPU: JSON objects -> codec -> oracle, every tick
    equal to the golden trace (the checker side of test_parity_gpu's
    test_engine_golden_trace_via_json)."""
    import harness
    from oracle.oracle import Oracle
    fx = harness.load_trace(name)
    codec = Codec(manage_all_nodes=False, manage_nodes_with_annotation_selector=MANAGE,
                  disregard_status_with_annotation_selector=DISREGARD)
    o = Oracle(harness.config_for(fx))
    harness.replay(fx, o, codec=codec)
    o.close()


def test_threaded_batch_equals_serial():
    """kwok_decode_pods / _nodes with several host threads give the records
    (and in-place canonical blobs) of the one-thread decode."""
    import harness
    fx = harness.load_trace("churn")
    pods = [e for t in fx["ticks"] for e in t["pod_events"] if e["op"] == "upsert"]
    nodes = [e for t in fx["ticks"] for e in t["node_events"] if e["op"] == "upsert"]
    rng = random.Random(3)
    pdocs = [scramble(pod_doc(e), rng) for e in pods]
    ndocs = [scramble(node_doc(e), rng) for e in nodes]
    codec = Codec(manage_all_nodes=False, manage_nodes_with_annotation_selector=MANAGE,
                  disregard_status_with_annotation_selector=DISREGARD)
    for kind, docs in (("pods", pdocs), ("nodes", ndocs)):
        one = getattr(codec, "decode_" + kind)(docs, threads=1)
        many = getattr(codec, "decode_" + kind)(docs, threads=5)
        recs = lambda b: [bytes(r) for r in (b.pods if kind == "pods" else b.nodes)]
        assert recs(one) == recs(many) and one.buf == many.buf and one.status == many.status


def test_parser_survives_mutated_documents():
    """Truncations, byte flips and deep nesting of real documents: every one
    decodes or is rejected with KWOK_EDOMAIN; nothing reads past its span."""
    import harness
    fx = harness.load_trace("specs")
    ev = [e for t in fx["ticks"] for e in t["pod_events"] if e["op"] == "upsert"][0]
    good = json.dumps(pod_doc(ev)).encode()
    rng = random.Random(11)
    docs = [good[:k] for k in range(0, len(good), 7)]
    for _ in range(400):
        b = bytearray(good)
        for _ in range(rng.randint(1, 4)):
            b[rng.randrange(len(b))] = rng.choice(b'{}[]",:\\0123456789tfnul \x00\xff')
        docs.append(bytes(b))
    docs.append(b"[" * 5000 + b"]" * 5000)
    docs.append(b'{"metadata":' + b'{"a":' * 100 + b"1" + b"}" * 100 + b"}")
    codec = Codec()
    b = codec.decode_pods(docs, strict=False, threads=4)
    assert set(b.status) <= {abi.OK, abi.EDOMAIN}, set(b.status)
    assert b.status[-1] == abi.EDOMAIN and b.status[-2] == abi.EDOMAIN
    assert b.status[len(good) // 7 + 1:].count(abi.OK) >= 1  # some flips land in values and still decode
