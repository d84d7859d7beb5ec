"""GPU: the node codec on the device (kwok_decode_nodes_gpu / kwok_ingest_nodes_json,
kwok_amd/csrc/json.hip k_json_nodes) against the host codec (kwok_decode_nodes,
codec.cpp), document for document: the same status and, for every decoded
document, the same kwok_node_event bytes and the same arena (the host codec
re-serialises non-empty addresses / allocatable / capacity blobs in place; the
device lists those documents for it).  The corpus: every golden trace's node
events as Kubernetes JSON (compact, indented, key order scrambled), the
domain rejections, escapes, byte-flipped and truncated documents, under
several manage / disregard selectors.  Then the golden traces replayed with
both watches through the device codecs (kwok_ingest_nodes_json +
kwok_ingest_pods_json), and C5's flap batches at 1M nodes from their documents.
Reference: node_controller.go:206-223 (needHeartbeat / needLockNode), :256-279
(watch routing), :356-391 (the A.5 inputs); controller.go:81-98 (selectors)."""
import json
import random

import numpy as np
import pytest

import harness
from harness import DISREGARD, MANAGE, node_doc, pod_doc
from kwok_amd import abi, workload
from kwok_amd.codec import Codec
from kwok_amd.engine import Engine, make_config
from test_codec import scramble

pytestmark = pytest.mark.gpu

SELECTORS = [dict(manage_all_nodes=False, manage_nodes_with_annotation_selector=MANAGE,
                  disregard_status_with_annotation_selector=DISREGARD),
             dict(manage_all_nodes=True),
             dict(manage_all_nodes=False, manage_nodes_with_label_selector="type in (kwok, fake),!skip",
                  disregard_status_with_label_selector="status=custom"),
             dict(manage_all_nodes=False, manage_nodes_with_annotation_selector="kwok.x-k8s.io/node",
                  disregard_status_with_label_selector="status notin (ok)")]


def compare(e, codec, docs, want_host=None, where=""):
    """every document: GPU status == host status; decoded ones byte for byte"""
    arena, offs, lens = Engine._docs(docs)
    ev, st, n_host, ar_gpu = e.decode_nodes_gpu(codec, arena=arena, offs=offs, lens=lens)
    b = codec.decode_nodes(docs, strict=False, threads=8)
    hs = np.array(b.status, np.int32)
    bad = np.nonzero(st != hs)[0]
    assert not len(bad), "%s: %d statuses differ, first doc %d: gpu %d host %d: %r" % (
        where, len(bad), bad[0], st[bad[0]], hs[bad[0]], docs[bad[0]][:300])
    for i in np.nonzero(hs == abi.OK)[0]:
        want = np.frombuffer(bytes(b.nodes[i]), abi.NODE_EVENT_DTYPE)[0]
        assert ev[i].tobytes() == want.tobytes(), "%s: doc %d event %r vs %r" % (where, i, ev[i], want)
    assert ar_gpu == bytes(b.buf), where + ": arenas (canonical blobs) differ"
    if want_host is not None:
        assert n_host == want_host, (where, n_host)
    return n_host


def with_labels(d, rng):
    """the same node with labels for the label selectors"""
    d = json.loads(json.dumps(d))
    lab = {}
    if rng.random() < 0.7:
        lab["type"] = rng.choice(["kwok", "fake", "real"])
    if rng.random() < 0.2:
        lab["skip"] = ""
    if rng.random() < 0.3:
        lab["status"] = rng.choice(["custom", "ok"])
    d["metadata"]["labels"] = lab
    return d


def golden_node_docs(rng):
    canon, scr = [], []
    for name in harness.TRACES:
        fx = harness.load_trace(name)
        for t in fx["ticks"]:
            for ev in t["node_events"]:
                if ev["op"] == "delete":
                    continue
                d = with_labels(node_doc(ev), rng)
                canon.append(json.dumps(d, separators=(",", ":")).encode())
                scr.append(scramble(d, rng))
    return canon, scr


@pytest.fixture(scope="module")
def eng():
    e = Engine(make_config(buckets=64, node_slots_per_bucket=16, pod_slots_per_bucket=128))
    yield e
    e.close()


@pytest.mark.parametrize("sel", range(len(SELECTORS)))
def test_golden_node_documents_equal_the_host_codec(eng, sel):
    """the golden traces' nodes (empty statuses on the device, statuses with
    blobs listed for the host), compact and with scrambled key order"""
    rng = random.Random(11)
    canon, scr = golden_node_docs(rng)
    codec = Codec(**SELECTORS[sel])
    compare(eng, codec, canon, where="canonical")
    compare(eng, codec, scr, where="scrambled")
    # kwok's own fleets: Nodes created with a zero status are all decided on the device
    empty = [json.dumps(json.loads(d)) .encode() for d in canon]
    zero = []
    for d in empty:
        x = json.loads(d)
        x["status"] = {"daemonEndpoints": {"kubeletEndpoint": {"Port": 0}},
                       "nodeInfo": {k: "" for k in abi.NODEINFO_KEYS}}
        zero.append(json.dumps(x).encode())
    compare(eng, codec, zero, want_host=0, where="zero status")


def test_node_rejections_escapes_and_mutations(eng):
    """the host codec's domain, decision for decision: wrong types, escapes in
    referenced and in routed strings, status shapes, empty blobs, first-key
    semantics; then byte-flipped and truncated documents"""
    base = {"metadata": {"name": "node-1", "annotations": {"kwok.x-k8s.io/node": "fake"}, "labels": {"type": "kwok"}},
            "status": {"phase": "Running", "nodeInfo": {"kubeletVersion": "fake", "osImage": "x"}}}

    def v(f):
        d = json.loads(json.dumps(base))
        f(d)
        return json.dumps(d).encode()

    docs = [
        v(lambda d: None),
        v(lambda d: d.pop("metadata")),
        v(lambda d: d.__setitem__("metadata", None)),
        v(lambda d: d["metadata"].pop("name")),
        v(lambda d: d["metadata"].__setitem__("name", "")),
        v(lambda d: d["metadata"].__setitem__("name", 7)),
        v(lambda d: d["metadata"].__setitem__("annotations", None)),
        v(lambda d: d["metadata"].__setitem__("annotations", [])),
        v(lambda d: d["metadata"]["annotations"].__setitem__("kwok.x-k8s.io/node", 1)),
        v(lambda d: d["metadata"]["labels"].__setitem__("type", None)),
        v(lambda d: d.__setitem__("status", None)),
        v(lambda d: d.__setitem__("status", "x")),
        v(lambda d: d.__setitem__("status", [1])),
        v(lambda d: d["status"].__setitem__("phase", 3)),
        v(lambda d: d["status"].__setitem__("phase", "")),
        v(lambda d: d["status"].__setitem__("phase", "Terminated")),
        v(lambda d: d["status"].__setitem__("addresses", [])),
        v(lambda d: d["status"].__setitem__("addresses", {})),
        v(lambda d: d["status"].__setitem__("addresses", None)),
        v(lambda d: d["status"].__setitem__("addresses", "x")),
        v(lambda d: d["status"].__setitem__("addresses", [{"type": "InternalIP", "address": "10.0.0.1"}])),
        v(lambda d: d["status"].__setitem__("allocatable", {})),
        v(lambda d: d["status"].__setitem__("allocatable", [])),
        v(lambda d: d["status"].__setitem__("allocatable", {"cpu": "4", "memory": "1Gi"})),
        v(lambda d: d["status"].__setitem__("capacity", {"pods": 110})),
        v(lambda d: d["status"].__setitem__("capacity", {"pods": 1.5})),
        v(lambda d: d["status"].__setitem__("nodeInfo", None)),
        v(lambda d: d["status"].__setitem__("nodeInfo", "x")),
        v(lambda d: d["status"]["nodeInfo"].__setitem__("architecture", 1)),
        v(lambda d: d["status"]["nodeInfo"].__setitem__("bootID", None)),
    ]
    # escapes: in a referenced string (EDOMAIN), in a routed key / compared value (host)
    docs.append(b'{"metadata":{"name":"node\\u002d2"},"status":{}}')
    docs.append(b'{"metadata":{"na\\u006de":"node-3"},"status":{}}')
    docs.append(b'{"metadata":{"na\\u006de":"node-4","name":5},"status":{}}')
    docs.append(b'{"metadata":{"name":"node-5","annotations":{"kwok.x-k8s.io\\/node":"fake"}},"status":{}}')
    docs.append(b'{"metadata":{"name":"node-6","annotations":{"kwok.x-k8s.io/node":"f\\u0061ke"}},"status":{}}')
    docs.append(b'{"metadata":{"name":"node-7"},"status":{"phase":"Runn\\u0069ng"}}')
    docs.append(b'{"metadata":{"name":"node-8"},"status":{"nodeInfo":{"osImage":"a\\nb"}}}')
    docs.append(b'{"metadata":{"name":"node-9"},"stat\\u0075s":{"phase":"x"}}')
    docs.append(b'{"metadata":{"name":"node-10"},"metadata":{"name":"other"}}')
    docs.append(b'{"metadata":{"name":"node-11"},"status":{"phase":"Running"},"status":{"phase":""}}')
    docs.append(b'{"metadata":{"name":"node-12","annotations":{"kwok.x-k8s.io/node":"x","kwok.x-k8s.io/node":"fake"}}}')
    docs.append(b'[{"metadata":{"name":"node-13"}}]')
    docs.append(b'{"metadata":{"name":"node-14"}')
    for sel in SELECTORS:
        compare(eng, Codec(**sel), docs, where="cases %r" % sel)
    rng = random.Random(3)
    canon, _ = golden_node_docs(rng)
    mut = []
    for d in canon[:200]:
        b = bytearray(d)
        i = rng.randrange(len(b))
        b[i] = rng.choice(b'{}[]",:\\ 0a')
        mut.append(bytes(b))
        mut.append(d[:rng.randrange(1, len(d))])
    for sel in SELECTORS[:2]:
        compare(eng, Codec(**sel), mut, where="mutated")


def _op(ev):
    return abi.OP_DELETE if ev["op"] == "delete" else abi.OP_UPSERT


@pytest.mark.parametrize("name", harness.TRACES)
def test_golden_trace_through_both_gpu_codecs(name):
    """both watches from their documents: nodes through kwok_ingest_nodes_json,
    pods through kwok_ingest_pods_json; handles, statuses and every tick's
    outputs equal the golden trace (Deleted node events carry the last state of
    the node, whose status the device does not read)"""
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    codec = Codec(manage_all_nodes=False, manage_nodes_with_annotation_selector=MANAGE,
                  disregard_status_with_annotation_selector=DISREGARD)
    last = {}
    for ti, t in enumerate(fx["ticks"]):
        nev = t["node_events"]
        if nev:
            docs = []
            for ev in nev:
                if ev["op"] == "delete":
                    d = last.get(ev["name"]) or {"metadata": {"name": ev["name"]}}
                else:
                    d = last[ev["name"]] = node_doc(ev)
                docs.append(json.dumps(d).encode())
            arena, offs, lens = Engine._docs(docs)
            hs, st, _nh = e.ingest_nodes_json(codec, arena, offs, lens, np.array([_op(x) for x in nev], np.uint8))
            assert list(st) == [0] * len(st), (ti, list(st))
        evs = t["pod_events"]
        if evs:
            arena, offs, lens = Engine._docs([pod_doc(ev) for ev in evs])
            ops = np.array([_op(ev) for ev in evs], np.uint8)
            handles = np.array([ev.get("handle", -1) for ev in evs], np.int32)
            hs, st, _rel, _nh = e.ingest_pods_json(codec, arena, offs, lens, ops, handles)
            assert list(st) == [0] * len(st), (ti, list(st))
            assert list(hs) == [ev["expect_handle"] for ev in evs], ti
        out = e.tick(t["now"])
        harness.compare_tick(fx["name"], ti, t["expect"], out)
    e.close()
