"""GPU: the pod codec on the device (kwok_decode_pods_gpu / kwok_ingest_pods_json,
kwok_amd/csrc/json.hip) against the host codec (kwok_decode_pods, codec.cpp),
document for document: the same status, and for every decoded document the
same kwok_pod_event bytes, name / namespace spans and pod spec (its
kwok_spec_key).  The corpus: every golden trace's pod events as Kubernetes JSON
(compact, indented, key order scrambled), the apiserver echo of every expected
pod patch (conforming statuses), the per-field no-op cases of
test_codec.py::test_conforms_is_strict_per_field, the domain rejections,
escapes, byte-flipped and truncated documents, deep nesting, and several
disregard selectors.  Then the golden traces replayed through
kwok_ingest_pods_json (decode + event switch on the device), and the C4
storm's 2M documents per tick decoded on the device equal to the host codec.
Reference: pod_controller.go:252-269, 301-343 (routing), 404-439 (no-op test)."""
import json
import random

import numpy as np
import pytest

import harness
from harness import DISREGARD, MANAGE, pod_doc
from kwok_amd import abi, workload
from kwok_amd.codec import Codec
from kwok_amd.engine import Engine, make_config, spec_key
from test_codec import scramble

pytestmark = pytest.mark.gpu

SELECTORS = [dict(disregard_status_with_annotation_selector=DISREGARD),
             dict(disregard_status_with_label_selector="app in (fake, x),!skip"),
             dict(disregard_status_with_annotation_selector="kwok.x-k8s.io/status",
                  disregard_status_with_label_selector="app notin (web)"),
             dict()]


def host_decode(codec, docs):
    b = codec.decode_pods(docs, strict=False, threads=8)
    return b


def compare(e, codec, docs, want_host=None, where=""):
    """every document: GPU status == host status; decoded ones field for field"""
    ev, names, keys, st, n_host = e.decode_pods_gpu(codec, docs)
    b = host_decode(codec, docs)
    hs = np.array(b.status, np.int32)
    bad = np.nonzero(st != hs)[0]
    assert not len(bad), "%s: %d statuses differ, first doc %d: gpu %d host %d: %r" % (
        where, len(bad), bad[0], st[bad[0]], hs[bad[0]], docs[bad[0]][:300])
    for i in np.nonzero(hs == abi.OK)[0]:
        d = b.pods[i]
        want = np.frombuffer(bytes(d.ev), abi.POD_EVENT_DTYPE)[0]
        assert ev[i].tobytes() == want.tobytes(), "%s: doc %d event %r vs %r" % (where, i, ev[i], want)
        assert (names[i, 0, 0], names[i, 0, 1]) == (d.name.off, d.name.len), (where, i)
        assert (names[i, 1, 0], names[i, 1, 1]) == (d.namespace_.off, d.namespace_.len), (where, i)
        spec = ([(b.text(c.name), b.text(c.image)) for c in d.containers[:d.n_containers]],
                [(b.text(c.name), b.text(c.image)) for c in d.init_containers[:d.n_init_containers]],
                [b.text(g) for g in d.readiness_gates[:d.n_readiness_gates]])
        assert int(keys[i]) == spec_key(*spec), (where, i)
    if want_host is not None:
        assert n_host == want_host, (where, n_host)
    return n_host, hs


def golden_docs(rng):
    """(canonical documents, scrambled documents, echo documents) of every trace"""
    canon, scr, echo = [], [], []
    for name in harness.TRACES:
        fx = harness.load_trace(name)
        by_handle = {}
        for t in fx["ticks"]:
            for ev in t["pod_events"]:
                d = pod_doc(ev)
                canon.append(json.dumps(d).encode())
                scr.append(scramble(d, rng))
                by_handle[ev["expect_handle"] if ev.get("handle", -1) == -1 else ev["handle"]] = ev
            for h, patch in t["expect"].get("pod_patches", []):
                d = pod_doc(by_handle[h])
                d["status"].update(json.loads(patch)["status"])
                echo.append(json.dumps(d, indent=1).encode())
    return canon, scr, echo


@pytest.fixture(scope="module")
def eng():
    e = Engine(make_config(buckets=64, node_slots_per_bucket=16, pod_slots_per_bucket=128))
    yield e
    e.close()


@pytest.mark.parametrize("sel", range(len(SELECTORS)))
def test_golden_documents_equal_the_host_codec(eng, sel):
    """canonical documents (metadata, spec, status in Go's order), the apiserver
    echo of expected patches (conforming on both sides) and documents with
    scrambled key order (statuses ahead of spec or metadata: the second pass) are
    all decided on the device"""
    rng = random.Random(5)
    canon, scr, echo = golden_docs(rng)
    codec = Codec(manage_all_nodes=True, **SELECTORS[sel])
    compare(eng, codec, canon, want_host=0, where="canonical")
    compare(eng, codec, echo, want_host=0, where="echo")
    compare(eng, codec, scr, want_host=0, where="scrambled")


def test_no_op_cases_and_rejections(eng):
    """test_codec.py's per-field CONFORMS cases and domain rejections, plus
    escapes: in a referenced string (EDOMAIN), in a compared one (host), in an
    ignored one (device)"""
    ev = dict(key="p", node="n", disregard=False, deleting=False, finalizers=0, creation=1704067140,
              phase="Running", status_nonempty=True, conforms=True, hostIP="196.168.0.1", podIP="10.0.0.9",
              spec={"containers": [["c", "img"]], "init": [["i", "busybox"]], "gates": ["g1", "g2"]})
    good = pod_doc(ev)
    docs = [good]
    muts = {
        "cond_status": lambda st: st["conditions"][1].update(status="False"),
        "cond_ltt": lambda st: st["conditions"][0].update(lastTransitionTime="2024-01-01T00:00:00Z"),
        "missing_gate": lambda st: st["conditions"].pop(),
        "dup_cond": lambda st: st["conditions"].insert(0, dict(st["conditions"][1], status="False")),
        "started": lambda st: st["containerStatuses"][0]["state"]["running"].update(startedAt="x"),
        "image": lambda st: st["containerStatuses"][0].update(image="other"),
        "image_null": lambda st: st["containerStatuses"][0].update(image=None),
        "ready_false": lambda st: st["containerStatuses"][0].update(ready=False),
        "restart": lambda st: st["containerStatuses"][0].update(restartCount=1),
        "restart_zero_str": lambda st: st["containerStatuses"][0].update(restartCount=""),
        "extra_zero": lambda st: st["containerStatuses"][0].update(containerID="", lastState={"waiting": None}),
        "extra_nonzero": lambda st: st["containerStatuses"][0].update(started=True),
        "state_extra": lambda st: st["containerStatuses"][0]["state"].update(waiting={"reason": "x"}),
        "state_zero": lambda st: st["containerStatuses"][0]["state"].update(waiting={}),
        "extra_container": lambda st: st["containerStatuses"].append(dict(st["containerStatuses"][0], name="x")),
        "cs_null": lambda st: st.update(containerStatuses=None),
        "cs_obj": lambda st: st.update(containerStatuses={}),
        "init_exit": lambda st: st["initContainerStatuses"][0]["state"]["terminated"].update(exitCode=1),
        "init_reason": lambda st: st["initContainerStatuses"][0]["state"]["terminated"].update(reason="Error"),
        "init_missing": lambda st: st.pop("initContainerStatuses"),
        "start_time": lambda st: st.pop("startTime"),
        "start_time_num": lambda st: st.update(startTime=5),
        "phase_pending": lambda st: st.update(phase="Pending"),
        "phase_odd": lambda st: st.update(phase="Weird"),
        "phase_num": lambda st: st.update(phase=3),
        "host_ip_null": lambda st: st.update(hostIP=None),
    }
    for name, f in muts.items():
        d = json.loads(json.dumps(good))
        f(d["status"])
        docs.append(d)
    ok2 = json.loads(json.dumps(good))  # extra condition fields / conditions: still a no-op
    ok2["status"]["conditions"][0]["reason"] = "whatever"
    ok2["status"]["conditions"].append({"type": "PodScheduled", "status": "True"})
    docs.append(ok2)
    base = {"metadata": {"name": "p", "creationTimestamp": "2024-01-01T00:00:00Z"},
            "spec": {"nodeName": "n", "containers": [{"name": "c", "image": "i"}]}}
    rej = [("ct_frac", lambda d: d["metadata"].update(creationTimestamp="2024-01-01T00:00:00.5Z")),
           ("ct_num", lambda d: d["metadata"].update(creationTimestamp=5)),
           ("ct_missing", lambda d: d["metadata"].pop("creationTimestamp")),
           ("too_many", lambda d: d["spec"].update(containers=d["spec"]["containers"] * 33)),
           ("gates_obj", lambda d: d["spec"].update(readinessGates={"a": 1})),  # ignored: not a list
           ("gates_elem", lambda d: d["spec"].update(readinessGates=["x"])),
           ("meta_arr", lambda d: d.update(metadata=[])),
           ("spec_null", lambda d: d.update(spec=None)),
           ("status_arr", lambda d: d.update(status=[1])),
           ("status_null", lambda d: d.update(status=None)),
           ("ann_num", lambda d: d["metadata"].update(annotations={"a": 1})),
           ("labels_arr", lambda d: d["metadata"].update(labels=["a"])),
           ("name_num", lambda d: d["metadata"].update(name=1)),
           ("name_null", lambda d: d["metadata"].update(name=None)),
           ("cont_str", lambda d: d["spec"].update(containers=["c"])),
           ("cont_obj", lambda d: d["spec"].update(containers={})),
           ("dup_meta", lambda d: None),
           ("fin_empty", lambda d: d["metadata"].update(finalizers=[])),
           ("fin_obj", lambda d: d["metadata"].update(finalizers={"a": 1})),
           ("dt_null", lambda d: d["metadata"].update(deletionTimestamp=None)),
           ("dt_obj", lambda d: d["metadata"].update(deletionTimestamp={})),
           ("empty_status", lambda d: d.update(status={"conditions": [], "podIPs": [], "qosClass": ""}))]
    for name, f in rej:
        d = json.loads(json.dumps(base))
        f(d)
        docs.append(d)
    raw = [json.dumps(good).encode()]
    raw.append(raw[0].replace(b'"n"', b'"\\u006e"', 1))                      # escaped nodeName: EDOMAIN
    raw.append(raw[0].replace(b'"Running"', b'"Runn\\u0069ng"', 1))          # escaped phase: host
    raw.append(raw[0].replace(b'"uid"', b'"u\\u0069d"', 1))                  # escaped ignored key: device
    raw.append(raw[0].replace(b'"type": "Ready"', b'"type": "Re\\u0061dy"', 1))  # escaped condition type: host
    raw.append(b'{"metadata": {"name": "a", "name": 5, "creationTimestamp": "2024-01-01T00:00:00Z"}, '
               b'"metadata": 1, "spec": {"containers": null}}')                   # duplicate keys: first wins
    raw.append(b'  {"metadata":{"name":"a","creationTimestamp":"2024-01-01T00:00:00Z"},"spec":{}}  \n')
    raw.append(b'{"metadata":{"name":"a","creationTimestamp":"2024-01-01T00:00:00Z"},"spec":{}} x')
    raw.append(b'{"metadata":{"name":"a","creationTimestamp":"2024-01-01T00:00:00Z","x":[-,+1,1e,.]},"spec":{}}')
    raw.append(b'{"metadata":{"name":"a\\ud800\\u0041","creationTimestamp":"2024-01-01T00:00:00Z"},"spec":{}}')
    raw.append(b'{"metadata":{"name":"a","creationTimestamp":"2024-01-01T00:00:00Z","z":"\\ud800\\u0041"},'
               b'"spec":{}}')
    codec = Codec(disregard_status_with_annotation_selector="fake=custom")
    n_host, hs = compare(eng, codec, docs + raw, where="cases")
    assert (hs[:len(docs)] == abi.OK).sum() > len(muts)
    assert n_host >= 2
    # the same documents with the status first, and between metadata and spec: the
    # device's second pass decides the same no-op test (no more listed for the host)
    for order in (("status", "metadata", "spec"), ("metadata", "status", "spec")):
        moved = [json.dumps({k: d[k] for k in order + tuple(k for k in d if k not in order) if k in d}).encode()
                 if isinstance(d, dict) else d for d in docs]
        n2, hs2 = compare(eng, codec, moved + raw, where="status first %r" % (order,))
        assert (hs2 == hs).all() and n2 == n_host, order


def test_mutated_and_nested_documents(eng):
    """byte flips and truncations of real documents, deep nesting: the device and
    the host agree on every status (and record); nothing reads past a span"""
    fx = harness.load_trace("specs")
    evs = [e for t in fx["ticks"] for e in t["pod_events"] if e["op"] == "upsert"]
    rng = random.Random(11)
    docs = []
    for ev in evs[:6]:
        good = json.dumps(pod_doc(ev)).encode()
        docs += [good[:k] for k in range(0, len(good), 5)]
        for _ in range(300):
            b = bytearray(good)
            for _ in range(rng.randint(1, 4)):
                b[rng.randrange(len(b))] = rng.choice(b'{}[]",:\\0123456789tfnul eE+-.\x00\xff\x1f')
            docs.append(bytes(b))
    docs.append(b"[" * 70 + b"]" * 70)
    docs.append(b'{"metadata":' + b'{"a":' * 63 + b"1" + b"}" * 63 + b', "spec": {}}')
    docs.append(b'{"metadata":' + b'{"a":' * 64 + b"{}" + b"}" * 64 + b"}")
    docs.append(b'{"metadata":' + b'{"a":' * 64 + b"1" + b"}" * 64 + b"}")
    docs.append(b'{"x":' + b"[" * 63 + b"]" * 63 + b"}")
    docs.append(b'{"x":' + b"[" * 64 + b"]" * 64 + b"}")
    codec = Codec(disregard_status_with_label_selector="app=fake")
    compare(eng, codec, docs, where="mutated")


@pytest.mark.parametrize("name", harness.TRACES)
def test_golden_trace_through_gpu_ingest(name):
    """kwok_ingest_pods_json: every pod event of the trace as its Kubernetes
    document, decoded and routed on the device (specs registered as they
    appear, nodes by spec.nodeName); handles, statuses and every tick's outputs
    equal the golden trace (the test_engine_golden_trace_via_json of the
    device codec)"""
    fx = harness.load_trace(name)
    e = Engine(harness.config_for(fx))
    codec = Codec(manage_all_nodes=False, manage_nodes_with_annotation_selector=MANAGE,
                  disregard_status_with_annotation_selector=DISREGARD)
    for ti, t in enumerate(fx["ticks"]):
        if t["node_events"]:
            recs, arena = harness.node_batch(t["node_events"])
            hs, st = e.ingest_nodes_raw(recs, arena)
            assert list(st) == [0] * len(st)
        evs = t["pod_events"]
        if evs:
            arena, offs, lens = Engine._docs([pod_doc(ev) for ev in evs])
            ops = np.array([abi.OP_DELETE if ev["op"] == "delete" else abi.OP_UPSERT for ev in evs], np.uint8)
            handles = np.array([ev.get("handle", -1) for ev in evs], np.int32)
            hs, st, _rel, n_host = e.ingest_pods_json(codec, arena, offs, lens, ops, handles)
            assert list(st) == [0] * len(st), (ti, list(st))
            assert list(hs) == [ev["expect_handle"] for ev in evs], ti
        out = e.tick(t["now"])
        harness.compare_tick(fx["name"], ti, t["expect"], out)
    e.close()


def c4_documents(n=1_000_000, seed=3):
    """one C4 tick's documents: n deletion-marked Running pods and n creates"""
    names = workload.node_names(0, n)
    ch = workload.ChurnJson(np.arange(n, dtype=np.int32), np.arange(n, dtype=np.int32) // 1, 0, n, n, seed=seed,
                            node_name_of=names)
    pip = (abi.ip4("10.0.0.1") + np.arange(n)).astype(np.uint32)
    dump = lambda: (np.ones(n, np.uint8), np.full(n, abi.PHASE_RUNNING, np.uint8), None, pip)  # noqa: E731
    return ch.batch_json(dump, workload.S0 + 90)


def test_c4_documents_equal_the_host_codec():
    """C4 at its stated size: the 2M pod documents of one churn tick (1M
    deletion-marked Running pods, half with finalizers, and 1M scheduled Pending
    creates, as the apiserver serialises them) decoded on the device, record for
    record equal to the host codec; none left to the host"""
    e = Engine(make_config(buckets=64, node_slots_per_bucket=16, pod_slots_per_bucket=128))
    codec = Codec(manage_all_nodes=True)
    arena, offs, lens, ops, handles = c4_documents()
    ev, names, keys, st, n_host = e.decode_pods_gpu(codec, arena=arena, offs=offs, lens=lens)
    assert n_host == 0 and (st == 0).all()
    h = workload.host_decode_arrays(codec, arena, offs, lens, threads=16)
    assert (h["status"] == 0).all()
    assert (ev.view(np.uint8) == h["ev"].view(np.uint8)).all()
    assert (names == h["names"]).all()
    assert (keys == spec_key([("fake-pod", "fake")])).all()
    n = len(offs) // 2
    assert (ev["flags"][:n] & abi.POD_CONFORMS).all() and (ev["flags"][:n] & abi.POD_DELETING).all()
    assert 0.45 < (ev["flags"][:n] & abi.POD_HAS_FINALIZERS).astype(bool).mean() < 0.55
    assert (ev["phase"][n:] == abi.PHASE_PENDING).all() and not (ev["flags"][n:] & abi.POD_CONFORMS).any()
    e.close()


@pytest.mark.parametrize("name", ["specs", "reference_pod_test", "churn"])
def test_spec_key_collisions_are_decided_exactly(name, monkeypatch):
    """kwok_spec_key is FNV-1a 64, not collision-resistant, and pod specs come
    from users.  With the keys cut to 1 bit (KWOK_DEBUG_SPEC_KEY_BITS) every
    spec collides with another: a document whose key hits a registered spec of
    other strings is handed to the host (JSON_SPEC_X) after the device compares
    the strings, so every trace still replays to the golden outputs"""
    monkeypatch.setenv("KWOK_DEBUG_SPEC_KEY_BITS", "1")
    test_golden_trace_through_gpu_ingest(name)
