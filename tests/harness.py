"""Trace harness: replays tests/golden/trace_*.json fixtures through any
ABI implementation (the HIP engine or the CPU oracle) and compares every tick
with the fixture's expected outputs, the way the reference's unit tests drive
NewNodeController/NewPodController against a fake clientset
(node_controller_test.go:37-155, pod_controller_test.go:37-194)."""
from __future__ import annotations

import json
import os
import time

import numpy as np

from kwok_amd import abi
from kwok_amd.engine import make_config

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TRACES = ["reference_node_test", "reference_pod_test", "doc_known_answer", "cidr_overflow", "specs", "churn",
          "e2e_kwok_test", "same_interval_echo"]


def load_trace(name):
    with open(os.path.join(GOLDEN, "trace_%s.json" % name)) as f:
        return json.load(f)


def cjson(v):
    return json.dumps(v, sort_keys=True, separators=(",", ":")) if v else ""


def node_batch(events):
    ar = abi.Arena()
    recs = np.zeros(len(events), abi.NODE_EVENT_DTYPE)
    for i, ev in enumerate(events):
        r = recs[i]
        r["op"] = abi.OP_DELETE if ev["op"] == "delete" else abi.OP_UPSERT
        r["name"] = ar.ref(ev["name"])
        if ev["op"] != "delete":
            r["managed"] = 1 if ev["managed"] else 0
            r["lockable"] = 1 if ev["lockable"] else 0
            ph = ev.get("phase") or ""
            r["phase"] = abi.PHASE_NONE if not ph else (abi.PHASE_RUNNING if ph == "Running" else abi.PHASE_OTHER)
            r["addresses"] = ar.ref(cjson(ev.get("addresses")))
            r["allocatable"] = ar.ref(cjson(ev.get("allocatable")))
            r["capacity"] = ar.ref(cjson(ev.get("capacity")))
            ni = ev.get("nodeInfo") or {}
            for k, key in enumerate(abi.NODEINFO_KEYS):
                r["node_info"][k] = ar.ref(ni.get(key, ""))
    return recs, bytes(ar.buf)


class SpecCache:
    def __init__(self, backend):
        self.b = backend
        self.ids = {}

    def get(self, spec):
        key = json.dumps(spec, sort_keys=True)
        if key not in self.ids:
            self.ids[key] = self.b.register_pod_spec(
                [tuple(c) for c in spec["containers"]], [tuple(c) for c in spec.get("init", [])],
                list(spec.get("gates", [])))
        return self.ids[key]


def pod_batch(events, specs: SpecCache):
    ar = abi.Arena()
    recs = np.zeros(len(events), abi.POD_EVENT_DTYPE)
    for i, ev in enumerate(events):
        r = recs[i]
        r["op"] = abi.OP_DELETE if ev["op"] == "delete" else abi.OP_UPSERT
        r["handle"] = ev.get("handle", -1)
        r["node_handle"] = -1
        r["node_name"] = ar.ref(ev["node"])
        r["phase"] = abi.POD_PHASES[ev.get("phase") or ""]
        fl = 0
        fl |= abi.POD_DISREGARD if ev.get("disregard") else 0
        fl |= abi.POD_DELETING if ev.get("deleting") else 0
        fl |= abi.POD_STATUS_NONEMPTY if ev.get("status_nonempty") else 0
        fl |= abi.POD_CONFORMS if ev.get("conforms") else 0
        fl |= abi.POD_HAS_FINALIZERS if ev.get("finalizers") else 0
        r["flags"] = fl
        r["creation_unix"] = ev["creation"] if ev.get("creation") is not None else 0
        r["host_ip"] = ar.ref(ev.get("hostIP") or "")
        r["pod_ip"] = ar.ref(ev.get("podIP") or "")
        r["spec_id"] = specs.get(ev["spec"]) if ev["op"] != "delete" else 0
    return recs, bytes(ar.buf)


# ---- the same events as Kubernetes JSON objects, decoded by the host codec
# (kwok_decode_node / kwok_decode_pod) instead of being written as records
MANAGE = "kwok.x-k8s.io/node=fake"        # ManageNodesWithAnnotationSelector
DISREGARD = "kwok.x-k8s.io/status=custom"  # DisregardStatusWithAnnotationSelector


def rfc3339(t):
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


def pod_status_like_template(ev, creation):
    """The status pod.status.tpl renders, as the apiserver stores it."""
    st = rfc3339(creation)
    spec = ev["spec"]
    conds = [{"lastProbeTime": None, "lastTransitionTime": st, "status": "True", "type": t}
             for t in ["Initialized", "Ready", "ContainersReady"] + list(spec["gates"])]
    cs = [{"image": i, "name": n, "ready": True, "restartCount": 0, "imageID": "", "lastState": {},
           "state": {"running": {"startedAt": st}}} for n, i in spec["containers"]]
    ics = [{"image": i, "name": n, "ready": True, "restartCount": 0,
            "state": {"terminated": {"exitCode": 0, "finishedAt": st, "reason": "Completed", "startedAt": st}}}
           for n, i in spec["init"]]
    out = {"conditions": conds, "startTime": st, "qosClass": "BestEffort"}
    if cs:
        out["containerStatuses"] = cs
    if ics:
        out["initContainerStatuses"] = ics
    return out


def pod_doc(ev):
    md = {"name": ev["key"], "namespace": "default", "creationTimestamp": rfc3339(ev["creation"]),
          "uid": "u-" + ev["key"]}
    if ev["disregard"]:
        md["annotations"] = {"kwok.x-k8s.io/status": "custom", "other": "x"}
    else:
        md["labels"] = {"app": "fake"}
    if ev["deleting"]:
        md["deletionTimestamp"] = rfc3339(ev["creation"] + 5)
    if ev["finalizers"]:
        md["finalizers"] = ["kwok.x-k8s.io/fake"] * ev["finalizers"]
    spec = {"nodeName": ev["node"], "containers": [{"name": n, "image": i} for n, i in ev["spec"]["containers"]]}
    if ev["spec"]["init"]:
        spec["initContainers"] = [{"name": n, "image": i} for n, i in ev["spec"]["init"]]
    if ev["spec"]["gates"]:
        spec["readinessGates"] = [{"conditionType": g} for g in ev["spec"]["gates"]]
    status = {}
    if ev["conforms"]:
        status = pod_status_like_template(ev, ev["creation"])
    elif ev["status_nonempty"]:
        status = {"qosClass": "BestEffort"}
    if ev["phase"]:
        status["phase"] = ev["phase"]
    if ev["hostIP"]:
        status["hostIP"] = ev["hostIP"]
    if ev["podIP"]:
        status["podIP"] = ev["podIP"]
        status["podIPs"] = [{"ip": ev["podIP"]}]
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec, "status": status}


def node_doc(ev):
    md = {"name": ev["name"], "annotations": {}}
    if ev["managed"]:
        md["annotations"]["kwok.x-k8s.io/node"] = "fake"
    if not ev["lockable"]:
        md["annotations"]["kwok.x-k8s.io/status"] = "custom"
    status = {"daemonEndpoints": {"kubeletEndpoint": {"Port": 0}}, "nodeInfo": dict(ev["nodeInfo"])}
    for k in ("addresses", "allocatable", "capacity"):
        if ev[k]:
            status[k] = ev[k]
    if ev["phase"]:
        status["phase"] = ev["phase"]
    return {"apiVersion": "v1", "kind": "Node", "metadata": md, "spec": {}, "status": status}


def json_node_batch(events, codec):
    """node_batch, but every upsert goes through JSON and the codec."""
    ups = [e for e in events if e["op"] != "delete"]
    b = codec.decode_nodes([json.dumps(node_doc(e), indent=1).encode() for e in ups])
    ar = abi.Arena()
    ar.buf = bytearray(b.buf)
    recs = np.zeros(len(events), abi.NODE_EVENT_DTYPE)
    k = 0
    for i, ev in enumerate(events):
        if ev["op"] == "delete":
            recs[i]["op"] = abi.OP_DELETE
            recs[i]["name"] = ar.ref(ev["name"])
        else:
            recs[i] = np.frombuffer(bytes(b.nodes[k]), abi.NODE_EVENT_DTYPE)[0]
            k += 1
    return recs, bytes(ar.buf)


def json_pod_batch(events, specs: SpecCache, codec):
    ups = [e for e in events if e["op"] != "delete"]
    b = codec.decode_pods([json.dumps(pod_doc(e)).encode() for e in ups])
    ar = abi.Arena()
    ar.buf = bytearray(b.buf)
    recs = np.zeros(len(events), abi.POD_EVENT_DTYPE)
    k = 0
    for i, ev in enumerate(events):
        if ev["op"] == "delete":  # watch.Deleted carries the last state: same record as pod_batch
            one, one_ar = pod_batch([ev], specs)
            base = len(ar.buf)
            ar.buf += one_ar
            for f in ("node_name", "host_ip", "pod_ip"):
                if one[0][f]["len"]:
                    one[0][f]["off"] += base
            recs[i] = one[0]
            continue
        d = b.pods[k]
        k += 1
        recs[i] = np.frombuffer(bytes(d.ev), abi.POD_EVENT_DTYPE)[0]
        recs[i]["handle"] = ev.get("handle", -1)  # the caller's object -> handle map
        spec = {"containers": [[b.text(c.name), b.text(c.image)] for c in d.containers[:d.n_containers]],
                "init": [[b.text(c.name), b.text(c.image)] for c in d.init_containers[:d.n_init_containers]],
                "gates": [b.text(g) for g in d.readiness_gates[:d.n_readiness_gates]]}
        recs[i]["spec_id"] = specs.get(spec)
    return recs, bytes(ar.buf)


def config_for(fx, **kw):
    c = fx["config"]
    return make_config(cidr=c["cidr"], node_ip=c["node_ip"], start_time=c["start_time"], buckets=c["buckets"],
                       node_slots_per_bucket=c["node_slots_per_bucket"],
                       pod_slots_per_bucket=c["pod_slots_per_bucket"], **kw)


def ingest_pods_mixed(backend, recs, arena, node_handle):
    """The batch in event order, every record the compact form can carry as
    kwok_pod_rec (kwok_ingest_pods_packed: its node by handle, node_handle maps
    names to the handles the node ingest returned) and the rest (a pod naming a
    node the engine holds no handle for) through kwok_ingest_pods, consecutive
    records of one form in one call: applying the calls in order is applying
    the batch.  Returns (handles, status, released) and the number of calls."""
    from kwok_amd.controller import ingest_pods_wire
    recs = recs.copy()
    for i in range(len(recs)):
        r = recs[i]
        if r["op"] == abi.OP_UPSERT and r["handle"] < 0 and r["node_handle"] < 0:
            name = bytes(arena[r["node_name"]["off"]:r["node_name"]["off"] + r["node_name"]["len"]]).decode()
            r["node_handle"] = node_handle.get(name, -1)
    hs, st, rel, calls = ingest_pods_wire(backend, recs, arena)
    return (hs, st, rel), calls


def replay(fx, backend, check=True, on_tick=None, codec=None, packed=False):
    """Replay a fixture through backend; assert equality tick by tick.  With a
    codec, events travel as Kubernetes JSON objects decoded by the host codec;
    packed: pods travel in the compact form where it can carry them
    (ingest_pods_mixed)."""
    specs = SpecCache(backend)
    node_handle = {}
    for ti, t in enumerate(fx["ticks"]):
        if t["node_events"]:
            recs, arena = json_node_batch(t["node_events"], codec) if codec else node_batch(t["node_events"])
            hs, st = backend.ingest_nodes_raw(recs, arena)
            for e, h, s_ in zip(t["node_events"], hs, st):
                if s_ == 0:
                    if e["op"] == "delete":
                        node_handle.pop(e["name"], None)
                    else:
                        node_handle[e["name"]] = int(h)
            if check:
                assert list(st) == [0] * len(st), (ti, list(st))
                assert list(hs) == [e["expect_handle"] for e in t["node_events"]], ti
        if t["pod_events"]:
            recs, arena = json_pod_batch(t["pod_events"], specs, codec) if codec else pod_batch(t["pod_events"], specs)
            if packed:
                (hs, st, _rel), _calls = ingest_pods_mixed(backend, recs, arena, node_handle)
            else:
                hs, st, _rel = backend.ingest_pods_raw(recs, arena)
            if check:
                assert list(st) == [0] * len(st), (ti, list(st))
                assert list(hs) == [e["expect_handle"] for e in t["pod_events"]], ti
        out = backend.tick(t["now"])
        if on_tick:
            on_tick(ti, t, out)
        if check:
            compare_tick(fx["name"], ti, t["expect"], out)
            c = fx["config"]
            exp_pods = {int(h): v for h, v in t["expect"]["pods"].items()}
            n = c["buckets"] * c["pod_slots_per_bucket"]
            used, phase, hip, pip = backend.dump_pods(0, n)
            got = {int(h): [abi.PHASE_NAMES[int(phase[h])], abi.ip4s(int(hip[h])), abi.ip4s(int(pip[h]))]
                   for h in np.nonzero(used)[0]}
            assert got == exp_pods, (fx["name"], ti)
    return True


def replay_queued(fx, backend):
    """Replay with every tick submitted before the previous one is collected
    (kwok_tick_submit / _collect); outputs must equal the plain replay's."""
    specs = SpecCache(backend)
    prev = None
    for ti, t in enumerate(fx["ticks"]):
        if t["node_events"]:
            recs, arena = node_batch(t["node_events"])
            backend.ingest_nodes_raw(recs, arena)
        if t["pod_events"]:
            recs, arena = pod_batch(t["pod_events"], specs)
            backend.ingest_pods_raw(recs, arena)
        backend.tick_submit(t["now"])
        if prev is not None:
            compare_tick(fx["name"], prev, fx["ticks"][prev]["expect"], backend.tick_collect())
        prev = ti
    compare_tick(fx["name"], prev, fx["ticks"][prev]["expect"], backend.tick_collect())
    return True


def compare_tick(name, ti, exp, out):
    where = "%s tick %d" % (name, ti)
    assert [list(d) for d in out.deletes] == exp["deletes"], where + " deletes"
    assert list(out.heartbeat_nodes) == exp["heartbeats"], where + " heartbeats"
    hb = exp["heartbeat_bytes"].encode()
    for i in range(len(out.heartbeat_nodes)):
        assert out.heartbeat_body(i) == hb, where + " heartbeat bytes #%d" % i
    assert [h for h, _ in out.node_inits] == [h for h, _ in exp["node_inits"]], where + " node_init handles"
    for (h, b), (_, e) in zip(out.node_inits, exp["node_inits"]):
        assert b == e.encode(), where + " node_init bytes %d\n got %r\nwant %r" % (h, b, e)
    assert [h for h, _ in out.pod_patches] == [h for h, _ in exp["pod_patches"]], where + " pod_patch handles"
    for (h, b), (_, e) in zip(out.pod_patches, exp["pod_patches"]):
        assert b == e.encode(), where + " pod_patch bytes %d\n got %r\nwant %r" % (h, b, e)
    for k, v in exp["counters"].items():
        assert out.counters[k] == v, where + " counter %s: got %d want %d" % (k, out.counters[k], v)
