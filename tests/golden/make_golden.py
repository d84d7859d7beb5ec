#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists; the GPU box only reads the JSON).

Three independent things are pinned here:

1. ``renderer_kat.json`` - the four byte-exact renderToJSON known-answer tests
   of the reference (pkg/kwok/controllers/renderer_test.go:32-67) replayed
   through ``gotmpl`` to show the mini renderer reproduces the reference
   renderer on the reference's own vectors.
2. ``render_cases.json`` - the reference's three default templates
   (pkg/kwok/controllers/templates/{node.heartbeat,node.status,pod.status}.tpl,
   read from /root/reference at generation time, never stored here) rendered
   over Go-shaped node/pod JSON documents, wrapped exactly like
   node_controller.go:388/398 and pod_controller.go:399.
3. ``ippool_cases.json`` and ``trace_*.json`` - the ipPool (utils.go:52-117)
   and the tick-level event-trace semantics (DESIGN.md "Tick contract"),
   restated here in Python with patch bytes produced by the template
   interpreter; the C oracle and the HIP engine must match these.

Usage: python tests/golden/make_golden.py  [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import datetime as _dt
import ipaddress
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gotmpl  # noqa: E402

TPL_DIR = "pkg/kwok/controllers/templates"

# ---------------------------------------------------------------------------
# Go-shaped documents (what json.Encode(corev1.Node / corev1.Pod) produces for
# the fields the templates read; renderer.go:65-75)
# ---------------------------------------------------------------------------
NODEINFO_KEYS = [  # sorted JSON key order == kwok_engine.h KWOK_NI_* order
    "architecture", "bootID", "containerRuntimeVersion", "kernelVersion",
    "kubeProxyVersion", "kubeletVersion", "machineID", "operatingSystem",
    "osImage", "systemUUID",
]


def rfc3339(unix):
    return _dt.datetime.fromtimestamp(unix, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def node_doc(n):
    status = {
        # NodeStatus.DaemonEndpoints / NodeInfo are structs: encoding/json
        # ignores omitempty on structs, so both are always present.
        "daemonEndpoints": {"kubeletEndpoint": {"Port": 0}},
        "nodeInfo": {k: n.get("nodeInfo", {}).get(k, "") for k in NODEINFO_KEYS},
    }
    if n.get("addresses"):
        status["addresses"] = n["addresses"]
    if n.get("allocatable"):
        status["allocatable"] = n["allocatable"]
    if n.get("capacity"):
        status["capacity"] = n["capacity"]
    if n.get("phase"):
        status["phase"] = n["phase"]
    return {"metadata": {"name": n["name"], "creationTimestamp": None}, "spec": {}, "status": status}


def pod_doc(p):
    spec = {"containers": [{"name": c, "image": i, "resources": {}} for c, i in p["spec"]["containers"]],
            "nodeName": p["node"]}
    if not spec["containers"]:
        del spec["containers"]
    if p["spec"].get("init"):
        spec["initContainers"] = [{"name": c, "image": i, "resources": {}} for c, i in p["spec"]["init"]]
    if p["spec"].get("gates"):
        spec["readinessGates"] = [{"conditionType": t} for t in p["spec"]["gates"]]
    status = {}
    if p.get("phase"):
        status["phase"] = p["phase"]
    if p.get("hostIP"):
        status["hostIP"] = p["hostIP"]
    if p.get("podIP"):
        status["podIP"] = p["podIP"]
    if p.get("status_nonempty") and not status:
        status["reason"] = "custom"
    md = {"name": p.get("key", "pod"), "namespace": "default",
          "creationTimestamp": rfc3339(p["creation"]) if p.get("creation") is not None else None}
    return {"metadata": md, "spec": spec, "status": status}


class Templates:
    def __init__(self, ref):
        rd = lambda f: open(os.path.join(ref, TPL_DIR, f)).read()
        self.hb = rd("node.heartbeat.tpl")
        # node_controller.go:101: nodeStatusTemplate = NodeStatusTemplate + "\n" + NodeHeartbeatTemplate
        self.node_init = rd("node.status.tpl") + "\n" + self.hb
        self.pod = rd("pod.status.tpl")


def wrap_status(patch):
    # json.Marshal(map[string]json.RawMessage{"status": patch})
    return '{"status":' + patch + "}"


def render_heartbeat(tpl, name, now, start, node_ip):
    f = {"Now": lambda: now, "StartTime": lambda: start, "NodeIP": lambda: node_ip}
    return wrap_status(gotmpl.render_to_json(tpl.hb, node_doc({"name": name}), f))


def render_node_init(tpl, n, now, start, node_ip):
    f = {"Now": lambda: now, "StartTime": lambda: start, "NodeIP": lambda: node_ip}
    return wrap_status(gotmpl.render_to_json(tpl.node_init, node_doc(n), f))


def render_pod(tpl, p, node_ip, pod_ip_fn):
    f = {"NodeIP": lambda: node_ip, "PodIP": pod_ip_fn, "Now": lambda: "X", "StartTime": lambda: "X"}
    return wrap_status(gotmpl.render_to_json(tpl.pod, pod_doc(p), f))


# ---------------------------------------------------------------------------
# ipPool restatement (utils.go:28-117) with the build's deterministic reuse
# rule: Get() takes the LOWEST usable address (the reference takes a random
# map key, utils.go:87-91).
# ---------------------------------------------------------------------------
class IPPool:
    def __init__(self, cidr):
        ip_s, _, plen = cidr.partition("/")
        self.base = int(ipaddress.IPv4Address(ip_s))          # parseCIDR keeps the host IP
        self.net = ipaddress.IPv4Network(cidr, strict=False)
        self.used, self.usable, self.index = set(), set(), 0

    def contains(self, s):
        if not s:
            return False
        return ipaddress.IPv4Address(s) in self.net

    def _new(self):
        while True:
            ip = str(ipaddress.IPv4Address(self.base + self.index))
            self.index += 1
            if ip in self.used:
                continue
            self.used.add(ip)
            self.usable.add(ip)
            return ip

    def get(self):
        if self.usable:
            ip = min(self.usable, key=lambda s: int(ipaddress.IPv4Address(s)))
        else:
            ip = self._new()
        self.usable.discard(ip)
        self.used.add(ip)
        return ip

    def put(self, ip):
        if not self.contains(ip):
            return
        self.used.discard(ip)
        self.usable.add(ip)

    def use(self, ip):
        if not self.contains(ip):
            return
        self.used.add(ip)


# ---------------------------------------------------------------------------
# Tick-level simulator: the build's deterministic tick contract.
# ---------------------------------------------------------------------------
def fnv1a32(s):
    h = 0x811C9DC5
    for b in s.encode():
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def node_conforms(n):
    """A.5: init patch is a no-op iff every templated default is already in place."""
    ni = n.get("nodeInfo", {})
    return bool(n.get("addresses")) and bool(n.get("allocatable")) and bool(n.get("capacity")) \
        and n.get("phase") == "Running" \
        and all(ni.get(k) for k in ("architecture", "kubeProxyVersion", "kubeletVersion", "operatingSystem")) \
        and ni.get("systemUUID", "") == ni.get("osImage", "")


class Sim:
    def __init__(self, cfg, tpl):
        self.cfg = cfg
        self.tpl = tpl
        self.B = cfg["buckets"]
        self.cn = cfg["node_slots_per_bucket"]
        self.cp = cfg["pod_slots_per_bucket"]
        self.pool = IPPool(cfg["cidr"])
        self.nodes = {}      # handle -> dict
        self.node_by_name = {}
        self.pods = {}       # handle -> dict
        self.start = rfc3339(cfg["start_time"])

    # -- slot policy: bucket = fnv1a32(node name) & (B-1); lowest free slot --
    def _alloc(self, table, bucket, cap):
        for i in range(cap):
            h = bucket * cap + i
            if h not in table:
                return h
        raise RuntimeError("bucket full")

    def _node_entry(self, name):
        h = self.node_by_name.get(name)
        if h is None:
            b = fnv1a32(name) & (self.B - 1)
            h = self._alloc(self.nodes, b, self.cn)
            self.nodes[h] = {"name": name, "exists": False, "managed": False, "lockable": False,
                             "event_lock": False, "refs": 0}
            self.node_by_name[name] = h
        return h

    def _maybe_free_node(self, h):
        n = self.nodes[h]
        if not n["exists"] and n["refs"] == 0:
            del self.node_by_name[n["name"]]
            del self.nodes[h]

    def ingest_node(self, ev):
        if ev["op"] == "delete":
            h = self.node_by_name.get(ev["name"])
            if h is None:
                return -1
            n = self.nodes[h]
            n.update(exists=False, managed=False, event_lock=False)
            self._maybe_free_node(h)
            return h
        h = self._node_entry(ev["name"])
        n = self.nodes[h]
        for k in ("addresses", "allocatable", "capacity", "phase", "nodeInfo"):
            n[k] = ev.get(k)
        n["exists"] = True
        if ev["managed"]:
            n["managed"] = True           # node_controller.go:259-260 (never cleared except Delete)
            if ev["lockable"]:
                n["event_lock"] = True     # :261-263
        n["lockable"] = bool(ev["lockable"])
        n["conforms"] = node_conforms(n)
        return h

    def ingest_pod(self, ev, handle=None):
        if ev["op"] == "delete":
            p = self.pods.pop(handle)
            nh = p["node_h"]
            # pod_controller.go:329-336: release on Deleted if node managed and IP in CIDR
            if self.nodes[nh]["managed"] and ev.get("podIP") and self.pool.contains(ev["podIP"]):
                self.pool.put(ev["podIP"])
            self.nodes[nh]["refs"] -= 1
            self._maybe_free_node(nh)
            return handle
        if handle is None:
            nh = self._node_entry(ev["node"])
            b = nh // self.cn
            handle = self._alloc(self.pods, b, self.cp)
            self.nodes[nh]["refs"] += 1
            p = {"node_h": nh, "event": False, "delete_pending": False}
            self.pods[handle] = p
        p = self.pods[handle]
        for k in ("key", "node", "disregard", "deleting", "finalizers", "creation", "phase",
                  "status_nonempty", "conforms", "hostIP", "podIP", "spec"):
            p[k] = ev.get(k)
        node = self.nodes[p["node_h"]]
        if p["deleting"]:
            if node["managed"]:          # pod_controller.go:306-308
                p["delete_pending"] = True
        elif node["managed"] and not p["disregard"]:   # needLockPod :252-269
            p["event"] = True
        return handle

    def tick(self, now_unix):
        now = rfc3339(now_unix)
        out = {"deletes": [], "heartbeats": [], "node_inits": [], "pod_patches": []}
        cnt = dict(heartbeat=0, node_init=0, pod_patch=0, delete=0, alloc=0, release=0,
                   evaluated=0, lock_checked=0)
        # 1. deletion phase (pod_controller.go:155-183): finalizer patch + delete, canonical order
        releases = []
        for h in sorted(self.pods):
            p = self.pods[h]
            if not p["delete_pending"]:
                continue
            out["deletes"].append([h, 1 if p["finalizers"] else 0])
            cnt["delete"] += 1
            nh = p["node_h"]
            del self.pods[h]
            if self.nodes[nh]["managed"] and p["podIP"] and self.pool.contains(p["podIP"]):
                releases.append(p["podIP"])
            self.nodes[nh]["refs"] -= 1
            self._maybe_free_node(nh)
        # node lock set: exists and (managed&lockable [heartbeat feedback] or event lock)
        lock_nodes = [h for h in sorted(self.nodes) if self.nodes[h]["exists"] and
                      ((self.nodes[h]["managed"] and self.nodes[h]["lockable"]) or self.nodes[h]["event_lock"])]
        relock = {h for h in lock_nodes if self.nodes[h]["managed"]}
        evaluated = [h for h in sorted(self.pods) if self.pods[h]["event"] or
                     (self.pods[h]["node_h"] in relock and not self.pods[h]["disregard"])]
        # 2. Uses (configurePod :378-382) of evaluated pods' existing IPs
        for h in evaluated:
            ip = self.pods[h]["podIP"]
            if ip and self.pool.contains(ip):
                self.pool.use(ip)
        # 3. Puts from this tick's deletions
        for ip in releases:
            self.pool.put(ip)
            cnt["release"] += 1
        # 4. heartbeat (node_controller.go:175-204) over managed nodes
        hb = render_heartbeat(self.tpl, "x", now, self.start, self.cfg["node_ip"])
        out["heartbeat_bytes"] = hb
        for h in sorted(self.nodes):
            if self.nodes[h]["managed"]:
                out["heartbeats"].append(h)
                cnt["heartbeat"] += 1
        # 5. node lock (node_controller.go:332-391)
        for h in lock_nodes:
            n = self.nodes[h]
            cnt["lock_checked"] += 1
            if not n["conforms"]:
                out["node_inits"].append([h, render_node_init(self.tpl, n, now, self.start, self.cfg["node_ip"])])
                cnt["node_init"] += 1
                ni = dict(n.get("nodeInfo") or {})
                for k, d in (("architecture", "amd64"), ("kubeProxyVersion", "fake"),
                             ("kubeletVersion", "fake"), ("operatingSystem", "linux")):
                    ni[k] = ni.get(k) or d
                ni["systemUUID"] = ni.get("osImage", "")
                n["nodeInfo"] = ni
                n["addresses"] = n.get("addresses") or [{"address": self.cfg["node_ip"], "type": "InternalIP"}]
                n["allocatable"] = n.get("allocatable") or {"cpu": "1k", "memory": "1Ti", "pods": "1M"}
                n["capacity"] = n.get("capacity") or {"cpu": "1k", "memory": "1Ti", "pods": "1M"}
                n["phase"] = "Running"
                n["conforms"] = True
            n["event_lock"] = False
        for n in self.nodes.values():
            n["event_lock"] = False
        # 6. pod evaluation (pod_controller.go:377-439) in canonical order
        for h in evaluated:
            p = self.pods[h]
            cnt["evaluated"] += 1
            got = []

            def pod_ip():
                ip = self.pool.get()
                got.append(ip)
                return ip

            patch = render_pod(self.tpl, p, self.cfg["node_ip"], pod_ip)
            need = p["phase"] != "Running" or not p["conforms"] or not p["hostIP"] or not p["podIP"]
            if got:
                cnt["alloc"] += 1
            assert need or not got
            if need:
                out["pod_patches"].append([h, patch])
                cnt["pod_patch"] += 1
                if p["status_nonempty"]:
                    p["hostIP"] = p["hostIP"] or self.cfg["node_ip"]
                    p["podIP"] = p["podIP"] or got[0]
                p["phase"] = "Running"
                p["conforms"] = True
                p["status_nonempty"] = True
            p["event"] = False
        for p in self.pods.values():
            p["event"] = False
        # fleet counters (after the tick)
        cnt["nodes_managed"] = sum(1 for n in self.nodes.values() if n["managed"])
        cnt["nodes_ready"] = sum(1 for n in self.nodes.values() if n["managed"] and n.get("conforms"))
        cnt["pods_total"] = len(self.pods)
        cnt["pods_pending"] = sum(1 for p in self.pods.values() if p["phase"] == "Pending")
        cnt["pods_running"] = sum(1 for p in self.pods.values() if p["phase"] == "Running")
        out["counters"] = cnt
        return out

    def dump_pods(self):
        return {h: [p["phase"] or "", p["hostIP"] or "", p["podIP"] or ""] for h, p in sorted(self.pods.items())}


# ---------------------------------------------------------------------------
# scenarios
# ---------------------------------------------------------------------------
S0 = 1704067200  # 2024-01-01T00:00:00Z


def base_cfg(**kw):
    c = dict(cidr="10.0.0.1/24", node_ip="196.168.0.1", start_time=S0, buckets=64,
             node_slots_per_bucket=8, pod_slots_per_bucket=64)
    c.update(kw)
    return c


def ne(name, managed=True, lockable=True, **kw):
    d = dict(op="upsert", name=name, managed=managed, lockable=lockable, phase="", addresses=None,
             allocatable=None, capacity=None, nodeInfo={})
    d.update(kw)
    return d


FAKE_SPEC = {"containers": [["fake-pod", "fake"]], "init": [], "gates": []}


def pe(key, node, **kw):
    d = dict(op="upsert", key=key, node=node, disregard=False, deleting=False, finalizers=0,
             creation=S0 - 60, phase="Pending", status_nonempty=True, conforms=False, hostIP="",
             podIP="", spec=FAKE_SPEC)
    d.update(kw)
    return d


def scenario_reference_node_test():
    """node_controller_test.go:38-154 restated as a trace (selector: name prefix 'node')."""
    caps = {"cpu": "4", "memory": "8Gi"}
    node0 = ne("node0", addresses=[{"address": "10.0.0.0", "type": "InternalIP"}], capacity=caps, allocatable=caps)
    other = ne("other-node", managed=False)
    ticks = [dict(nodes=[node0, other], pods=[])]
    # node1 = node0 after its lock patch, allocatable cpu 16 (test :120-129)
    node1 = ne("node1", addresses=[{"address": "10.0.0.0", "type": "InternalIP"}], capacity=caps,
               allocatable={"cpu": "16", "memory": "8Gi"}, phase="Running",
               nodeInfo={"architecture": "amd64", "kubeProxyVersion": "fake", "kubeletVersion": "fake",
                         "operatingSystem": "linux"})
    ticks.append(dict(nodes=[node1], pods=[]))
    ticks.append(dict(nodes=[], pods=[]))
    return base_cfg(node_ip="10.0.0.1"), ticks


def scenario_reference_pod_test():
    """pod_controller_test.go:38-193: pod0 on managed node0 (empty status), xxxx on an
    unmanaged node, pod1 gets the disregard annotation + custom status, then
    list.Items[0] gets a deletionTimestamp."""
    spec = {"containers": [["test-container", "test-image"]], "init": [], "gates": []}
    t0 = dict(nodes=[ne("node0")], pods=[
        pe("pod0", "node0", phase="", status_nonempty=False, spec=spec),
        pe("xxxx", "xxxx", phase="", status_nonempty=False, spec=spec)])
    t1 = dict(nodes=[], pods=[
        pe("pod1", "node0", phase="", status_nonempty=False, spec=spec),
        dict(pe("pod1", "node0", phase="", status_nonempty=True, disregard=True, spec=spec), modify=True)])
    t2 = dict(nodes=[], pods=[dict(op="delete_ts", key="pod0", node="node0", finalizers=0)])
    t3 = dict(nodes=[], pods=[])
    return base_cfg(node_ip="10.0.0.1", cidr="10.0.0.1/24"), [t0, t1, t2, t3]


def scenario_doc_known_answer():
    """site/content/en/docs/user/kwok-manage-nodes-and-pods.md:125-134: 10 pods on one
    node get 10.0.0.1..10.0.0.10."""
    pods = [pe("fake-pod-%d" % i, "kwok-node-0", spec={"containers": [["fake-container", "fake-image"]],
                                                        "init": [], "gates": []}) for i in range(10)]
    return base_cfg(), [dict(nodes=[ne("kwok-node-0")], pods=pods), dict(nodes=[], pods=[])]


def scenario_cidr_overflow():
    """/24: fresh index 255 leaves the CIDR (utils.go:68-81 ignores the bound);
    out-of-CIDR IPs are never recycled (Put is a no-op), in-CIDR ones are reused
    lowest-first."""
    pods = [pe("p%03d" % i, "n0") for i in range(260)]
    t0 = dict(nodes=[ne("n0")], pods=pods)
    # delete (via deletionTimestamp) p005, p100, p256 (out of CIDR), p258 (out of CIDR)
    dels = []
    for k in (5, 100, 256, 258):
        ip = str(ipaddress.IPv4Address(int(ipaddress.IPv4Address("10.0.0.1")) + k))
        dels.append(dict(pe("p%03d" % k, "n0", deleting=True, finalizers=(k % 2), phase="Running",
                            conforms=True, hostIP="196.168.0.1", podIP=ip), modify=True))
    t1 = dict(nodes=[], pods=dels)
    t2 = dict(nodes=[], pods=[pe("q%d" % i, "n0") for i in range(5)])
    return base_cfg(cidr="10.0.0.1/24", pod_slots_per_bucket=512), [t0, t1, t2, dict(nodes=[], pods=[])]


def scenario_specs():
    """Template branches: no containers (containerStatuses null), init containers,
    readiness gates, existing hostIP/podIP, empty status, partial nodeInfo
    (systemUUID <- osImage, node.status.tpl:40), non-Running node phase."""
    nodes = [ne("alpha", phase="Pending", nodeInfo={"osImage": "ubuntu", "architecture": "arm64",
                                                     "kernelVersion": "v5-10"}),
             ne("beta", managed=True, lockable=False),
             ne("gamma", addresses=[{"address": "192.168.1.7", "type": "InternalIP"},
                                    {"address": "gamma", "type": "Hostname"}])]
    specs = [
        {"containers": [], "init": [], "gates": []},
        {"containers": [["a", "img-a"], ["b", "registry.local/img-b:v1"]], "init": [["init", "busybox"]],
         "gates": ["example.com/gate"]},
        {"containers": [["c", "nginx"]], "init": [["i1", "x"], ["i2", "yy"]], "gates": []},
    ]
    pods = [
        pe("s0", "alpha", spec=specs[0]),
        pe("s1", "alpha", spec=specs[1]),
        pe("s2", "gamma", spec=specs[2], hostIP="172.16.0.9"),
        pe("s3", "gamma", spec=specs[1], podIP="10.0.0.200"),  # existing in-CIDR IP -> Use
        pe("s4", "gamma", phase="", status_nonempty=False, spec=specs[2]),
        pe("s5", "beta", spec=specs[0]),     # node not lockable: locked only by its event
        pe("s6", "gamma", disregard=True),   # disregarded: never evaluated
        pe("s7", "alpha", phase="Running", conforms=True, hostIP="196.168.0.1", podIP="10.0.0.50"),
        pe("s8", "alpha", phase="Succeeded", conforms=True, hostIP="196.168.0.1", podIP="10.0.0.51"),
        pe("s9", "gamma", creation=S0 + 86400 * 400 + 3723),
    ]
    return base_cfg(cidr="10.0.0.1/24"), [dict(nodes=nodes, pods=pods), dict(nodes=[], pods=[]),
                                          dict(nodes=[], pods=[])]


def scenario_churn(seed=0x6B776F6B, n_nodes=24, ticks=8):
    """Mixed churn: creates, deletionTimestamp deletes (with/without finalizers),
    external Deleted events (release at ingest), node flap (delete + re-create),
    annotation-managed subset, disregard, existing/duplicate IPs."""
    rng = random.Random(seed)
    cfg = base_cfg(cidr="10.0.0.1/26", buckets=16, node_slots_per_bucket=8, pod_slots_per_bucket=64)
    names = ["node-%07d" % i for i in range(n_nodes)]
    managed = {n: rng.random() < 0.7 for n in names}
    out = []
    live = {}  # key -> node
    seq = 0
    first = dict(nodes=[ne(n, managed=managed[n], lockable=rng.random() > 0.1) for n in names], pods=[])
    for _ in range(60):
        n = rng.choice(names)
        k = "pod-%08d" % seq
        seq += 1
        live[k] = n
        first["pods"].append(pe(k, n, phase=rng.choice(["Pending", "Pending", ""]),
                                status_nonempty=True, finalizers=rng.randint(0, 1)))
    out.append(first)
    for t in range(1, ticks):
        tk = dict(nodes=[], pods=[])
        # flap one node
        if t % 3 == 0:
            n = rng.choice(names)
            tk["nodes"].append(dict(op="delete", name=n))
            tk["nodes"].append(ne(n, managed=managed[n]))
        # deletions via deletionTimestamp (IP carried from the sim's view is filled in by the harness)
        for k in rng.sample(sorted(live), min(len(live), rng.randint(3, 10))):
            n = live.pop(k)
            ext = rng.random() < 0.3
            tk["pods"].append(dict(op="delete_ts" if not ext else "delete_ext", key=k, node=n,
                                   finalizers=rng.randint(0, 1)))
        for _ in range(rng.randint(5, 15)):
            n = rng.choice(names)
            k = "pod-%08d" % seq
            seq += 1
            live[k] = n
            ip = ""
            if rng.random() < 0.1:
                ip = "10.0.0.%d" % rng.randint(1, 63)  # pre-existing IP (restart) -> Use, maybe duplicate
            tk["pods"].append(pe(k, n, podIP=ip, disregard=rng.random() < 0.05,
                                 finalizers=rng.randint(0, 1)))
        out.append(tk)
    return cfg, out


def scenario_e2e_kwok_test(tpl):
    """test/kwok/kwok.test.sh restated as a trace, with the deployment's flags
    (kustomize/kwok/kwok-deployment.yaml:22-29: annotation selector
    kwok.x-k8s.io/node=fake, disregard kwok.x-k8s.io/status=custom, CIDR
    10.0.0.1/24) and its objects (test/kwok/fake-node.yaml, fake-deployment.yaml:
    5 replicas of fake-container / fake on fake-node):
      t0  test_node_ready / test_pod_running (:39-73): fake-node is initialised and
          heartbeats; the 5 pods go Running with 10.0.0.1..5;
      t1  test_modify_node_status (:76-89): the node gets the disregard annotation,
          then a status patch nodeInfo.kubeletVersion = fake-new: heartbeats go on,
          no init patch overwrites the status;
      t2  test_modify_pod_status (:92-104): the first pod gets the disregard
          annotation, then a status patch podIP = 192.168.0.1: it is not patched
          again and keeps that podIP;
      t3  a steady tick."""
    node_ip = "10.244.0.7"  # --node-ip=$(POD_IP): the kwok pod's address
    spec = {"containers": [["fake-container", "fake"]], "init": [], "gates": []}
    pods = [pe("fake-pod-7d4b9c5f8d-%s" % s, "fake-node", spec=spec) for s in ("2xkqp", "8hz4w", "c6rnm", "lt9vb", "x5w7j")]
    t0 = dict(nodes=[ne("fake-node")], pods=pods)
    # the node's status after its init patch (node.status.tpl), then the user's edit
    init = json.loads(render_node_init(tpl, ne("fake-node"), rfc3339(S0 + 30), rfc3339(S0), node_ip))["status"]
    st = dict(addresses=init["addresses"], allocatable=init["allocatable"], capacity=init["capacity"],
              phase=init["phase"], nodeInfo=dict(init["nodeInfo"]))
    edited = dict(st, nodeInfo=dict(st["nodeInfo"], kubeletVersion="fake-new"))
    t1 = dict(nodes=[ne("fake-node", lockable=False, **st), ne("fake-node", lockable=False, **edited)], pods=[])
    first = pods[0]["key"]
    running = dict(phase="Running", conforms=True, hostIP=node_ip, podIP="10.0.0.1", spec=spec)
    t2 = dict(nodes=[], pods=[dict(pe(first, "fake-node", disregard=True, **running), modify=True),
                              dict(pe(first, "fake-node", disregard=True, **dict(running, podIP="192.168.0.1")),
                                   modify=True)])
    return base_cfg(node_ip=node_ip, cidr="10.0.0.1/24"), [t0, t1, t2, dict(nodes=[], pods=[])]


def scenario_same_interval_echo(tpl):
    """The reference's in-interval IP for a pod created with an empty status
    (pod_controller.go:279-319, 404-439): configurePod renders pod.status.tpl
    with no `.status`, so the first patch carries no hostIP / podIP; the patch's
    own Modified event re-enters lockPodChan within the same interval, and the
    second configurePod renders `{{ with .status }}` with NodeIP and
    ipPool.Get().  The engine does not re-ingest the echo of its own patch
    (contract point); a caller that wants the reference's timing
    ingests the echo and ticks again at the same clock (t1 here, `same_now`).
      t0  e0, e1 (empty status) and r0 (Pending, non-empty) on node n0: e0/e1
          patched without IPs, r0 gets 10.0.0.1;
      t1  same clock: the echoes of e0 / e1 (Running, conforming status, no IPs):
          patched with NodeIP and 10.0.0.2 / 10.0.0.3 - the bytes and IPs the
          reference's second in-interval configurePod produces;
      t2  a steady tick."""
    spec = {"containers": [["c", "img"]], "init": [], "gates": []}
    t0 = dict(nodes=[ne("n0")], pods=[pe("e0", "n0", phase="", status_nonempty=False, spec=spec),
                                      pe("e1", "n0", phase="", status_nonempty=False, spec=spec),
                                      pe("r0", "n0", spec=spec)])
    echo = dict(phase="Running", status_nonempty=True, conforms=True, hostIP="", podIP="", spec=spec)
    t1 = dict(nodes=[], pods=[dict(pe("e0", "n0", **echo), modify=True), dict(pe("e1", "n0", **echo), modify=True)],
              same_now=True)
    return base_cfg(node_ip="10.0.0.254", cidr="10.0.0.1/24"), [t0, t1, dict(nodes=[], pods=[])]


def run_scenario(name, cfg, ticks, tpl):
    sim = Sim(cfg, tpl)
    handles = {}
    fx = {"name": name, "config": cfg, "ticks": []}
    now = cfg["start_time"]
    for i, tk in enumerate(ticks):
        if not tk.get("same_now"):
            now += 30
        rec = {"now": now, "node_events": [], "pod_events": []}
        for ev in tk["nodes"]:
            h = sim.ingest_node(ev)
            rec["node_events"].append(dict(ev, expect_handle=h))
        for ev in tk["pods"]:
            ev = dict(ev)
            op = ev.pop("op")
            if op in ("delete_ts", "delete_ext"):
                h = handles[ev["key"]]
                cur = sim.pods[h]
                full = {k: cur[k] for k in ("key", "node", "disregard", "creation", "phase",
                                             "status_nonempty", "conforms", "hostIP", "podIP", "spec")}
                full["finalizers"] = ev["finalizers"]
                if op == "delete_ts":
                    full.update(op="upsert", deleting=True)
                    sim.ingest_pod(full, h)
                    rec["pod_events"].append(dict(full, handle=h, expect_handle=h))
                else:
                    full.update(op="delete", deleting=False)
                    sim.ingest_pod(full, h)
                    del handles[ev["key"]]
                    rec["pod_events"].append(dict(full, handle=h, expect_handle=h))
                continue
            ev["op"] = op
            modify = ev.pop("modify", False)
            h = handles.get(ev["key"]) if modify else None
            h2 = sim.ingest_pod(ev, h)
            if not modify:
                handles[ev["key"]] = h2
            rec["pod_events"].append(dict(ev, handle=(h if modify else -1), expect_handle=h2))
        res = sim.tick(now)
        for h, _ in res["deletes"]:
            for k, v in list(handles.items()):
                if v == h:
                    del handles[k]
        rec["expect"] = res
        rec["expect"]["pods"] = {str(h): v for h, v in sim.dump_pods().items()}
        fx["ticks"].append(rec)
    return fx


# ---------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    tpl = Templates(args.ref)

    # 1. renderer_test.go:32-67 known answers
    kat = [
        dict(name="basic", tmpl='{"k":{{ .k }}}', data={"k": "v1"}, funcs={}, expected='{"k":"v1"}'),
        dict(name="basic with yaml format", tmpl="k: {{ .k }}", data={"k": "v1"}, funcs={}, expected='{"k":"v1"}'),
        dict(name="with funcMap", tmpl='{"foo":{{ Foo }},"k":{{ .k }}}', data={"k": "v1"},
             funcs={"Foo": "foo"}, expected='{"foo":"foo","k":"v1"}'),
        dict(name="with whitespace", tmpl='        {"foo":{{ Foo }},"k":{{ .k }}}       ', data={"k": "v1"},
             funcs={"Foo": "foo"}, expected='{"foo":"foo","k":"v1"}'),
    ]
    for c in kat:
        fns = {k: (lambda v=v: v) for k, v in c["funcs"].items()}
        got = gotmpl.render_to_json(c["tmpl"], c["data"], fns)
        assert got == c["expected"], (c["name"], got)
    json.dump(kat, open(os.path.join(HERE, "renderer_kat.json"), "w"), indent=1)

    # 2. render cases
    T, S = rfc3339(S0 + 30), rfc3339(S0)
    cases = []
    cases.append(dict(kind="heartbeat", now=S0 + 30, start=S0, node_ip="196.168.0.1",
                      expected=render_heartbeat(tpl, "node-0000000", T, S, "196.168.0.1")))
    node_inputs = [
        dict(name="empty", node=ne("node-0000000")),
        dict(name="ref-node0", node=ne("node0", addresses=[{"address": "10.0.0.0", "type": "InternalIP"}],
                                       capacity={"cpu": "4", "memory": "8Gi"},
                                       allocatable={"cpu": "4", "memory": "8Gi"})),
        dict(name="partial-nodeinfo", node=ne("n", phase="Pending",
                                              nodeInfo={"osImage": "ubuntu", "kubeletVersion": "v1.26.0",
                                                        "bootID": "b-1"})),
    ]
    for ni in node_inputs:
        for node_ip in ("196.168.0.1", "10.0.0.1"):
            cases.append(dict(kind="node_init", label=ni["name"], node=ni["node"], now=S0 + 30, start=S0,
                              node_ip=node_ip, expected=render_node_init(tpl, ni["node"], T, S, node_ip)))
    pod_inputs = [
        dict(name="pending-alloc", pod=pe("p", "n"), alloc="10.0.0.1"),
        dict(name="pending-alloc-15", pod=pe("p", "n"), alloc="255.255.255.254"),
        dict(name="empty-status", pod=pe("p", "n", phase="", status_nonempty=False), alloc=None),
        dict(name="existing-ips", pod=pe("p", "n", hostIP="1.2.3.4", podIP="10.9.8.7"), alloc=None),
        dict(name="no-containers", pod=pe("p", "n", spec={"containers": [], "init": [], "gates": []}),
             alloc="10.0.0.2"),
        dict(name="init-and-gates", pod=pe("p", "n", spec={"containers": [["a", "img-a"], ["b", "img/b:v1"]],
                                                           "init": [["i", "busybox"]], "gates": ["x.io/g", "gate-y"]}),
             alloc="10.0.0.3"),
        dict(name="ts-2025", pod=pe("p", "n", creation=S0 + 366 * 86400 + 45296), alloc="10.0.0.4"),
    ]
    for pi in pod_inputs:
        for node_ip in ("196.168.0.1", "10.0.0.1"):
            a = pi["alloc"]
            cases.append(dict(kind="pod", label=pi["name"], pod=pi["pod"], node_ip=node_ip, alloc=a,
                              expected=render_pod(tpl, pi["pod"], node_ip, lambda: a)))
    json.dump(cases, open(os.path.join(HERE, "render_cases.json"), "w"), indent=1)

    # 3a. ipPool op sequences
    ipc = []
    for cidr, ops in [
        ("10.0.0.1/24", ["get"] * 10),                                             # doc known answer
        ("10.0.0.1/24", ["get"] * 257 + ["put:10.0.0.7", "put:10.0.1.0", "put:10.0.0.3", "get", "get", "get"]),
        ("10.0.0.1/24", ["use:10.0.0.2", "use:10.0.0.3", "get", "get", "use:10.9.0.1", "get"]),
        ("10.0.0.1/24", ["get", "get", "put:10.0.0.1", "use:10.0.0.1", "get", "get"]),  # Use keeps usable
        ("192.168.5.77/30", ["get"] * 6 + ["put:192.168.5.77", "put:192.168.5.76", "get", "get"]),
    ]:
        pool = IPPool(cidr)
        res = []
        for op in ops:
            if op == "get":
                res.append(pool.get())
            elif op.startswith("put:"):
                pool.put(op[4:])
                res.append(None)
            else:
                pool.use(op[4:])
                res.append(None)
        ipc.append(dict(cidr=cidr, ops=ops, results=res))
    json.dump(ipc, open(os.path.join(HERE, "ippool_cases.json"), "w"), indent=1)

    # 3b. traces
    for name, fn in [("reference_node_test", scenario_reference_node_test),
                     ("reference_pod_test", scenario_reference_pod_test),
                     ("doc_known_answer", scenario_doc_known_answer),
                     ("cidr_overflow", scenario_cidr_overflow),
                     ("specs", scenario_specs),
                     ("churn", scenario_churn),
                     ("e2e_kwok_test", lambda: scenario_e2e_kwok_test(tpl)),
                     ("same_interval_echo", lambda: scenario_same_interval_echo(tpl))]:
        cfg, ticks = fn()
        fx = run_scenario(name, cfg, ticks, tpl)
        json.dump(fx, open(os.path.join(HERE, "trace_%s.json" % name), "w"), indent=None, separators=(",", ":"))
        print("wrote trace_%s.json (%d ticks)" % (name, len(fx["ticks"])))


if __name__ == "__main__":
    main()
