"""The drop-in controller (kwok_amd/controller.py, the Python restatement of
integration/go/.../gpu_controller.go) against a fake clientset, with the CPU
oracle as its backend: the reference's own unit tests
(node_controller_test.go:37-155, pod_controller_test.go:37-194) restated
through the drop-in, and the echo contract - the watch echoes of the engine's
own patches are dropped by resourceVersion, and dropping them changes no call
the controller makes."""
import time

import pytest

from fake_clientset import FakeClientset
from kwok_amd.controller import Config, Controller
from oracle.oracle import Oracle

MANAGE = "kwok.x-k8s.io/node=fake"
S0 = 1704067200


def node(name, managed=True, status=None, labels=None):
    md = {"name": name, "annotations": {"kwok.x-k8s.io/node": "fake"} if managed else {}}
    if labels:
        md["labels"] = labels
    st = {"daemonEndpoints": {"kubeletEndpoint": {"Port": 0}}, "nodeInfo": {}}
    st.update(status or {})
    return {"apiVersion": "v1", "kind": "Node", "metadata": md, "spec": {}, "status": st}


def pod(name, node_name, creation=S0 - 60, status=None, containers=(("test-container", "test-image"),), **md):
    m = {"name": name, "namespace": "default", "creationTimestamp": time.strftime("%Y-%m-%dT%H:%M:%SZ",
                                                                                  time.gmtime(creation))}
    m.update(md)
    return {"apiVersion": "v1", "kind": "Pod", "metadata": m,
            "spec": {"nodeName": node_name, "containers": [{"name": n, "image": i} for n, i in containers]},
            "status": status or {}}


SMALL = dict(buckets=64, node_slots_per_bucket=32, pod_slots_per_bucket=512, pod_handle_stride=0, max_pod_specs=64)


BACKEND = Oracle  # tests/test_controller_gpu.py runs the reference tests with the HIP engine


def controller(cs, suppress=True, backend=None, geometry=SMALL, **kw):
    conf = Config(client_set=cs, **kw)
    c = Controller(conf, backend=backend or BACKEND, suppress_echoes=suppress, geometry=geometry)
    c.start()
    return c


def test_reference_node_controller():
    """node_controller_test.go:38-154 through the drop-in: node0's allocatable
    survives the init patch, a created node1 is managed (Size 2) and keeps its
    own cpu, managed nodes end Running and the unmanaged one does not."""
    res = {"cpu": "4", "memory": "8Gi"}
    cs = FakeClientset(node("node0", status={"addresses": [{"type": "InternalIP", "address": "10.0.0.0"}],
                                             "capacity": dict(res), "allocatable": dict(res)}),
                       node("other-node", managed=False))
    c = controller(cs, manage_nodes_with_annotation_selector=MANAGE, node_ip="10.0.0.1")
    c.step(S0 + 30)
    node0 = cs.get("nodes", "node0")
    assert node0["status"]["allocatable"]["cpu"] == "4"
    assert node0["status"]["addresses"] == [{"type": "InternalIP", "address": "10.0.0.0"}]
    node1 = dict(node0, metadata={"name": "node1", "annotations": node0["metadata"]["annotations"]})
    node1["status"] = dict(node0["status"], allocatable={"cpu": "16", "memory": "8Gi"})
    cs.create(node1)
    c.step(S0 + 60)
    assert c.size() == 2 and c.has("node0") and c.has("node1") and not c.has("other-node")
    assert cs.get("nodes", "node1")["status"]["allocatable"]["cpu"] == "16"
    for n in cs.list("nodes"):
        running = n["status"].get("phase") == "Running"
        assert running == (n["metadata"]["name"] != "other-node"), n["metadata"]["name"]
        if running:  # heartbeat conditions at the last tick's clock
            cond = {x["type"]: x for x in n["status"]["conditions"]}
            assert cond["Ready"]["status"] == "True" and cond["Ready"]["lastHeartbeatTime"] == "2024-01-01T00:01:00Z"
    c.close()


def test_reference_pod_controller():
    """pod_controller_test.go:38-193 through the drop-in: pod0 on a managed
    node, xxxx on an unmanaged one; pod1 created then given the disregard
    annotation and a custom status.reason (kept); list.Items[0] gets a
    deletionTimestamp and is deleted; pods on managed nodes end Running."""
    cs = FakeClientset(node("node0"), pod("pod0", "node0"), pod("xxxx", "xxxx"))
    c = controller(cs, manage_nodes_with_annotation_selector=MANAGE, node_ip="10.0.0.1", cidr="10.0.0.1/24",
                   disregard_status_with_annotation_selector="fake=custom")
    cs.create(pod("pod1", "node0"))
    p1 = cs.get("pods", ("default", "pod1"))
    p1["metadata"]["annotations"] = {"fake": "custom"}
    p1["status"]["reason"] = "custom"
    cs.update(p1)
    c.step(S0 + 30)
    assert cs.get("pods", ("default", "pod1"))["status"]["reason"] == "custom"
    assert len(cs.list("pods")) == 3
    p0 = cs.get("pods", ("default", "pod0"))
    p0["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:40Z"
    cs.update(p0)
    c.step(S0 + 60)
    c.step(S0 + 90)
    pods = {p["metadata"]["name"]: p for p in cs.list("pods")}
    assert sorted(pods) == ["pod1", "xxxx"]
    assert pods["pod1"]["status"]["phase"] == "Running"
    assert pods["xxxx"]["status"].get("phase") != "Running"
    c.close()


def scenario(cs, c, ticks=5, nodes=20, pods_per_node=4, seed=3, fin_frac=0.3):
    """nodes and pods created, modified, deleted between ticks; returns the
    clientset's write calls per tick"""
    import random
    rng = random.Random(seed)
    for i in range(nodes):
        cs.create(node("node-%03d" % i, managed=i % 5 != 4))
    live, k = [], 0
    per_tick = []
    for t in range(ticks):
        for _ in range(nodes * pods_per_node // ticks):
            status = {"phase": "Pending"} if rng.random() < 0.8 else {}
            fin = ["kwok.x-k8s.io/x"] if rng.random() < fin_frac else []
            p = pod("pod-%05d" % k, "node-%03d" % rng.randrange(nodes), status=status)
            if fin:
                p["metadata"]["finalizers"] = fin
            cs.create(p)
            live.append(p["metadata"]["name"])
            k += 1
            if rng.random() < 0.1:  # Added + Modified in one interval
                q = cs.get("pods", ("default", live[-1]))
                q["metadata"].setdefault("labels", {})["touched"] = "yes"
                cs.update(q)
            if rng.random() < 0.05:  # Added + Deleted in one interval
                cs.delete("pods", ("default", live.pop()))
        for name in rng.sample(live, min(len(live), 3)):  # deletion requested
            q = cs.get("pods", ("default", name))
            q["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:10Z"
            cs.update(q)
            live.remove(name)
        if t == 2:  # an external status change: not an echo, ingested
            q = cs.get("nodes", "node-000")
            q["status"]["phase"] = "Pending"
            cs.update(q)
        n0 = len(cs.calls)
        c.step(S0 + 30 * (t + 1))
        if cs.deliver == "queued":
            cs.pump()
        per_tick.append(cs.calls[n0:])
    return per_tick


@pytest.mark.parametrize("deliver", ["sync", "queued"])
def test_echoes_dropped_and_change_nothing(deliver):
    """With echo suppression the controller ingests only the cluster's own
    events; without it every patch's echo goes back through the codec and the
    engine.  Every write call (PatchStatus / Patch / Delete with its body) is
    the same in both runs, tick by tick.  deliver=sync: echoes overtake their
    patch's response (dropped at the next tick's flush); queued: they arrive
    after it (dropped on arrival).  No finalizers here: the echo of a pod's
    finalizer patch is the one echo whose ingest is NOT harmless - the engine
    already deleted the pod and released its podIP, so re-ingesting the echo
    (a pod holding that address) and its Deleted event would release the address
    a second time while another pod holds it (test_finalizer_patch_echo_is_dropped)."""
    runs = {}
    for sup in (True, False):
        cs = FakeClientset(deliver=deliver)
        c = controller(cs, suppress=sup, manage_nodes_with_annotation_selector=MANAGE, cidr="10.0.0.1/24")
        runs[sup] = (scenario(cs, c, fin_frac=0.0), c.stats, {k: v["status"] for k, v in cs.store["pods"].items()})
        c.close()
    (a, sa, pa), (b, sb, pb) = runs[True], runs[False]
    assert [len(x) for x in a] == [len(x) for x in b]
    for t, (x, y) in enumerate(zip(a, b)):
        assert x == y, "tick %d" % t
    assert pa == pb
    dropped = sa.echoes_on_arrival + sa.echoes_at_flush
    assert dropped > 0 and sb.echoes_on_arrival + sb.echoes_at_flush == 0
    assert (sa.echoes_on_arrival > 0) == (deliver == "queued")
    assert (sa.echoes_at_flush > 0) == (deliver == "sync")
    # suppressed: the heartbeat echoes (one per managed node per tick) never reach the engine
    assert sb.node_records - sa.node_records >= 16 * 4
    assert sb.pod_records > sa.pod_records
    # pods on managed nodes ended Running with IPs
    assert sum(1 for st in pa.values() if st.get("phase") == "Running" and st.get("podIP")) > 0


@pytest.mark.parametrize("deliver", ["sync", "queued"])
def test_finalizer_patch_echo_is_dropped(deliver):
    """DeletePod of a pod with finalizers (pod_controller.go:155-183): the
    finalizer patch's echo (deletionTimestamp, no finalizers) is dropped - the
    engine already deleted the pod - so no second Delete is ever issued, and the
    Deleted event forgets the pod's echoes.  (The controller forgets a deleted
    pod's echoes before its apply notes the finalizer patch's: the Go drop-in does
    so in the tick callback, ahead of the concurrent task.)"""
    cs = FakeClientset(node("n0"), deliver=deliver)
    c = controller(cs, manage_nodes_with_annotation_selector=MANAGE, cidr="10.0.0.1/24")
    cs.create(pod("a", "n0", status={"phase": "Pending"}, finalizers=["x.io/f"]))
    cs.create(pod("b", "n0", status={"phase": "Pending"}))
    c.step(S0 + 30)
    cs.pump()
    uids = [cs.get("pods", ("default", name))["metadata"]["uid"] for name in ("a", "b")]
    for name in ("a", "b"):  # kubectl delete: deletionTimestamp set, finalizers kept
        q = cs.get("pods", ("default", name))
        q["metadata"]["deletionTimestamp"] = "2024-01-01T00:01:00Z"
        cs.update(q)
    cs.pump()
    n0 = len(cs.calls)
    d0 = c.stats.echoes_on_arrival + c.stats.echoes_at_flush
    c.step(S0 + 60)
    cs.pump()
    calls = [(v, k) for v, kind, k, _ in cs.calls[n0:] if kind == "pods"]
    assert calls == [("patch_merge", ("default", "a")), ("delete", ("default", "a")), ("delete", ("default", "b"))]
    for t in range(2):
        n1 = len(cs.calls)
        c.step(S0 + 90 + 30 * t)
        cs.pump()
        assert not [x for x in cs.calls[n1:] if x[1] == "pods"], "tick %d: pod calls after the deletes" % t
    assert c.stats.echoes_on_arrival + c.stats.echoes_at_flush >= d0 + 1  # the finalizer patch's echo
    assert cs.list("pods") == [] and not any(u in c.echo.rv for u in uids)  # forgotten at their Deleted events
    c.close()


def empty_status_scenario(cs, c):
    """pods created with an empty status next to Pending ones; returns the pod
    write calls of each of three steps"""
    cs.create(node("n0"))
    cs.create(node("n1", managed=False))
    c.step(S0 + 30)
    cs.pump()
    cs.create(pod("e0", "n0"))
    cs.create(pod("r0", "n0", status={"phase": "Pending"}))
    cs.create(pod("e1", "n0", containers=(("a", "img-a"), ("b", "img-b"))))
    cs.create(pod("u0", "n1"))  # unmanaged node: never patched
    cs.pump()
    per = []
    for t in range(3):
        n0 = len(cs.calls)
        c.step(S0 + 60 + 30 * t)
        cs.pump()
        per.append([x for x in cs.calls[n0:] if x[1] == "pods"])
    return per


@pytest.mark.parametrize("deliver", ["sync", "queued"])
def test_empty_status_pod_gets_its_ip_in_the_same_interval(deliver):
    """pod_controller.go:279-319 with pod.status.tpl's `{{ with .status }}`: a
    pod created with an empty status is patched without hostIP / podIP; that
    patch's Modified event re-enters lockPodChan and the second configurePod,
    in the same interval, renders NodeIP and a pool address.  The drop-in
    ingests the patch's returned object and ticks again at the same clock: both
    patches land in one step, the IPs follow the pool order of the reference
    (r0 in the first pass, e0 / e1 in the second), the echoes of both patches
    are dropped and the next steps write nothing."""
    cs = FakeClientset(deliver=deliver)
    c = controller(cs, manage_nodes_with_annotation_selector=MANAGE, node_ip="10.0.0.254", cidr="10.0.0.1/24")
    per = empty_status_scenario(cs, c)
    names = [k[1] for _, _, k, _ in per[0]]
    assert names == ["e0", "r0", "e1", "e0", "e1"], names
    first, second = per[0][0][3], per[0][3][3]
    assert b'"podIP"' not in first and b'"hostIP"' not in first
    assert b'"hostIP":"10.0.0.254"' in second and b'"podIP":"10.0.0.2"' in second
    assert per[1] == [] and per[2] == []
    st = {p["metadata"]["name"]: p["status"] for p in cs.list("pods")}
    assert (st["e0"]["podIP"], st["r0"]["podIP"], st["e1"]["podIP"]) == ("10.0.0.2", "10.0.0.1", "10.0.0.3")
    assert all(st[k]["phase"] == "Running" and st[k]["hostIP"] == "10.0.0.254" for k in ("e0", "r0", "e1"))
    assert st["u0"] == {}
    assert c.stats.reentered == 2
    c.close()


def test_runs_for_added_modified_deleted_in_one_batch():
    """flushPods' cut: a new pod's second event needs its handle, so the batch
    is ingested in runs; Added + Deleted leaves no pod and releases nothing it
    does not hold; Added + Modified is one pod, patched once."""
    cs = FakeClientset(node("n0"))
    c = controller(cs, manage_nodes_with_annotation_selector=MANAGE, cidr="10.0.0.1/24")
    c.step(S0 + 30)
    cs.create(pod("a", "n0", status={"phase": "Pending"}))
    cs.create(pod("b", "n0", status={"phase": "Pending"}))
    q = cs.get("pods", ("default", "a"))
    q["metadata"]["labels"] = {"x": "y"}
    cs.update(q)
    cs.delete("pods", ("default", "b"))
    cs.create(pod("c", "n0", status={"phase": "Pending"}))
    n0 = len(cs.calls)
    c.step(S0 + 60)
    assert c.stats.pod_runs >= 2
    pods = {p["metadata"]["name"]: p["status"] for p in cs.list("pods")}
    assert sorted(pods) == ["a", "c"]
    assert pods["a"]["podIP"] == "10.0.0.1" and pods["c"]["podIP"] == "10.0.0.2"
    patched = [k for v, kind, k, _ in cs.calls[n0:] if kind == "pods"]
    assert patched == [("default", "a"), ("default", "c")]
    c.close()


def test_c1_size_through_the_drop_in():
    """BASELINE configs[0]'s shape (1k nodes x 10k pods, ManageAllNodes) through
    the drop-in and the fake clientset: the first tick inits every node and runs
    every Pending pod with a fresh IP; the next tick is heartbeats only (the
    echoes of the first tick's 11k patches were dropped)."""
    cs = FakeClientset(deliver="queued")
    for i in range(1000):
        cs.create(node("node-%07d" % i, managed=True))
    for j in range(10000):
        cs.create(pod("pod-%08d" % j, "node-%07d" % (j // 10), containers=(("fake-pod", "fake"),),
                      status={"phase": "Pending"}))
    c = controller(cs, manage_all_nodes=True, cidr="10.0.0.1/8")
    n = c.step(S0 + 30)
    cs.pump()
    assert n == 1000 + 1000 + 10000  # heartbeats + inits + pod patches
    assert c.stats.echoes_on_arrival == 12000
    n = c.step(S0 + 60)
    assert n == 1000 and c.stats.pod_records == 10000  # only the Added events were ingested
    ips = sorted(int(p["status"]["podIP"].split(".")[3]) + 256 * int(p["status"]["podIP"].split(".")[2])
                 for p in cs.list("pods"))
    assert ips == list(range(1, 10001))
    c.close()


def test_shim_ingest_sequence_small_on_the_oracle():
    """tests/test_controller_gpu.py's 1M x 10M shim replay at 20k nodes with the
    oracle on both sides: the batch's runs, the echo property and the counters
    the GPU test asserts hold for the restatement itself"""
    from test_controller_gpu import shim_ingest_sequence
    shim_ingest_sequence(lambda cfg: Oracle(cfg, threads=0), 20_000)
