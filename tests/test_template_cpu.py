"""CPU: the engine's host template renderer (kwok_template_render: the Go
text/template subset + yaml.v2 -> encoding/json of renderer.go:49-89) and
the custom pod status template compiler (kwok_pod_template_patch: compiled to
the kernels' A | hostIP | B | podIP | C program, assembled on the host as
k_emit does), both against tests/golden/gotmpl.py - the independent Python
interpreter that the reference's renderer_test.go known answers pin.
Templates: the reference's own .tpl files (read from /root/reference when it
is present), and custom templates written for these tests
(tests/templates/*.tpl).  Parity of the HIP kernels with the compiled
programs: tests/test_custom_template_gpu.py."""
import ipaddress
import json
import os

import numpy as np
import pytest

import gotmpl_path  # noqa: F401
import gotmpl
from kwok_amd import engine
from kwok_amd.engine import KwokError

HERE = os.path.dirname(os.path.abspath(__file__))
REF_TPL = "/root/reference/pkg/kwok/controllers/templates"
START = 1704067200
NODE_IP = "196.168.0.1"


def tpl(name):
    return open(os.path.join(HERE, "templates", name)).read()


def rfc3339(u):
    import datetime as dt
    return dt.datetime.fromtimestamp(u, dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def ip(v):
    return str(ipaddress.IPv4Address(v))


def random_specs(seed, n):
    rng = np.random.default_rng(seed)
    names = ["c%d" % i for i in range(5)]
    images = ["img", "busybox:1.36", "registry.k8s.io/pause:3.9", "a/b@sha256:0ab1"]
    out = []
    for _ in range(n):
        k = int(rng.integers(0, 4))
        cs = [(names[i], images[int(rng.integers(0, len(images)))]) for i in range(k)]
        ics = [("init%d" % i, images[int(rng.integers(0, len(images)))]) for i in range(int(rng.integers(0, 3)))]
        gates = ["example.com/gate-%d" % i for i in range(int(rng.integers(0, 3)))]
        out.append((cs, ics, gates))
    return out


def pod_doc(cs, ics, gates, creation, status):
    spec = {"containers": [{"name": c, "image": i, "resources": {}} for c, i in cs] or None, "nodeName": "n0"}
    if ics:
        spec["initContainers"] = [{"name": c, "image": i, "resources": {}} for c, i in ics]
    if gates:
        spec["readinessGates"] = [{"conditionType": g} for g in gates]
    return {"metadata": {"name": "p", "namespace": "default", "creationTimestamp": rfc3339(creation)},
            "spec": spec, "status": status}


def expected_patch(text, cs, ics, gates, creation, host_ip, pod_ip, nonempty):
    """configurePod's patch for a pod the engine emits (pod_controller.go:377-401)"""
    status = {}
    if nonempty:
        status["phase"] = "Pending"
        if host_ip:
            status["hostIP"] = ip(host_ip)
    funcs = {"NodeIP": lambda: NODE_IP, "PodIP": lambda: ip(pod_ip), "StartTime": lambda: rfc3339(START)}
    body = gotmpl.render_to_json(text, pod_doc(cs, ics, gates, creation, status), funcs)
    return ('{"status":%s}' % body).encode()


def test_renderer_known_answers():
    for kat in json.load(open(os.path.join(HERE, "golden", "renderer_kat.json"))):
        assert engine.template_render(kat["tmpl"], kat["data"], kat["funcs"]) == kat["expected"], kat["name"]


@pytest.mark.skipif(not os.path.isdir(REF_TPL), reason="reference templates not present")
def test_reference_templates_render_like_gotmpl():
    rd = lambda f: open(os.path.join(REF_TPL, f)).read()  # noqa: E731
    funcs = {"Now": "2024-01-01T00:00:30Z", "StartTime": "2024-01-01T00:00:00Z", "NodeIP": NODE_IP,
             "PodIP": "10.0.0.7"}
    gf = {k: (lambda v=v: v) for k, v in funcs.items()}
    pod = rd("pod.status.tpl")
    for k, (cs, ics, gates) in enumerate(random_specs(1, 40)):
        for status in ({}, {"phase": "Pending"}, {"phase": "Running", "hostIP": "10.1.2.3", "podIP": "10.0.0.9"}):
            doc = pod_doc(cs, ics, gates, START - 60 - k, status)
            assert engine.template_render(pod, doc, funcs) == gotmpl.render_to_json(pod, doc, gf), (k, status)
    node = rd("node.status.tpl") + "\n" + rd("node.heartbeat.tpl")
    for doc in ({"metadata": {"name": "n0"}, "spec": {}, "status": {"nodeInfo": {}, "daemonEndpoints": {}}},
                {"metadata": {"name": "n1"}, "spec": {}, "status": {
                    "addresses": [{"address": "10.9.9.9", "type": "InternalIP"}],
                    "allocatable": {"cpu": "4", "memory": "8Gi", "pods": "110"},
                    "capacity": {"cpu": "4", "memory": "8Gi", "pods": "110"},
                    "nodeInfo": {"architecture": "arm64", "osImage": "x", "kubeletVersion": "v1.26.0"},
                    "phase": "Running"}}):
        assert engine.template_render(node, doc, funcs) == gotmpl.render_to_json(node, doc, gf)


@pytest.mark.skipif(not os.path.isdir(REF_TPL), reason="reference templates not present")
def test_reference_pod_template_compiles_to_the_default_program():
    """the generic compiler, fed the reference's own pod.status.tpl, gives the
    bytes the engine's built-in default program gives (and gotmpl.py)"""
    text = open(os.path.join(REF_TPL, "pod.status.tpl")).read()
    for k, (cs, ics, gates) in enumerate(random_specs(2, 30)):
        for hip, pip, ne in ((0, 0x0A000005, True), (0x0A010203, 0x0A000009, True), (0, 0, False)):
            got = engine.pod_template_patch(text, cs, ics, gates, START, NODE_IP, START - 60 - k, hip, pip, ne)
            assert got == expected_patch(text, cs, ics, gates, START - 60 - k, hip, pip, ne), (k, hip, ne)


@pytest.mark.parametrize("name", ["pod_a.tpl", "pod_b.tpl", "pod_c.tpl"])
def test_custom_pod_templates_compile_and_match_gotmpl(name):
    text = tpl(name)
    for k, (cs, ics, gates) in enumerate(random_specs(3, 30)):
        for hip, pip, ne in ((0, 0x0A000005, True), (0x0A010203, 0xAC10FFFE, True), (0, 0, False)):
            got = engine.pod_template_patch(text, cs, ics, gates, START, NODE_IP, 1000000000 + 86399 * k, hip, pip, ne)
            want = expected_patch(text, cs, ics, gates, 1000000000 + 86399 * k, hip, pip, ne)
            assert got == want, (name, k, hip, ne)


REJECT = {
    "reads a field the engine does not hold": "conditions: []\nhostIP: {{ .metadata.name }}\n",
    "Now varies per tick": "conditions: []\nstartTime: {{ Now }}\n",
    "a branch on the phase": "{{ if .status.phase }}conditions: []{{ end }}\n",
    "hostIP as the first key (a region under 16 bytes)":
        "{{ with .status }}hostIP: {{ NodeIP }}\npodIP: {{ PodIP }}\n{{ end }}phase: Running\n",
    "PodIP twice (two ipPool.Get)":
        "conditions: []\n{{ with .status }}hostIP: {{ NodeIP }}\npodIP: {{ PodIP }}\npodIPx: {{ PodIP }}\n{{ end }}"
        "phase: Running\n",
    "a YAML float": "conditions: []\ncpu: 1.5\n{{ with .status }}hostIP: {{ NodeIP }}\npodIP: {{ PodIP }}\n{{ end }}"
                    "phase: Running\n",
    "a pipe": "conditions: {{ .spec.containers | len }}\n",
    "status IPs ignored when the pod holds them":
        "conditions: []\n{{ with .status }}hostIP: {{ NodeIP }}\npodIP: {{ PodIP }}\n{{ end }}phase: Running\n",
}


@pytest.mark.parametrize("why", list(REJECT))
def test_templates_outside_the_program_are_rejected(why):
    with pytest.raises(KwokError) as ei:
        engine.pod_template_patch(REJECT[why], [("c", "img")], pod_ip=0x0A000001)
    assert ei.value.code == -3, why  # KWOK_EDOMAIN


def test_comments_trim_markers_else_if():
    doc = {"a": "", "b": "x", "l": [1, 2]}
    t1 = "{{- /* c */ -}}\nk: {{ if .a }}A{{ else if .b }}B{{ else }}C{{ end }}\nnum: {{ len .l }}\n"
    t2 = "k: {{ if .a }}A{{ else }}{{ if .b }}B{{ else }}C{{ end }}{{ end }}\nnum: 2\n"
    assert engine.template_render(t1, doc) == engine.template_render(t2, doc) == '{"k":"B","num":2}'
    assert engine.template_render("k: {{ not .a }}\nm: {{ eq .b \"x\" }}\n", doc) == '{"k":true,"m":true}'
    assert engine.template_render("{{ range .l }}- {{ . }}\n{{ end }}", doc) == "[1,2]"
    for bad in ("k: {{ printf \"%d\" 1 }}", "k: {{ .b", "{{ if .a }}x", "k: |\n  block\n", "k: 0x10\n"):
        with pytest.raises(KwokError):
            engine.template_render(bad, doc)


# ---- custom node initialization templates ----------------------------------
NODES = [
    {},
    {"addresses": '[{"address":"10.9.9.9","type":"InternalIP"}]',
     "allocatable": '{"cpu":"4","memory":"8Gi","pods":"110"}', "capacity": '{"cpu":"4","memory":"8Gi","pods":"110"}',
     "nodeInfo": {"architecture": "arm64", "osImage": "ubuntu", "kubeletVersion": "v1.26.0"}, "phase": 2},
    {"allocatable": '{"cpu":"1","pods":"8"}', "nodeInfo": {"kernelVersion": "6.1.0"}},
]


def node_record(n, name="n0"):
    from kwok_amd import abi
    ar = abi.Arena()
    ev = np.zeros(1, abi.NODE_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["managed"] = 1
    ev["lockable"] = 1
    ev["phase"] = n.get("phase", 0)
    ev[0]["name"] = ar.ref(name)
    for f in ("addresses", "allocatable", "capacity"):
        ev[0][f] = ar.ref(n.get(f, ""))
    for k, key in enumerate(abi.NODEINFO_KEYS):
        ev[0]["node_info"][k] = ar.ref(n.get("nodeInfo", {}).get(key, ""))
    return ev, bytes(ar.buf)


def node_doc(n):
    st = {"daemonEndpoints": {"kubeletEndpoint": {"Port": 0}},
          "nodeInfo": {k: n.get("nodeInfo", {}).get(k, "") for k in
                       __import__("kwok_amd.abi", fromlist=["x"]).NODEINFO_KEYS}}
    for f in ("addresses", "allocatable", "capacity"):
        if n.get(f):
            st[f] = json.loads(n[f])
    if n.get("phase") == 2:
        st["phase"] = "Running"
    return {"metadata": {"name": "n0"}, "spec": {}, "status": st}


@pytest.mark.skipif(not os.path.isdir(REF_TPL), reason="reference templates not present")
@pytest.mark.parametrize("which", ["reference", "node_a.tpl"])
def test_node_templates_compile_and_match_gotmpl(which):
    rd = lambda f: open(os.path.join(REF_TPL, f)).read()  # noqa: E731
    text = rd("node.status.tpl") if which == "reference" else tpl(which)
    full = text + "\n" + rd("node.heartbeat.tpl")  # node_controller.go:101
    now = START + 30
    funcs = {"NodeIP": lambda: NODE_IP, "Now": lambda: rfc3339(now), "StartTime": lambda: rfc3339(START)}
    for n in NODES:
        ev, ar = node_record(n)
        got = engine.node_template_patch(text, ev[0], ar, START, NODE_IP, now)
        want = ('{"status":%s}' % gotmpl.render_to_json(full, node_doc(n), funcs)).encode()
        assert got == want, n


def test_node_templates_outside_the_blob_are_rejected():
    """a node template must leave the conditions to the heartbeat template and
    read only the status fields the engine holds"""
    bad = "conditions: []\nphase: Running\n"
    ev, ar = node_record({})
    with pytest.raises(KwokError):
        engine.node_template_patch(bad, ev[0], ar)
    with pytest.raises(KwokError):  # Now outside the conditions varies per tick
        engine.node_template_patch("phase: Running\nx: {{ Now }}\n", ev[0], ar)
    with pytest.raises(KwokError):  # a field the engine does not hold
        engine.node_template_patch("phase: {{ .metadata.name }}\n", ev[0], ar)


@pytest.mark.skipif(not os.path.isdir(REF_TPL), reason="reference templates not present")
def test_reference_node_template_compiles_to_the_default_blob():
    """the generic compiler, fed the reference's node.status.tpl, gives the init
    patch the built-in default path gives (the oracle's, pinned by the goldens)"""
    from kwok_amd.engine import make_config
    from oracle.oracle import Oracle
    text = open(os.path.join(REF_TPL, "node.status.tpl")).read()
    for n in NODES:
        o = Oracle(make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8, node_ip=NODE_IP,
                               start_time=START))
        ev, ar = node_record(n)
        o.ingest_nodes_raw(ev, ar)
        out = o.tick(START + 30)
        assert len(out.node_inits) == 1
        assert engine.node_template_patch(text, ev[0], ar, START, NODE_IP, START + 30) == out.node_inits[0][1], n
        o.close()


# ---- custom heartbeat templates --------------------------------------------
@pytest.mark.parametrize("name", ["heartbeat_a.tpl", "heartbeat_b.tpl"])
def test_heartbeat_templates_match_gotmpl(name):
    text = tpl(name)
    for now in (START + 30, START + 86400 * 365 + 7):
        funcs = {"NodeIP": lambda: NODE_IP, "Now": lambda: rfc3339(now), "StartTime": lambda: rfc3339(START)}
        want = ('{"status":%s}' % gotmpl.render_to_json(text, {"metadata": {}, "spec": {}, "status": {}}, funcs)).encode()
        assert engine.heartbeat_template_patch(text, START, NODE_IP, now) == want
    # node inits splice the custom conditions: node_controller.go:101 appends the heartbeat template text
    full = tpl("node_a.tpl") + "\n" + text
    for n in NODES:
        ev, ar = node_record(n)
        funcs = {"NodeIP": lambda: NODE_IP, "Now": lambda: rfc3339(START + 30), "StartTime": lambda: rfc3339(START)}
        want = ('{"status":%s}' % gotmpl.render_to_json(full, node_doc(n), funcs)).encode()
        assert engine.node_template_patch(tpl("node_a.tpl"), ev[0], ar, START, NODE_IP, START + 30, heartbeat_tpl=text) == want


def test_default_heartbeat_equals_the_oracle_body():
    from kwok_amd.engine import make_config
    from oracle.oracle import Oracle
    o = Oracle(make_config(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8, node_ip=NODE_IP, start_time=START))
    ev, ar = node_record({})
    o.ingest_nodes_raw(ev, ar)
    out = o.tick(START + 30)
    assert engine.heartbeat_template_patch(None, START, NODE_IP, START + 30) == out.heartbeat_body(0)
    if os.path.isdir(REF_TPL):  # the reference's own template compiles to the same body
        ref = open(os.path.join(REF_TPL, "node.heartbeat.tpl")).read()
        assert engine.heartbeat_template_patch(ref, START, NODE_IP, START + 30) == out.heartbeat_body(0)
    o.close()


@pytest.mark.parametrize("bad", ["conditions: []\nphase: Running\n",          # a second key
                                 "conditions:\n- type: {{ .metadata.name }}\n",  # a per-node field
                                 "conditions:\n" + "- message: %s\n  type: T\n" % ("x" * 1300)])  # too long
def test_heartbeat_templates_outside_the_stream_are_rejected(bad):
    with pytest.raises(KwokError):
        engine.heartbeat_template_patch(bad)
