"""GPU parity of every k_emit source path against the CPU oracle.

k_emit writes a pod patch from its spec's per-shape unit tables (static bytes
plus value-row overlays) or, for specs without tables, assembles each 16-byte
unit from at most two source regions (kernels.hip "k_emit"); the spec programs
and node blobs come from the block's LDS cache when they fit and from global
memory otherwise.  Every test runs with the tables (fused into k_pod_jobs and
not), without them, and mixed.  These
tests drive both paths for pod patches (pod_controller.go:404-439 over
pod.status.tpl) and node-init patches (node_controller.go:356-391 over
node.status.tpl), in the same tick and separately, with patches far past
2 KiB, IP strings of every width (7-15 characters), creation times spread over
decades, and empty / non-empty statuses."""
import numpy as np
import pytest

from gpu_common import Driver, new_pods
from kwok_amd import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["table", "table-fused", "table-fused-k_emit-inits", "table-unfused", "general",
                                      "mixed"])
def emit_path(request, monkeypatch):
    """pod patches from the per-shape unit tables (on split ticks written by
    k_pod_jobs itself, the fused emission, when the tick is dense, its last
    blocks writing the node inits; "table-fused" on every split tick,
    KWOK_FUSE_EMIT=1; "table-fused-k_emit-inits" the same with the node inits
    left to k_emit, KWOK_FOLD_INITS=0; "table-unfused": always by k_emit from
    job records, KWOK_FUSE_EMIT=0), from the general region emitter
    (KWOK_EMIT_TAB_UNITS=0), or both (a cap that tables only the first specs
    registered, so chunks mix the two and fall back as a whole; no fusion)"""
    if request.param == "table-fused":
        monkeypatch.setenv("KWOK_FUSE_EMIT", "1")
    elif request.param == "table-fused-k_emit-inits":
        monkeypatch.setenv("KWOK_FUSE_EMIT", "1")
        monkeypatch.setenv("KWOK_FOLD_INITS", "0")
    elif request.param == "table-unfused":
        monkeypatch.setenv("KWOK_FUSE_EMIT", "0")
    elif request.param == "general":
        monkeypatch.setenv("KWOK_EMIT_TAB_UNITS", "0")
    elif request.param == "mixed":
        monkeypatch.setenv("KWOK_EMIT_TAB_UNITS", "20000")
    return request.param

HOST_IPS = ["1.2.3.4", "10.20.30.40", "100.100.100.100", "192.168.100.200", "255.255.255.255", "9.99.9.99"]


def spec_set(rng, n, max_containers=4, max_init=2, max_gates=2, tag="s"):
    """n distinct pod specs (containers, init containers, readiness gates)"""
    out = []
    for i in range(n):
        nc = int(rng.integers(0, max_containers + 1))
        ni = int(rng.integers(0, max_init + 1))
        ng = int(rng.integers(0, max_gates + 1))
        cs = [("c%d-%s%d" % (k, tag, i), "registry.io/img-%d:v%d" % (i, k)) for k in range(nc)]
        ics = [("init%d-%s%d" % (k, tag, i), "busybox:1.%d" % k) for k in range(ni)]
        gs = ["gate.io/%s%d-%d" % (tag, i, k) for k in range(ng)]
        out.append((cs, ics, gs))
    return out


def run_pods(d, names, n_pods, ticks=3, seed_ip=True):
    nh, st = d.nodes(names, managed=1, lockable=1)
    assert (st == 0).all()
    rng = d.rng
    ev, ar = new_pods(rng, nh, n_pods, d.spec, 0.05 if seed_ip else 0.0, (0x0A000000, 0x0AFFFFFF),
                      host_ips=HOST_IPS, host_ip_frac=0.3, years=40)
    h, s, _ = d.pods(ev, ar)
    assert (s == 0).all()
    outs = [d.tick("tick %d" % t) for t in range(ticks)]
    return outs


def test_many_specs_uncached_pods():
    """> 64 specs and > 4 KiB of spec programs: pod patches from global memory"""
    kw = dict(cidr="10.0.0.1/8", node_ip="196.168.0.1", buckets=256, node_slots_per_bucket=16,
              pod_slots_per_bucket=256)
    rng = np.random.default_rng(11)
    d = Driver(kw, 11, specs=spec_set(rng, 90))
    outs = run_pods(d, ["node-%05d" % i for i in range(600)], 8000)
    assert outs[0].counters["pod_patch"] > 7000
    d.e.close()
    d.o.close()


def test_long_patches_cached():
    """one spec whose patch is ~3.5 KiB (25 containers), beside the default spec,
    both staged in LDS (spec bytes <= 4 KiB)"""
    big = ([("container-%02d" % k, "img-%02d" % k) for k in range(25)], [], [])
    kw = dict(cidr="10.0.0.1/16", node_ip="10.1.2.3", buckets=64, node_slots_per_bucket=16, pod_slots_per_bucket=128)
    d = Driver(kw, 12, specs=[([("fake-pod", "fake")], [], []), big])
    outs = run_pods(d, ["n%d" % i for i in range(200)], 3000)
    lens = [len(b) for _, b in outs[0].pod_patches]
    assert max(lens) > 2048
    d.e.close()
    d.o.close()


def test_long_patches_uncached():
    """a ~6 KiB patch (32 containers, 8 init containers, 6 readiness gates):
    more than the LDS spec cache holds"""
    big = ([("c%02d" % k, "quay.io/org/image-%02d:tag" % k) for k in range(32)],
           [("i%d" % k, "init-img-%d" % k) for k in range(8)], ["ready.io/g%d" % k for k in range(6)])
    kw = dict(cidr="172.16.0.1/12", node_ip="196.168.0.1", buckets=64, node_slots_per_bucket=16,
              pod_slots_per_bucket=128)
    d = Driver(kw, 13, specs=[([("fake-pod", "fake")], [], []), big])
    outs = run_pods(d, ["n%d" % i for i in range(200)], 3000)
    assert max(len(b) for _, b in outs[0].pod_patches) > 5000
    d.e.close()
    d.o.close()


def node_status(rng, i, distinct):
    """apiserver-shaped node status fields (compact JSON, as the codec emits them)"""
    if not distinct:
        return {}
    ip = "10.%d.%d.%d" % (i >> 16 & 255, i >> 8 & 255, i & 255)
    st = {"addresses": '[{"address":"%s","type":"InternalIP"},{"address":"host-%d","type":"Hostname"}]' % (ip, i)}
    if rng.random() < 0.7:
        cpu = int(rng.integers(1, 128))
        st["allocatable"] = '{"cpu":"%d","memory":"%dGi","pods":"110"}' % (cpu, cpu * 4)
        st["capacity"] = '{"cpu":"%d","memory":"%dGi","pods":"110"}' % (cpu, cpu * 4)
    if rng.random() < 0.5:
        st["nodeInfo"] = {"architecture": "arm64", "kernelVersion": "6.1.%d" % (i % 90), "osImage": "ubuntu-%d" % i,
                          "kubeletVersion": "v1.26.%d" % (i % 7), "machineID": "m%08x" % i}
    return st


@pytest.mark.parametrize("many_specs", [False, True])
def test_distinct_node_blobs(many_specs):
    """every node with its own addresses / capacity / nodeInfo: > 2 KiB of node
    blobs, so node-init patches come from global memory; pods in the same tick
    from the LDS cache (few specs) or from global memory (many specs)"""
    rng = np.random.default_rng(21)
    specs = spec_set(rng, 80) if many_specs else None
    kw = dict(cidr="10.0.0.1/8", node_ip="196.168.0.1", buckets=128, node_slots_per_bucket=32,
              pod_slots_per_bucket=256)
    d = Driver(kw, 21, specs=specs)
    names = ["worker-%05d" % i for i in range(1500)]
    status = [node_status(rng, i, rng.random() < 0.8) for i in range(len(names))]
    nh, st = d.nodes(names, managed=1, lockable=1, status=status)
    assert (st == 0).all()
    ev, ar = new_pods(rng, nh, 6000, d.spec, 0.0, None, host_ips=HOST_IPS, host_ip_frac=0.2, years=5)
    d.pods(ev, ar)
    out = d.tick("blobs tick 0")
    assert out.counters["node_init"] == 1500 and out.counters["pod_patch"] > 5000
    # re-init: a node Modified with its status removed is locked and initialised again
    re = list(range(0, 1500, 7))
    d.nodes([names[i] for i in re], managed=1, lockable=1, status=[node_status(rng, i + 7, True) for i in re])
    out = d.tick("blobs tick 1")
    d.tick("blobs tick 2")
    d.e.close()
    d.o.close()


def test_node_inits_cached_and_ip_widths():
    """few distinct blobs (LDS path) with NodeIP / hostIP / podIP strings of
    every width in one tick"""
    kw = dict(cidr="1.0.0.1/8", node_ip="255.255.255.254", buckets=64, node_slots_per_bucket=16,
              pod_slots_per_bucket=128)
    d = Driver(kw, 22)
    rng = d.rng
    names = ["n-%d" % i for i in range(300)]
    status = [node_status(rng, i % 3, True) if i % 2 else {} for i in range(len(names))]
    nh, st = d.nodes(names, managed=1, lockable=1, status=status)
    assert (st == 0).all()
    ev, ar = new_pods(rng, nh, 4000, d.spec, 0.3, (0x01000000, 0x01FFFFFF), host_ips=HOST_IPS, host_ip_frac=0.5,
                      years=50)
    d.pods(ev, ar)
    out = d.tick("widths tick 0")
    _, _, hip, pip = d.live()
    widths = {len(abi.ip4s(int(v))) for v in np.concatenate([hip, pip]) if v}
    assert min(widths) <= 8 and max(widths) >= 14
    assert out.counters["node_init"] == 300
    d.tick("widths tick 1")
    d.e.close()
    d.o.close()
