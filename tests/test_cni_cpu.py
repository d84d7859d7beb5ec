"""CPU: EnableCNI semantics on the oracle (pod_controller.go:377-389 configurePod
with cni.Setup, :337-342 cni.Remove on Deleted): the ipPool is never used, the
pods a tick evaluates without a podIP are listed for cni.Setup, a pod gets the
IP the caller assigned in its first patch (status then non-empty, so hostIP /
podIP are rendered), a pod still waiting for cni.Setup is not patched, and
deletions release nothing.  Parity of the HIP engine with this:
tests/test_cni_gpu.py.  Pinned by the reference's code only (no reference
test covers EnableCNI)."""
import ipaddress

import numpy as np

from kwok_amd import abi, workload
from kwok_amd.engine import make_config
from oracle.oracle import Oracle

CNI_BASE = int(ipaddress.IPv4Address("172.20.0.2"))


def fake_cni(handles, start):
    """host-local IPAM: sequential addresses in call order"""
    return np.arange(start, start + len(handles), dtype=np.uint32)


def test_cni_mode_on_oracle():
    o = Oracle(make_config(cidr="10.0.0.1/24", buckets=64, node_slots_per_bucket=8, pod_slots_per_bucket=64,
                           enable_cni=True))
    spec = o.register_pod_spec([("c", "img")])
    ar = abi.Arena()
    ev = np.zeros(100, abi.NODE_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["managed"] = 1
    ev["lockable"] = 1
    for i in range(100):
        ev[i]["name"] = ar.ref("node-%03d" % i)
    nh, st = o.ingest_nodes_raw(ev, bytes(ar.buf))
    assert (st == 0).all()
    pods = workload.pod_events(nh, spec, 5)
    pods["flags"][::7] = 0  # some pods with an empty status
    pods["phase"][::7] = abi.PHASE_NONE
    ph, st, _ = o.ingest_pods_raw(pods, b"")
    assert (st == 0).all()
    pend = o.cni_pending()
    assert list(pend) == sorted(ph.tolist())  # every pod, canonical order
    half = pend[:250]
    assert (o.cni_assign(half, fake_cni(half, CNI_BASE)) == 0).all()
    out = o.tick(workload.S0 + 30)
    c = out.counters
    assert c["alloc"] == 0 and c["pod_patch"] == 250 and c["pods_pending"] == 500 - 250 - (pods["phase"] == 0)[
        np.isin(ph, pend[250:])].sum()
    got = {h: b for h, b in out.pod_patches}
    for h, ip in zip(half, fake_cni(half, CNI_BASE)):
        assert b'"podIP":"%s"' % abi.ip4s(int(ip)).encode() in got[int(h)]
        assert b'"hostIP":"196.168.0.1"' in got[int(h)]
    # the rest are still pending cni.Setup, and listed again
    rest = o.cni_pending()
    assert list(rest) == list(pend[250:])
    o.cni_assign(rest, fake_cni(rest, CNI_BASE + 250))
    out = o.tick(workload.S0 + 60)
    assert out.counters["pod_patch"] == 250 and out.counters["alloc"] == 0
    used, phase, hip, pip = o.dump_pods(0, 64 * 64)
    live = used.astype(bool)
    assert (phase[live] == abi.PHASE_RUNNING).all()
    assert sorted(pip[live].tolist()) == list(range(CNI_BASE, CNI_BASE + 500))
    assert len(o.cni_pending()) == 0
    # deletions: DeletePod without any ipPool.Put; Deleted events release nothing
    mark = np.zeros(10, abi.POD_EVENT_DTYPE)
    mark["op"] = abi.OP_UPSERT
    mark["handle"] = ph[:10]
    mark["spec_id"] = spec
    mark["phase"] = abi.PHASE_RUNNING
    mark["flags"] = abi.POD_DELETING | abi.POD_STATUS_NONEMPTY
    mark["creation_unix"] = workload.S0 - 60
    o.ingest_pods_raw(mark, b"")
    out = o.tick(workload.S0 + 90)
    assert out.counters["delete"] == 10 and out.counters["release"] == 0
    gone = np.zeros(5, abi.POD_EVENT_DTYPE)
    gone["op"] = abi.OP_DELETE
    gone["handle"] = ph[10:15]
    ar = abi.Arena()
    for i, h in enumerate(ph[10:15]):
        gone[i]["pod_ip"] = ar.ref(abi.ip4s(int(pip[h])))
    _, st, rel = o.ingest_pods_raw(gone, bytes(ar.buf))
    assert (st == 0).all() and (rel == 0).all()
    o.close()
