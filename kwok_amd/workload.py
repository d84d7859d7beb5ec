"""Synthetic kwok workloads (SURVEY.md §8(d) / BASELINE.json configs), built
vectorised with numpy so 1M-node / 10M-pod fleets ingest in seconds.

Shapes follow the reference's own benchmark objects
(test/kwokctl/kwokctl_benchmark_test.sh:71-117): nodes `node-%07d`
(ManageAllNodes, empty status), pods with one container
{name: fake-pod, image: fake}, 10 pods per node, ingested Pending with no IPs,
creationTimestamp = S - 60 s, NodeIP 196.168.0.1, CIDR 10.0.0.1/8.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import abi

S0 = 1704067200  # 2024-01-01T00:00:00Z
NODE_IP = "196.168.0.1"
CIDR = "10.0.0.1/8"
PODS_PER_NODE = 10
BUCKETS = 4096


def node_names(first: int, count: int) -> np.ndarray:
    """`node-%07d` names as a (count, 12) uint8 array."""
    idx = np.arange(first, first + count, dtype=np.int64)
    out = np.empty((count, 12), np.uint8)
    out[:, :5] = np.frombuffer(b"node-", np.uint8)
    for k in range(7):
        out[:, 11 - k] = ord("0") + (idx // 10 ** k) % 10
    return out


def fnv1a32_rows(rows: np.ndarray) -> np.ndarray:
    h = np.full(rows.shape[0], 0x811C9DC5, np.uint32)
    prime = np.uint32(0x01000193)
    with np.errstate(over="ignore"):
        for k in range(rows.shape[1]):
            h = (h ^ rows[:, k].astype(np.uint32)) * prime
    return h


def slots_for(total_nodes: int, buckets: int = BUCKETS, pods_per_node: int = PODS_PER_NODE):
    """Per-bucket slot capacities with ~7 sigma headroom over the Poisson load."""
    avg = total_nodes / buckets
    cn = int(math.ceil(avg + 7 * math.sqrt(max(avg, 1.0)) + 4))
    cn = (cn + 3) // 4 * 4
    cp = (cn * pods_per_node + 7) // 8 * 8
    return cn, cp


@dataclass
class Fleet:
    total_nodes: int
    rank: int
    world: int
    names: np.ndarray        # (n_local, 12) names owned by this rank
    node_events: np.ndarray  # NODE_EVENT_DTYPE
    arena: bytes
    cn: int
    cp: int
    node_handles: np.ndarray = None  # set by build_engine_fleet


def make_fleet(nodes_per_rank: int, rank: int = 0, world: int = 1, buckets: int = BUCKETS,
               managed_frac: float = 1.0, lockable_frac: float = 1.0, seed: int = 0) -> Fleet:
    """Weak scaling: the fleet has nodes_per_rank * world nodes; this rank owns
    the nodes whose bucket falls in its contiguous bucket range.
    managed_frac < 1: ManageAllNodes=false with an annotation selector that
    matches that fraction of the nodes (needHeartbeat, node_controller.go:206);
    lockable_frac < 1: the rest carry a disregard annotation (needLockNode
    false, :210-223).  Both drawn per node name index with `seed`."""
    total = nodes_per_rank * world
    names = node_names(0, total)
    b = fnv1a32_rows(names) & np.uint32(buckets - 1)
    lo = rank * buckets // world
    hi = (rank + 1) * buckets // world
    sel = (b >= lo) & (b < hi)
    mine = names[sel]
    n = mine.shape[0]
    rng = np.random.default_rng(seed)
    managed = rng.random(total) < managed_frac if managed_frac < 1 else np.ones(total, bool)
    lockable = rng.random(total) < lockable_frac if lockable_frac < 1 else np.ones(total, bool)
    ev = np.zeros(n, abi.NODE_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["managed"] = managed[sel]
    ev["lockable"] = lockable[sel]
    ev["name"]["off"] = np.arange(n, dtype=np.uint32) * 12
    ev["name"]["len"] = 12
    cn, cp = slots_for(total, buckets)
    return Fleet(total, rank, world, mine, ev, mine.tobytes(), cn, cp)


def pod_events(node_handles: np.ndarray, spec_id: int, pods_per_node: int = PODS_PER_NODE,
               creation: int = S0 - 60) -> np.ndarray:
    """Pending pods (status {phase: Pending}, no IPs), pods_per_node per node."""
    n = node_handles.shape[0] * pods_per_node
    ev = np.zeros(n, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["phase"] = abi.PHASE_PENDING
    ev["flags"] = abi.POD_STATUS_NONEMPTY
    ev["handle"] = -1
    ev["spec_id"] = spec_id
    ev["node_handle"] = np.repeat(node_handles.astype(np.int32), pods_per_node)
    ev["creation_unix"] = creation
    return ev


def build_engine_fleet(engine_cls, nodes_per_rank, rank=0, world=1, device=0, cidr=CIDR, node_ip=NODE_IP,
                       start=S0, buckets=BUCKETS, pods_per_node=PODS_PER_NODE, managed_frac=1.0, lockable_frac=1.0,
                       seed=0, **cfg_kw):
    """Create an engine (or oracle) for this rank and ingest its share of the
    fleet.  Returns (engine, fleet, pod_handles)."""
    from .engine import make_config
    fl = make_fleet(nodes_per_rank, rank, world, buckets, managed_frac, lockable_frac, seed)
    cfg = make_config(cidr=cidr, node_ip=node_ip, start_time=start, buckets=buckets,
                      node_slots_per_bucket=fl.cn, pod_slots_per_bucket=fl.cp, rank=rank, world_size=world,
                      device=device, **cfg_kw)
    e = engine_cls(cfg)
    spec = e.register_pod_spec([("fake-pod", "fake")])
    hs, st = e.ingest_nodes_raw(fl.node_events, fl.arena)
    if (st != 0).any():
        raise RuntimeError("node ingest rejected %d records (first code %d)" % ((st != 0).sum(), st[st != 0][0]))
    fl.node_handles = hs
    pods = pod_events(hs, spec, pods_per_node)
    ph, pst, _ = e.ingest_pods_raw(pods, b"")
    if (pst != 0).any():
        raise RuntimeError("pod ingest rejected %d records (first code %d)" % ((pst != 0).sum(), pst[pst != 0][0]))
    return e, fl, ph


def ip_strings(ips: np.ndarray, base: int = 0):
    """Dotted quads (net.IP.String()) of IPv4 addresses, vectorised: one byte
    arena plus (off, len) per address; off counts from `base`."""
    ips = np.asarray(ips, np.uint32)
    n = ips.shape[0]
    octs = [((ips >> np.uint32(s)) & np.uint32(255)).astype(np.int64) for s in (24, 16, 8, 0)]
    lens = [1 + (o >= 10) + (o >= 100) for o in octs]
    total = lens[0] + lens[1] + lens[2] + lens[3] + 3
    off = np.zeros(n, np.int64)
    if n:
        off[1:] = np.cumsum(total)[:-1]
    buf = np.zeros(int(total.sum()) if n else 0, np.uint8)
    pos = off.copy()
    for k, (o, ln) in enumerate(zip(octs, lens)):
        m3 = ln == 3
        buf[pos[m3]] = 48 + o[m3] // 100
        m2 = ln >= 2
        buf[(pos + (ln == 3))[m2]] = 48 + (o[m2] // 10) % 10
        buf[pos + ln - 1] = 48 + o % 10
        pos += ln
        if k < 3:
            buf[pos] = ord(".")
            pos += 1
    return buf, (off + base).astype(np.uint32), total.astype(np.uint32)


class Churn:
    """BASELINE configs[3], the pod churn storm, as watch events (the shapes
    WatchPods sees, pod_controller.go:301-343).  Every tick, the `n_churn`
    oldest live pods get a deletionTimestamp: a Modified event carrying the
    pod's Running status (hostIP = NodeIP, its podIP), half of them with
    finalizers; the engine's tick deletes them (DeletePod, :155-202) and
    releases their IPs.  As many new Pending pods are created on the same nodes
    (so per-node pod counts stay fixed), and take IPs in the same tick (reuse of
    the released addresses, utils.go:83-108).  The later Deleted events of the
    deleted pods are not sent: the engine already freed those handles and the
    shim drops them.

    `dump` returns (used, phase, host_ip, pod_ip) over the pod handles
    [first, first + n_handles): every handle of a single-rank engine (or the
    oracle), or one rank's bucket range of a sharded one."""

    def __init__(self, pod_handles, node_of_pod, spec_id, n_handles, n_churn, seed=0, node_ip=NODE_IP,
                 creation=S0 - 60, first=0, alloc=None, packed=False):
        self.first = first
        # packed: the batch as kwok_pod_rec (kwok_ingest_pods_packed: 20 B per record,
        # IPs as integers, nodes by handle) instead of kwok_pod_event + dotted quads;
        # packed=12: as kwok_pod_rec12 (kwok_ingest_pods_packed12: 12 B, hostIP by flag)
        self.packed = packed
        # alloc(shape, dtype): the batch is written into (and reused from) these
        # buffers - e.g. page-locked host memory (engine.host_array), which the
        # ingest copies to the GPU by DMA
        self.alloc = alloc
        self.bufs = None
        self.live = np.asarray(pod_handles, np.int32).copy()  # FIFO: oldest first
        self.node_of = np.zeros(n_handles, np.int32)
        self.node_of[self.live - first] = node_of_pod
        self.ctime = np.zeros(n_handles, np.int64)
        self.ctime[self.live - first] = creation
        self.spec = spec_id
        self.n = n_churn
        self.rng = np.random.default_rng(seed)
        self.node_ip = node_ip.encode()

    def batch(self, dump, now):
        """(events, arena): n_churn deletion-marked pods, then n_churn new pods
        (packed: (records, None))"""
        D = min(self.n, self.live.shape[0])
        dead = self.live[:D]
        loc = dead - self.first
        used, phase, _, pip = dump()
        assert used[loc].all(), "churn: a live pod is missing from the engine"
        if self.packed:
            return self._batch_packed(D, dead, loc, phase, pip, now), None
        ip_buf, ip_off, ip_len = ip_strings(pip[loc], base=len(self.node_ip))
        if self.alloc is None:
            arena = self.node_ip + ip_buf.tobytes()
            ev = np.zeros(2 * D, abi.POD_EVENT_DTYPE)
        else:
            if self.bufs is None or len(self.bufs[0]) < 2 * D:
                self.bufs = (self.alloc((2 * self.n,), abi.POD_EVENT_DTYPE),
                             self.alloc((len(self.node_ip) + 16 * self.n,), np.uint8))
            ev = self.bufs[0][:2 * D]
            ev[...] = np.zeros(1, abi.POD_EVENT_DTYPE)[0]
            arena = self.bufs[1][:len(self.node_ip) + ip_buf.size]
            arena[:len(self.node_ip)] = np.frombuffer(self.node_ip, np.uint8)
            arena[len(self.node_ip):] = ip_buf
        d = ev[:D]
        d["op"] = abi.OP_UPSERT
        d["handle"] = dead
        d["node_handle"] = -1
        d["spec_id"] = self.spec
        d["phase"] = phase[loc]
        d["creation_unix"] = self.ctime[loc]
        fin = np.where(self.rng.random(D) < 0.5, abi.POD_HAS_FINALIZERS, 0)
        running = phase[loc] == abi.PHASE_RUNNING
        d["flags"] = (abi.POD_DELETING | fin | np.where(running, abi.POD_CONFORMS | abi.POD_STATUS_NONEMPTY, 0)
                      | np.where(pip[loc] != 0, abi.POD_STATUS_NONEMPTY, 0))
        d["host_ip"]["off"] = 0
        d["host_ip"]["len"] = np.where(running, len(self.node_ip), 0)
        d["pod_ip"]["off"] = ip_off
        d["pod_ip"]["len"] = np.where(pip[loc] != 0, ip_len, 0)
        c = ev[D:]
        c["op"] = abi.OP_UPSERT
        c["handle"] = -1
        c["node_handle"] = self.rng.permutation(self.node_of[loc])
        c["spec_id"] = self.spec
        c["phase"] = abi.PHASE_PENDING
        c["flags"] = abi.POD_STATUS_NONEMPTY
        c["creation_unix"] = now - 5
        self._pending = (D, c["node_handle"].copy(), now - 5)
        return ev, arena

    def _batch_packed(self, D, dead, loc, phase, pip, now):
        r12 = self.packed == 12
        dt = abi.POD_REC12_DTYPE if r12 else abi.POD_REC_DTYPE
        if self.alloc is None:
            ev = np.zeros(2 * D, dt)
        else:
            if self.bufs is None or len(self.bufs[0]) < 2 * D or self.bufs[0].dtype != dt:
                self.bufs = (self.alloc((2 * self.n,), dt),)
            ev = self.bufs[0][:2 * D]
        d = ev[:D]
        running = phase[loc] == abi.PHASE_RUNNING
        fin = np.where(self.rng.random(D) < 0.5, abi.POD_HAS_FINALIZERS, 0)
        d["target"] = dead
        d["spec_id"] = self.spec
        d["flags"] = ((abi.POD_DELETING | fin | np.where(running, abi.POD_CONFORMS | abi.POD_STATUS_NONEMPTY, 0)
                       | np.where(pip[loc] != 0, abi.POD_STATUS_NONEMPTY, 0))
                      | (phase[loc].astype(np.int64) << abi.REC_PHASE_SHIFT))
        c = ev[D:]
        c["target"] = self.rng.permutation(self.node_of[loc])
        c["spec_id"] = self.spec
        c["flags"] = abi.POD_STATUS_NONEMPTY | (abi.PHASE_PENDING << abi.REC_PHASE_SHIFT)
        if r12:  # (the marked pods keep their creationTimestamp; a create's is its value)
            d["op"] = abi.OP_UPSERT | np.where(running, abi.REC_HOST_NODE_IP, 0)
            d["value"] = pip[loc]
            c["op"] = abi.OP_UPSERT | abi.REC_NEW
            c["value"] = now - 5
        else:
            d["op"] = abi.OP_UPSERT
            d["creation"] = self.ctime[loc]
            d["host_ip"] = np.where(running, abi.ip4(self.node_ip.decode()), 0)
            d["pod_ip"] = pip[loc]
            c["op"] = abi.OP_UPSERT | abi.REC_NEW
            c["creation"] = now - 5
            c["host_ip"] = 0
            c["pod_ip"] = 0
        self._pending = (D, c["target"].copy(), now - 5)
        return ev

    def applied(self, handles, status, new_only=False):
        """account the ingest result of the last batch (new_only: handles are the
        creates' only, kwok_ingest_pods_packed12)"""
        D, nodes, ct = self._pending
        assert (status == 0).all(), "churn batch rejected: %s" % np.unique(status[status != 0])
        new = handles[:D] if new_only else handles[D:]
        self.node_of[new - self.first] = nodes
        self.ctime[new - self.first] = ct
        self.live = np.concatenate([self.live[D:], new])


class Flap:
    """BASELINE configs[4], node failure / flap injection under partial
    management: every tick, `frac` of the managed nodes are deleted and created
    again (watch Deleted then Added of a Node with an empty status and the same
    name, node_controller.go:256-270): they drop out of and rejoin the managed
    set (heartbeat handle list epoch), are locked again and get the node-init
    patch (configureNode, :356-391); their pods stay and are re-evaluated."""

    def __init__(self, fleet, frac=0.01, seed=0):
        ev = fleet.node_events
        self.idx = np.nonzero(ev["managed"] != 0)[0]
        self.fleet = fleet
        self.k = max(1, int(len(self.idx) * frac))
        self.rng = np.random.default_rng(seed)

    def batch(self, compact=False, alloc=None):
        """(events, arena): k Deleted records, then k Added records.  compact:
        the batch's own arena of the k names (as a watch client decodes a
        batch into one buffer), in alloc(shape, dtype) memory if given"""
        pick = self.rng.choice(self.idx, self.k, replace=False)
        src = self.fleet.node_events[pick]
        ev = np.concatenate([src, src])
        ev["op"][:self.k] = abi.OP_DELETE
        if not compact:
            return ev, self.fleet.arena
        names = self.fleet.names[pick]
        w = names.shape[1]
        ev["name"]["off"] = np.tile(np.arange(self.k, dtype=np.uint32) * w, 2)
        mk = alloc or (lambda shape, dt: np.empty(shape, dt))
        ar = mk((names.size,), np.uint8)
        ar[:] = names.reshape(-1)
        evp = mk((len(ev),), abi.NODE_EVENT_DTYPE)
        evp[:] = ev
        return evp, ar


    # the node documents a watch carries for a flap (batch_json): the Deleted event holds the
    # node as kwok patched it (node.status.tpl's init patch: addresses, allocatable, capacity,
    # nodeInfo, phase, conditions), the Added event a Node created again with a zero status
    # (json.Marshal of corev1.Node: daemonEndpoints and the ten nodeInfo strings always present)
    _NI_ZERO = (b'"nodeInfo":{"machineID":"","systemUUID":"","bootID":"","kernelVersion":"","osImage":"",'
                b'"containerRuntimeVersion":"","kubeletVersion":"","kubeProxyVersion":"","operatingSystem":"",'
                b'"architecture":""}')
    _DEL_STATUS = (b'"status":{"capacity":{"cpu":"1k","memory":"1Ti","pods":"1M"},'
                   b'"allocatable":{"cpu":"1k","memory":"1Ti","pods":"1M"},"conditions":[{"type":"Ready",'
                   b'"status":"True","lastHeartbeatTime":"2024-01-01T00:00:00Z","lastTransitionTime":'
                   b'"2024-01-01T00:00:00Z","reason":"KubeletReady","message":"kubelet is posting ready status"}],'
                   b'"addresses":[{"type":"InternalIP","address":"196.168.0.1"}],"daemonEndpoints":'
                   b'{"kubeletEndpoint":{"Port":0}},"nodeInfo":{"machineID":"","systemUUID":"","bootID":"",'
                   b'"kernelVersion":"","osImage":"","containerRuntimeVersion":"","kubeletVersion":"fake",'
                   b'"kubeProxyVersion":"fake","operatingSystem":"linux","architecture":"amd64"},"phase":"Running"}')

    def _doc(self, name, lockable, deleted, serial):
        ann = b'"kwok.x-k8s.io/node":"fake"' + (b'' if lockable else b',"kwok.x-k8s.io/status":"custom"')
        md = (b'"metadata":{"name":"' + name + b'","uid":"7d3c0e9a-0000-4000-8000-%012d",' % serial +
              b'"resourceVersion":"%d","creationTimestamp":"2024-01-01T00:00:00Z","annotations":{' % (1000 + serial) +
              ann + b'}}')
        st = self._DEL_STATUS if deleted else b'"status":{"daemonEndpoints":{"kubeletEndpoint":{"Port":0}},' + \
            self._NI_ZERO + b'}'
        return b'{"kind":"Node","apiVersion":"v1",' + md + b',"spec":{},' + st + b'}'

    def batch_json(self):
        """the same batch as batch() (k Deleted, then k Added), as the watch's node
        documents: (arena, offs, lens, ops, events) - events: batch()'s records"""
        pick = self.rng.choice(self.idx, self.k, replace=False)
        src = self.fleet.node_events[pick]
        names = self.fleet.names[pick]
        docs = []
        serial = getattr(self, "serial", 0)
        for deleted in (True, False):
            for q in range(self.k):
                docs.append(self._doc(names[q].tobytes(), bool(src["lockable"][q]), deleted, serial))
                serial += 1
        self.serial = serial
        lens = np.fromiter((len(d) for d in docs), np.uint32, len(docs))
        offs = np.zeros(len(docs), np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        ops = np.full(len(docs), abi.OP_UPSERT, np.uint8)
        ops[:self.k] = abi.OP_DELETE
        ev = np.concatenate([src, src])
        ev["op"][:self.k] = abi.OP_DELETE
        return b"".join(docs), offs, lens, ops, ev


# ---- the C4 storm as the documents a watch carries (kwok_ingest_pods_json) ----
def rfc3339_rows(t: np.ndarray) -> np.ndarray:
    """RFC3339 UTC strings of unix seconds as a (n, 20) uint8 array"""
    import time as _time
    t = np.asarray(t, np.int64)
    u, inv = np.unique(t, return_inverse=True)
    rows = np.frombuffer(b"".join(_time.strftime("%Y-%m-%dT%H:%M:%SZ", _time.gmtime(int(x))).encode() for x in u),
                         np.uint8).reshape(len(u), 20)
    return rows[inv.reshape(-1)]


def _digits(v: np.ndarray, width: int) -> np.ndarray:
    v = np.asarray(v, np.int64)
    out = np.empty((v.shape[0], width), np.uint8)
    for k in range(width):
        out[:, width - 1 - k] = ord("0") + (v // 10 ** k) % 10
    return out


class DocTemplate:
    """A JSON document with fixed-width slots, filled for many documents at
    once (numpy): `text` with slot markers {name} of the slot's width in
    placeholder bytes '@'.  Variable-length strings go in a slot followed by
    spaces (whitespace between tokens), e.g. an IP `"10.0.0.5"` in a 17-byte
    slot."""

    def __init__(self, text: str, widths: dict):
        import re
        parts = re.split(r"\{(\w+)\}", text)
        buf, self.slots = bytearray(), {}
        for i, p in enumerate(parts):
            if i % 2:
                self.slots.setdefault(p, []).append((len(buf), widths[p]))
                buf += b"@" * widths[p]
            else:
                buf += p.encode()
        self.tpl = np.frombuffer(bytes(buf), np.uint8)

    def fill(self, n: int, values: dict, out=None, static=True) -> np.ndarray:
        """n documents into out ((n, len) uint8, allocated if None); static=False:
        only the slots are written (out already holds the template)"""
        if out is None:
            out = np.empty((n, self.tpl.size), np.uint8)
        if static:
            out[...] = self.tpl[None, :]
        for name, where in self.slots.items():
            v = values[name]
            for off, w in where:
                out[:, off:off + w] = v if v.ndim == 2 else v[None, :]
        return out


def quoted_ips(ips: np.ndarray, width: int = 17) -> np.ndarray:
    """`"a.b.c.d"` + spaces, (n, width) uint8 (net.IP.String() of each address)"""
    buf, off, ln = ip_strings(ips)
    n = len(ips)
    out = np.full((n, width), ord(" "), np.uint8)
    out[:, 0] = ord('"')
    for k in range(15):
        m = k < ln
        out[m, 1 + k] = buf[off[m] + k]
    out[np.arange(n), 1 + ln] = ord('"')
    return out


_META = ('{"metadata":{"name":"{name}","namespace":"default","uid":"{uid}","resourceVersion":"{rv}",'
         '"creationTimestamp":"{ct}",')
_SPEC = ('"spec":{"containers":[{"name":"fake-pod","image":"fake","resources":{},'
         '"terminationMessagePath":"/dev/termination-log","terminationMessagePolicy":"File",'
         '"imagePullPolicy":"Always"}],"restartPolicy":"Always","terminationGracePeriodSeconds":30,'
         '"dnsPolicy":"ClusterFirst","serviceAccountName":"default","serviceAccount":"default","nodeName":"{node}",'
         '"securityContext":{},"schedulerName":"default-scheduler","tolerations":[{"key":"node.kubernetes.io/not-ready",'
         '"operator":"Exists","effect":"NoExecute","tolerationSeconds":300},{"key":"node.kubernetes.io/unreachable",'
         '"operator":"Exists","effect":"NoExecute","tolerationSeconds":300}],"priority":0,"enableServiceLinks":true,'
         '"preemptionPolicy":"PreemptLowerPriority"},')
_COND = '{"type":"%s","status":"True","lastProbeTime":null,"lastTransitionTime":"{ct}"}'
# a Running pod kwok patched (pod.status.tpl's fields as the apiserver stores them), now marked for deletion
DELETING_DOC = DocTemplate(
    _META + '"deletionTimestamp":"{dt}","deletionGracePeriodSeconds":0,"labels":{"app":"fake"},"finalizers":{fin}},'
    + _SPEC + '"status":{"phase":"Running","conditions":[' + ",".join(_COND % t for t in (
        "Initialized", "Ready", "ContainersReady")).replace("{ct}", "{ct2}") +
    '],"hostIP":{hip},"podIP":{pip},"podIPs":[{"ip":{pip}}],"startTime":"{ct3}","containerStatuses":[{"name":'
    '"fake-pod","state":{"running":{"startedAt":"{ct4}"}},"lastState":{},"ready":true,"restartCount":0,'
    '"image":"fake","imageID":""}],"qosClass":"BestEffort"}}',
    dict(name=12, uid=36, rv=8, ct=20, ct2=20, ct3=20, ct4=20, dt=20, fin=22, node=12, hip=17, pip=17))
# a new Pending pod, scheduled (spec.nodeName) and defaulted by the apiserver
PENDING_DOC = DocTemplate(_META + '"labels":{"app":"fake"}},' + _SPEC +
                          '"status":{"phase":"Pending","qosClass":"BestEffort"}}',
                          dict(name=12, uid=36, rv=8, ct=20, node=12))


class ChurnJson(Churn):
    """Churn's storm as Kubernetes documents (kwok_ingest_pods_json): the
    deletion-marked pods as the Running objects kwok patched (full status,
    deletionTimestamp, half with a finalizer), the creates as scheduled Pending
    pods, ~1.6 KB / ~1.1 KB each.  node_name_of[handle]: the (12,) name bytes
    of each node handle (the fleet's names)."""

    def __init__(self, *a, node_name_of=None, **kw):
        super().__init__(*a, **kw)
        self.node_name_of = node_name_of
        self.serial = 0

    @classmethod
    def from_churn(cls, ch, node_name_of, alloc=None):
        """the storm continued from another Churn's live pods, as documents"""
        x = cls.__new__(cls)
        x.__dict__.update(ch.__dict__)
        x.node_name_of, x.serial, x.alloc, x.packed, x.bufs, x.jbuf = node_name_of, 0, alloc, False, None, None
        return x

    def names(self, n):
        s = np.arange(self.serial, self.serial + n, dtype=np.int64)
        self.serial += n
        name = np.empty((n, 12), np.uint8)
        name[:, :4] = np.frombuffer(b"pod-", np.uint8)
        name[:, 4:] = _digits(s, 8)
        uid = np.broadcast_to(np.frombuffer(b"0b7f2c2e-0000-4000-8000-", np.uint8), (n, 24))
        return name, np.concatenate([uid, _digits(s, 12)], axis=1), _digits(s % 10 ** 8, 8)

    def batch_json(self, dump, now):
        D = min(self.n, self.live.shape[0])
        dead = self.live[:D]
        loc = dead - self.first
        used, phase, _, pip = dump()
        assert used[loc].all() and (phase[loc] == abi.PHASE_RUNNING).all(), "churn: live Running pods"
        nm, uid, rv = self.names(D)
        ct = rfc3339_rows(self.ctime[loc])
        fin = self.rng.random(D) < 0.5
        finb = np.full((D, 22), ord(" "), np.uint8)
        finb[:, :2] = np.frombuffer(b"[]", np.uint8)
        finb[fin] = np.frombuffer(b'["kwok.x-k8s.io/fake"]', np.uint8)
        ips = quoted_ips(pip[loc])
        # the documents live in one buffer (self.alloc'ed: page-locked), the templates written once;
        # every batch rewrites the slots only
        Ld, Lc = DELETING_DOC.tpl.size, PENDING_DOC.tpl.size
        static = getattr(self, "jbuf", None) is None or self.jbuf.size < D * (Ld + Lc) or self.jD != D
        if static:
            mk = self.alloc or (lambda shape, dt: np.empty(shape, dt))
            self.jbuf = mk((D * (Ld + Lc),), np.uint8)
            self.jD = D
        d = self.jbuf[:D * Ld].reshape(D, Ld)
        c = self.jbuf[D * Ld:D * (Ld + Lc)].reshape(D, Lc)
        DELETING_DOC.fill(D, dict(name=nm, uid=uid, rv=rv, ct=ct, ct2=ct, ct3=ct, ct4=ct,
                                  dt=rfc3339_rows(np.full(1, now))[0], fin=finb,
                                  node=self.node_name_of[self.node_of[loc]],
                                  hip=quoted_ips(np.array([abi.ip4(self.node_ip.decode())], np.uint32))[0],
                                  pip=ips), out=d, static=static)
        nodes = self.rng.permutation(self.node_of[loc])
        nm2, uid2, rv2 = self.names(D)
        PENDING_DOC.fill(D, dict(name=nm2, uid=uid2, rv=rv2, ct=rfc3339_rows(np.full(1, now - 5))[0],
                                 node=self.node_name_of[nodes]), out=c, static=static)
        arena = self.jbuf[:D * (Ld + Lc)]
        lens = np.concatenate([np.full(D, Ld, np.uint32), np.full(D, Lc, np.uint32)])
        offs = np.zeros(2 * D, np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        ops = np.full(2 * D, abi.OP_UPSERT, np.uint8)
        handles = np.concatenate([dead, np.full(D, -1, np.int32)]).astype(np.int32)
        self._pending = (D, nodes.copy(), now - 5)
        return arena, offs, lens, ops, handles


def node_names_by_handle(fl) -> np.ndarray:
    """(max handle + 1, 12) name bytes of the fleet's node handles"""
    out = np.zeros((int(fl.node_handles.max()) + 1, 12), np.uint8)
    out[fl.node_handles] = fl.names
    return out


def host_decode_arrays(codec, arena, offs, lens, threads=8):
    """kwok_decode_pods (the host codec) over documents already in one arena:
    {"ev": POD_EVENT_DTYPE, "names": (n, 2, 2) u32, "status": i32}"""
    import ctypes as C
    n = len(offs)
    rec = np.zeros(n * C.sizeof(abi.PodDoc), np.uint8)
    st = np.zeros(n, np.int32)
    a = np.ascontiguousarray(arena, np.uint8)
    o = np.ascontiguousarray(offs, np.uint64)
    ln = np.ascontiguousarray(lens, np.uint32)
    codec._lib.kwok_decode_pods(codec._h, a.ctypes.data, a.nbytes, o.ctypes.data, ln.ctypes.data, n, threads,
                                rec.ctypes.data, st.ctypes.data)
    r = rec.reshape(n, C.sizeof(abi.PodDoc))
    ev = np.ascontiguousarray(r[:, :48]).view(abi.POD_EVENT_DTYPE).reshape(n)
    names = np.ascontiguousarray(r[:, 48:64]).view(np.uint32).reshape(n, 2, 2)
    return {"ev": ev, "names": names, "status": st}
