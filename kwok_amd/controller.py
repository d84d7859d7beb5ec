"""The drop-in controller: the reference's Controller API over the engine.

This is the Python restatement of the Go drop-in
(integration/go/pkg/kwok/controllers/gpu_controller.go + engine_cgo.go), call
for call, so that its ingest / tick / apply sequence runs in the tests against
a fake clientset (tests/fake_clientset.py) the way the reference's unit tests
run NodeController / PodController against client-go's fake clientset
(node_controller_test.go:37-155, pod_controller_test.go:37-194).

Reference interface it stands in for (hezhizhen/kwok, pkg/kwok/controllers):
  Config                 controller.go:64-77
  NewController / Start  controller.go:80-164 (the loop replaces KeepNodeHeartbeat
                         node_controller.go:175-204, LockNodes :301-329, LockPods
                         pod_controller.go:234-250, DeletePods :186-202)
  Has / Size             node_controller.go:403-409
  watch routing          node_controller.go:256-270, pod_controller.go:301-343
                         (the host codec, kwok_decode_*, then kwok_ingest_*)
  apply                  PatchStatus node_controller.go:152,345; Patch status
                         pod_controller.go:221; finalizer Patch + Delete :161-174

Per tick (step):
  1. the watch events since the last tick, minus the ECHOES of the engine's own
     patches: an event whose resourceVersion is the one a patch of the engine
     returned for that object is the state the engine already assumed (DESIGN.md
     §1: patches are assumed applied; the heartbeat echo's re-lock,
     node_controller.go:152 -> :256-263, is part of every tick), so it is dropped
     instead of re-ingested.  Echoes that arrive after their patch returned are
     dropped on arrival (not queued, not encoded); those that overtake their
     patch's response are dropped here, when every apply has returned.  An echo
     that follows another event of its object in the same batch is kept: that
     event is a change the engine has not seen, older than the patch, and the
     echo is the newest state, carrying both;
  2. node events -> JSON -> kwok_decode_nodes -> kwok_ingest_nodes;
  3. pod events -> JSON -> kwok_decode_pods -> kwok_ingest_pods, in runs in which
     no new pod appears twice (a pod's second event needs the handle its first
     one created: Added + Modified, Added + Deleted in one interval);
  4. EnableCNI: cni.Setup for the pods the tick will evaluate without a podIP
     (kwok_cni_pending / kwok_cni_assign, pod_controller.go:383-389);
  5. kwok_tick at the fixed clock; the lists (kwok_read_outputs without an arena),
     ONE heartbeat body (the engine is created with KWOK_CFG_HEARTBEAT_ONCE) sent
     to every managed node, node-init and pod patches read in pieces of at most
     READ_CHUNK bytes (kwok_read_arena), deletes; every body applied through the
     clientset, every returned resourceVersion noted as an echo;
  6. the same interval again for pods patched without a podIP (created with an
     empty status: pod.status.tpl renders no IPs then, `{{ with .status }}`):
     in the reference that patch's own Modified event re-enters lockPodChan
     (pod_controller.go:279-319) and the pod gets hostIP / podIP at once.  Here
     the object the patch returned is ingested as that event (its watch echo is
     then dropped like every echo) and the engine ticks again at the same clock;
     that tick's pod patches, node inits and deletes are applied, its heartbeats
     are not (the interval's heartbeats were sent).

The backend is the HIP engine; tests may pass another implementation of the
same ABI (the CPU oracle) as the checker.
"""
from __future__ import annotations

import ctypes as C
import json
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .codec import Codec
from .engine import Engine, make_config

READ_CHUNK = 64 << 20  # engine_cgo.go readChunk

HEARTBEAT, NODE_INIT, POD_PATCH, DELETE, DELETE_FIN = range(5)  # engine_cgo.go kind*


NOT_SENT = 1  # ingest_pod_runs: a record not sent to the engine (a Deleted event of an unknown pod)


def ingest_pods_wire(eng, recs, arena):
    """engine_cgo.go ingestPods: every record the compact wire forms can carry
    (kwok_pack_pod_events: IPs as integers, a new pod's node by handle) as a
    12-byte kwok_pod_rec12 through kwok_ingest_pods_packed12 when its hostIP is
    empty or the engine's NodeIP (every pod kwok runs) and it is no create
    holding a podIP, else as a 20-byte kwok_pod_rec through
    kwok_ingest_pods_packed, and the rest (a pod naming a node the engine holds
    no handle for) as kwok_pod_event through kwok_ingest_pods; consecutive
    records of one form in one call, in event order (applying the calls in order
    is applying the batch).  Returns (handles, statuses, released, calls)."""
    from .engine import pack_pod_events
    packed, pst = pack_pod_events(recs, arena)
    n = len(recs)
    node_ip = eng.node_ip
    ok = pst == abi.OK
    hip = packed["host_ip"]
    new = (packed["op"] & abi.REC_NEW) != 0
    small = ((hip == 0) | (hip == node_ip)) & ~(new & (packed["pod_ip"] != 0))
    form = np.where(ok, np.where(small, 12, 20), 0)
    hs, st, rel = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.uint32)
    i = calls = 0
    while i < n:
        f = form[i]
        j = i + 1
        while j < n and form[j] == f:
            j += 1
        if f == 12:
            r12 = abi.pack12(packed[i:j], node_ip)
            nh, st[i:j], rel[i:j] = eng.ingest_pods_packed12(r12)
            nw = (r12["op"] & abi.REC_NEW) != 0
            hs[i:j] = r12["target"]  # every other record's handle is its target
            hs[i:j][nw] = nh
        elif f == 20:
            hs[i:j], st[i:j], rel[i:j] = eng.ingest_pods_packed(packed[i:j])
        else:
            hs[i:j], st[i:j], rel[i:j] = eng.ingest_pods_raw(recs[i:j], arena)
        calls += 1
        i = j
    return hs, st, rel, calls


def ingest_pod_runs(eng, pod_by_uid, recs, uids, deleted, arena, sender=None):
    """gpu_controller.go flushPods' ingest, on decoded records: the batch in
    event order, cut into runs in which no new pod appears twice - a pod's first
    event in the batch may create it (handle -1) and its later events need that
    handle, so run k+1 is ingested once run k's handles are known (Added +
    Modified, or Added + Deleted with its podIP release, pod_controller.go:
    329-336, within one interval).  A Deleted event names the pod's handle; one
    for a pod the engine never held (or already deleted) is not sent.  recs:
    POD_EVENT_DTYPE with spec_id / node_handle set for upserts (op and handle are
    set here); uids: hashable per record; pod_by_uid: the caller's uid -> handle
    map, updated.  Returns (handles, statuses, runs): per record, NOT_SENT for
    those not sent.  sender(idx, ops, handles) -> (handles, statuses): another
    ingest of the records idx (the documents on the GPU codec, ingest_doc_runs);
    recs is then only its length."""
    n = len(recs)
    uids = list(uids)
    deleted = np.asarray(deleted, bool)
    hs = np.full(n, -1, np.int32)
    st = np.full(n, NOT_SENT, np.int32)
    runs = 0

    def flush(lo, hi):
        nonlocal runs
        idx = np.arange(lo, hi)
        hv = np.fromiter((pod_by_uid.get(uids[i], -1) for i in range(lo, hi)), np.int64, hi - lo)
        dl = deleted[lo:hi]
        send = ~dl | (hv >= 0)
        idx, hv, dl = idx[send], hv[send], dl[send]
        if not len(idx):
            return
        ops = np.where(dl, abi.OP_DELETE, abi.OP_UPSERT)
        if sender is not None:
            h1, s1 = sender(idx, ops, hv)
        else:
            recs["op"][idx] = ops
            recs["handle"][idx] = hv
            h1, s1, _rel, _calls = ingest_pods_wire(eng, recs[idx], arena)
        runs += 1
        hs[idx], st[idx] = h1, s1
        for k in np.nonzero(s1 == abi.OK)[0].tolist():
            i = int(idx[k])
            if dl[k]:
                pod_by_uid.pop(uids[i], None)
            else:
                pod_by_uid[uids[i]] = int(h1[k])

    lo, created = 0, set()
    for i in range(n):
        u = uids[i]
        if u in created:  # its handle comes from the run before
            flush(lo, i)
            lo = i
            created.clear()
        if not deleted[i] and u not in pod_by_uid:
            created.add(u)
    flush(lo, n)
    return hs, st, runs


def ingest_doc_runs(eng, codec, pod_by_uid, docs, uids, deleted):
    """gpu_controller.go flushPodsJSON: the batch's pod documents decoded on the
    GPU (kwok_ingest_pods_json: k_json_pods, the host codec only for the
    documents the device leaves undecided, specs registered as they appear, the
    records never leaving HBM), in the same runs as ingest_pod_runs.  Returns
    (handles, statuses, runs, documents the host decided)."""
    arena, offs, lens = Engine._docs(docs)
    n_host = [0]

    def send(idx, ops, hv):
        hs, st, _rel, nh = eng.ingest_pods_json(codec, arena, offs[idx], lens[idx], ops.astype(np.uint8),
                                                hv.astype(np.int32))
        n_host[0] += nh
        return hs, st

    hs, st, runs = ingest_pod_runs(eng, pod_by_uid, np.empty(len(docs)), uids, deleted, None, sender=send)
    return hs, st, runs, n_host[0]


class NotFound(Exception):
    """apierrors.IsNotFound: tolerated by LockPod / DeletePod (pod_controller.go:164,174,224)"""


@dataclass
class Config:
    """controller.go:64-77 (Go field names in snake case).  Templates: None =
    templates.Default*.  start_time: the StartTime() value (controller.go:33),
    injected as the reference tests inject their FuncMap."""
    client_set: object
    enable_cni: bool = False
    manage_all_nodes: bool = False
    manage_nodes_with_annotation_selector: str = ""
    manage_nodes_with_label_selector: str = ""
    disregard_status_with_annotation_selector: str = ""
    disregard_status_with_label_selector: str = ""
    cidr: str = "10.0.0.1/24"
    node_ip: str = "196.168.0.1"
    pod_status_template: str | None = None
    node_initialization_template: str | None = None
    node_heartbeat_template: str | None = None
    start_time: int = 1704067200
    cni: object = None  # EnableCNI: .setup(uid, name, namespace) -> [ip, ...]; .remove(uid, name, namespace)


@dataclass
class WatchObj:
    obj: dict
    uid: str
    rv: str
    deleted: bool


class Echoes:
    """gpu_controller.go echoes: the resourceVersions the engine's own patches
    returned, per object.  An object can take several patches in one tick (a
    node's heartbeat and its init patch; a pod's finalizer patch), each with its
    own echo, so every returned version is kept until its echo is seen (the last
    ECHO_KEEP per object: echoes lost to a watch restart do not pile up)."""

    ECHO_KEEP = 8

    def __init__(self):
        self.rv = {}

    def note(self, uid, rv):
        if uid and rv:
            v = self.rv.setdefault(uid, [])
            v.append(rv)
            if len(v) > self.ECHO_KEEP:
                del v[0]

    def is_echo(self, uid, rv):
        v = self.rv.get(uid)
        if v and rv in v:
            v.remove(rv)
            if not v:
                del self.rv[uid]
            return True
        return False

    def forget(self, uid):
        self.rv.pop(uid, None)


@dataclass
class Stats:
    """what the controller did (tests read it; the Go shim logs it)"""
    echoes_on_arrival: int = 0
    echoes_at_flush: int = 0
    reentered: int = 0    # pods patched without a podIP, ingested again in the same interval
    node_records: int = 0
    pod_records: int = 0
    pod_docs_host: int = 0  # pod documents the GPU codec left to the host codec
    node_docs_host: int = 0  # node documents the GPU codec left to the host codec
    pod_runs: int = 0
    bodies: int = 0
    rejected: list = field(default_factory=list)


def _meta(obj):
    return obj.get("metadata") or {}


class Controller:
    """NewController(conf) + Start: the engine-backed controller."""

    # engine_cgo.go newGPUEngine's geometry (tests pass a smaller one for the CPU oracle,
    # which holds every bucket at its full handle stride)
    GEOMETRY = dict(buckets=4096, node_slots_per_bucket=64, pod_slots_per_bucket=640, pod_handle_stride=65528,
                    max_pod_specs=4096)

    def __init__(self, conf: Config, backend=None, codec_threads=1, suppress_echoes=True, geometry=None,
                 gpu_codec=True):
        self.conf = conf
        self.suppress = suppress_echoes  # False: every echo re-ingested (tests: the A/B that echoes change nothing)
        custom = {}
        if conf.pod_status_template is not None:
            custom["pod_status_template"] = conf.pod_status_template
        if conf.node_initialization_template is not None:
            custom["node_init_template"] = conf.node_initialization_template
        if conf.node_heartbeat_template is not None:
            custom["node_heartbeat_template"] = conf.node_heartbeat_template
        # engine_cgo.go newGPUEngine: the same geometry and KWOK_CFG_HEARTBEAT_ONCE
        geo = dict(self.GEOMETRY, **(geometry or {}))
        cfg = make_config(cidr=conf.cidr, node_ip=conf.node_ip, start_time=conf.start_time,
                          enable_cni=conf.enable_cni, heartbeat_once=True, **geo, **custom)
        self.eng = (backend or Engine)(cfg)
        self.codec = Codec(manage_all_nodes=conf.manage_all_nodes,
                           manage_nodes_with_annotation_selector=conf.manage_nodes_with_annotation_selector,
                           manage_nodes_with_label_selector=conf.manage_nodes_with_label_selector,
                           disregard_status_with_annotation_selector=conf.disregard_status_with_annotation_selector,
                           disregard_status_with_label_selector=conf.disregard_status_with_label_selector)
        self.threads = codec_threads
        # node and pod documents decoded on the GPU (kwok_ingest_nodes_json / kwok_ingest_pods_json)
        # when the backend has them (the CPU oracle backend takes the host codec)
        self.gpu_codec = gpu_codec and hasattr(self.eng, "ingest_pods_json")
        self.nodes: list[WatchObj] = []
        self.pods: list[WatchObj] = []
        self.queued = set()  # uids with an event in the current batch
        self.echo = Echoes()
        self.stats = Stats()
        self.node_name = {}   # node handle -> name
        self.node_handle = {}  # name -> node handle
        self.pod_by_uid = {}
        self.pod_uid = {}     # pod handle -> uid
        self.pod_ref = {}     # pod handle -> (namespace, name)
        self.hb = None        # heartbeat handle list of epoch hb_epoch
        self.hb_epoch = None
        self.spec_ids = {}
        self.finalizer = None
        self.reenter = []     # objects of pod patches without a podIP (step 6)

    def close(self):
        self.eng.close()
        self.codec.close()

    # ---- Start: the watches (node_controller.go:119-143, pod_controller.go:130-153) ----
    def start(self):
        cs = self.conf.client_set
        cs.watch("nodes", lambda typ, obj: self.on_event(True, typ, obj),
                 label_selector=self.conf.manage_nodes_with_label_selector)
        cs.watch("pods", lambda typ, obj: self.on_event(False, typ, obj), field_selector="spec.nodeName!=")

    def on_event(self, nodes: bool, typ: str, obj: dict):
        if typ not in ("ADDED", "MODIFIED", "DELETED"):
            return
        md = _meta(obj)
        w = WatchObj(obj, md.get("uid", ""), md.get("resourceVersion", ""), typ == "DELETED")
        # an echo is dropped only while no other event of its object waits in this
        # tick's batch: after one (a change the engine has not seen, older than the
        # engine's patch) the echo is the object's newest state - it carries both
        if self.suppress and typ == "MODIFIED" and self.echo.is_echo(w.uid, w.rv) and w.uid not in self.queued:
            self.stats.echoes_on_arrival += 1
            return
        self.queued.add(w.uid)
        (self.nodes if nodes else self.pods).append(w)

    # ---- Has / Size (node_controller.go:403-409) ----------------------------------
    def has(self, name: str) -> bool:
        return bool(name) and self.eng.node_has(name)

    def size(self) -> int:
        return self.eng.node_size()

    # ---- one heartbeat interval (the loop's timer body) ---------------------------
    def step(self, now: int) -> int:
        nw, pw = self.nodes, self.pods
        self.nodes, self.pods, self.queued = [], [], set()
        nb = self._encode(nw)
        pb = self._encode(pw)
        self._flush_nodes(nb)
        self._flush_pods(pb)
        if self.conf.enable_cni:
            self._setup_cni()
        n = self._tick(now)
        # step 6: pods patched without a podIP re-enter at once (pod_controller.go:279-319)
        for _ in range(4):  # (a re-entered pod's second patch carries its IPs: one round suffices)
            if not self.reenter:
                break
            objs, self.reenter = self.reenter, []
            self.stats.reentered += len(objs)
            ws = [WatchObj(o, _meta(o).get("uid", ""), _meta(o).get("resourceVersion", ""), False) for o in objs]
            self._flush_pods((ws, [json.dumps(w.obj, separators=(",", ":")).encode() for w in ws]))
            if self.conf.enable_cni:
                self._setup_cni()
            n += self._tick(now, heartbeats=False)
        return n

    def _encode(self, ws):
        keep, seen = [], set()
        for w in ws:
            # (the same rule as on arrival: only before any kept event of the object)
            if self.suppress and not w.deleted and self.echo.is_echo(w.uid, w.rv) and w.uid not in seen:
                self.stats.echoes_at_flush += 1
                continue
            seen.add(w.uid)
            keep.append(w)
            if w.deleted:  # the object's last event: echoes still noted for it will not come
                self.echo.forget(w.uid)
        return keep, [json.dumps(w.obj, separators=(",", ":")).encode() for w in keep]

    def _flush_nodes(self, batch):
        """gpu_controller.go flushNodes: on the HIP engine the documents are decoded on
        the GPU (kwok_ingest_nodes_json); a backend without it takes the host codec"""
        ws, docs = batch
        if not ws:
            return
        if self.gpu_codec:
            return self._flush_nodes_gpu(ws, docs)
        b = self.codec.decode_nodes(docs, strict=False, threads=self.threads)
        keep, names = [], []
        for i, w in enumerate(ws):
            if b.status[i] != abi.OK:  # outside the engine's domain: not simulated
                self.stats.rejected.append(("node", _meta(w.obj).get("name"), b.status[i]))
                continue
            r = np.frombuffer(bytes(b.nodes[i]), abi.NODE_EVENT_DTYPE).copy()
            r["op"] = abi.OP_DELETE if w.deleted else abi.OP_UPSERT
            keep.append(r)
            names.append(b.text(b.nodes[i].name))
        if not keep:
            return
        recs = np.concatenate(keep)
        hs, st = self.eng.ingest_nodes_raw(recs, bytes(b.buf))
        self.stats.node_records += len(recs)
        for k in range(len(recs)):
            if st[k] != abi.OK:
                continue
            if recs[k]["op"] == abi.OP_DELETE:
                self.node_name.pop(int(hs[k]), None)
                self.node_handle.pop(names[k], None)
            else:
                self.node_name[int(hs[k])] = names[k]
                self.node_handle[names[k]] = int(hs[k])

    def _flush_nodes_gpu(self, ws, docs):
        """gpu_controller.go flushNodes on the device codec: the documents straight to
        kwok_ingest_nodes_json (a Deleted event's status is not read); names from the
        watch objects"""
        arena, offs, lens = Engine._docs(docs)
        ops = np.array([abi.OP_DELETE if w.deleted else abi.OP_UPSERT for w in ws], np.uint8)
        hs, st, nh = self.eng.ingest_nodes_json(self.codec, arena, offs, lens, ops)
        self.stats.node_docs_host += nh
        self.stats.node_records += int(np.isin(st, (abi.EDOMAIN, abi.EINVAL), invert=True).sum())
        for k, w in enumerate(ws):
            name = _meta(w.obj).get("name", "")
            if st[k] != abi.OK:
                if st[k] in (abi.EDOMAIN, abi.EINVAL):  # outside the engine's domain: not simulated
                    self.stats.rejected.append(("node", name, int(st[k])))
                continue
            if w.deleted:
                self.node_name.pop(int(hs[k]), None)
                self.node_handle.pop(name, None)
            else:
                self.node_name[int(hs[k])] = name
                self.node_handle[name] = int(hs[k])

    def _spec_id(self, b, d):
        spec = (tuple((b.text(c.name), b.text(c.image)) for c in d.containers[:d.n_containers]),
                tuple((b.text(c.name), b.text(c.image)) for c in d.init_containers[:d.n_init_containers]),
                tuple(b.text(g) for g in d.readiness_gates[:d.n_readiness_gates]))
        sid = self.spec_ids.get(spec)
        if sid is None:
            sid = self.spec_ids[spec] = self.eng.register_pod_spec(*spec)
        return sid

    def _flush_pods(self, batch):
        """gpu_controller.go flushPods: decode, then ingest in runs (ingest_pod_runs).
        On the HIP engine the documents are decoded on the GPU (ingest_doc_runs);
        a backend without kwok_ingest_pods_json (the CPU oracle) takes the host codec."""
        ws, docs = batch
        if not ws:
            return
        if self.gpu_codec:
            return self._flush_pods_gpu(ws, docs)
        b = self.codec.decode_pods(docs, strict=False, threads=self.threads)
        idx, recs = [], []
        for i, w in enumerate(ws):
            if b.status[i] != abi.OK:
                self.stats.rejected.append(("pod", _meta(w.obj).get("name"), b.status[i]))
                continue
            d = b.pods[i]
            r = np.frombuffer(bytes(d.ev), abi.POD_EVENT_DTYPE).copy()
            if w.deleted:
                # EnableCNI: cni.Remove for a pod on a managed node (pod_controller.go:337-342),
                # also when the engine deleted it already (its handle is gone)
                if self.conf.enable_cni and self.conf.cni and self.has(b.text(d.ev.node_name)):
                    self.conf.cni.remove(w.uid, b.text(d.name), b.text(d.namespace_))
            else:
                try:
                    r["spec_id"] = self._spec_id(b, d)
                except Exception as ex:  # KWOK_EDOMAIN: outside the supported domain
                    self.stats.rejected.append(("pod-spec", b.text(d.name), str(ex)))
                    continue
                # the node by handle when the engine holds it; otherwise by spec.nodeName
                r["node_handle"] = self.node_handle.get(b.text(d.ev.node_name), -1)
            idx.append(i)
            recs.append(r)
        if not recs:
            return
        recs = np.concatenate(recs)
        uids = [ws[i].uid for i in idx]
        deleted = [ws[i].deleted for i in idx]
        refs = [(b.text(b.pods[i].namespace_), b.text(b.pods[i].name)) for i in idx]
        hs, st, runs = ingest_pod_runs(self.eng, self.pod_by_uid, recs, uids, deleted, bytes(b.buf))
        self.stats.pod_records += int((st != NOT_SENT).sum())
        self.stats.pod_runs += runs
        for k in range(len(recs)):
            if st[k] != abi.OK:
                continue
            h = int(hs[k])
            if deleted[k]:
                self.pod_uid.pop(h, None)
                self.pod_ref.pop(h, None)
            else:
                self.pod_uid[h] = uids[k]
                self.pod_ref[h] = refs[k]

    def _flush_pods_gpu(self, ws, docs):
        """gpu_controller.go flushPodsJSON: the documents straight to
        kwok_ingest_pods_json in runs; names and nodes from the watch objects"""
        uids = [w.uid for w in ws]
        deleted = [w.deleted for w in ws]
        hs, st, runs, n_host = ingest_doc_runs(self.eng, self.codec, self.pod_by_uid, docs, uids, deleted)
        self.stats.pod_records += int((st != NOT_SENT).sum())
        self.stats.pod_runs += runs
        self.stats.pod_docs_host += n_host
        for k, w in enumerate(ws):
            md = _meta(w.obj)
            if st[k] not in (abi.OK, NOT_SENT):
                self.stats.rejected.append(("pod", md.get("name"), int(st[k])))
                continue
            if w.deleted:
                # EnableCNI: cni.Remove for a pod on a managed node (pod_controller.go:337-342),
                # also when the engine deleted it already (its handle is gone)
                if self.conf.enable_cni and self.conf.cni and self.has((w.obj.get("spec") or {}).get("nodeName", "")):
                    self.conf.cni.remove(w.uid, md.get("name", ""), md.get("namespace", ""))
                if st[k] == abi.OK:
                    self.pod_uid.pop(int(hs[k]), None)
                    self.pod_ref.pop(int(hs[k]), None)
            else:
                h = int(hs[k])
                self.pod_uid[h] = w.uid
                self.pod_ref[h] = (md.get("namespace", ""), md.get("name", ""))

    def _setup_cni(self):
        hs = self.eng.cni_pending()
        if not len(hs):
            return
        keep, ips = [], []
        for h in hs:
            uid, (ns, name) = self.pod_uid[int(h)], self.pod_ref[int(h)]
            try:
                got = self.conf.cni.setup(uid, name, ns)
            except Exception:  # a failed Setup leaves the pod unpatched this tick
                continue
            ip = abi.ip4(got[0]) if got else 0
            if ip:
                keep.append(int(h))
                ips.append(ip)
        if keep:
            self.eng.cni_assign(keep, ips)

    # ---- tick + apply (engine_cgo.go tick / applyPatches, gpu_controller.go step) -----
    def _tick(self, now, heartbeats=True):
        e = self.eng
        res = e.tick_raw(now)
        new_epoch = self.hb is None or res.heartbeat_epoch != self.hb_epoch
        if new_epoch:
            self.hb = np.empty(res.n_heartbeat, np.int32)
        L = {"ini": np.empty(res.n_node_init, np.int32), "ini_off": np.empty(res.n_node_init, np.uint64),
             "ini_len": np.empty(res.n_node_init, np.uint32),
             "pp": np.empty(res.n_pod_patch, np.int32), "pp_off": np.empty(res.n_pod_patch, np.uint64),
             "pp_len": np.empty(res.n_pod_patch, np.uint32),
             "dl": np.empty(res.n_delete, np.int32), "dlf": np.empty(res.n_delete, np.uint8)}
        p = lambda k: L[k].ctypes.data if L[k].size else None  # noqa: E731
        out = abi.Outputs(self.hb.ctypes.data if (new_epoch and self.hb.size) else None, 0,
                          p("ini"), p("ini_off"), p("ini_len"), p("pp"), p("pp_off"), p("pp_len"),
                          p("dl"), p("dlf"), None, 0, 0)
        e._check(e._fn("read_outputs")(e._h, C.byref(out)), "read_outputs")
        self.hb_epoch = res.heartbeat_epoch
        n = 0
        if res.n_heartbeat and heartbeats:
            body = e.read_arena(out.heartbeat_off, res.heartbeat_len).tobytes()
            for h in self.hb:
                self._apply(HEARTBEAT, int(h), body)
                n += 1
        n += self._apply_patches(NODE_INIT, L["ini"], L["ini_off"], L["ini_len"])
        n += self._apply_patches(POD_PATCH, L["pp"], L["pp_off"], L["pp_len"])
        gone = []
        for h, f in zip(L["dl"], L["dlf"]):  # Patch(removeFinalizers) if finalizers, then Delete(grace 0)
            # the engine freed the handle: the pod's noted echoes go BEFORE the apply, so
            # that the echo of its finalizer patch (noted by the apply) is dropped
            # (gpu_controller.go forgets in the tick callback, ahead of the task)
            self.echo.forget(self.pod_uid.get(int(h)))
            self._apply(DELETE_FIN if f else DELETE, int(h), None)
            gone.append(int(h))
            n += 1
        for h in gone:  # the later Deleted watch event finds no handle
            uid = self.pod_uid.pop(h, None)
            self.pod_by_uid.pop(uid, None)
            self.pod_ref.pop(h, None)
        self.stats.bodies += n
        return n

    def _apply_patches(self, kind, hs, offs, lens):
        i = n = 0
        ends = offs.astype(np.int64) + lens
        while i < len(hs):
            lo = int(offs[i])
            j = max(i + 1, int(np.searchsorted(ends, lo + READ_CHUNK, side="right")))
            buf = self.eng.read_arena(lo, int(ends[j - 1]) - lo).tobytes()
            for k in range(i, j):
                o = int(offs[k]) - lo
                self._apply(kind, int(hs[k]), buf[o:o + int(lens[k])])
                n += 1
            i = j
        return n

    def _apply(self, kind, h, body):
        cs = self.conf.client_set
        if kind in (HEARTBEAT, NODE_INIT):  # configureHeartbeatNode / configureNode bodies
            try:
                obj = cs.patch_node_status(self.node_name[h], body)
            except NotFound:
                return
            self.echo.note(_meta(obj).get("uid"), _meta(obj).get("resourceVersion"))
        elif kind == POD_PATCH:  # LockPod (pod_controller.go:205-231)
            ns, name = self.pod_ref[h]
            try:
                obj = cs.patch_pod_status(ns, name, body)
            except NotFound:
                return
            self.echo.note(_meta(obj).get("uid"), _meta(obj).get("resourceVersion"))
            if b'"podIP"' not in body:  # an empty status: its echo re-enters (step 6)
                self.reenter.append(obj)
        else:  # DeletePod (pod_controller.go:155-183)
            ns, name = self.pod_ref[h]
            if kind == DELETE_FIN:
                if self.finalizer is None:
                    from .engine import finalizer_patch
                    self.finalizer = finalizer_patch()
                try:
                    obj = cs.patch_pod(ns, name, self.finalizer)
                except NotFound:
                    return
                self.echo.note(_meta(obj).get("uid"), _meta(obj).get("resourceVersion"))
            try:
                cs.delete_pod(ns, name)
            except NotFound:
                pass


def new_controller(conf: Config, backend=None) -> Controller:
    """NewController (controller.go:80): the engine-backed controller"""
    return Controller(conf, backend)
