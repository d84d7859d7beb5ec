"""Python binding of the C-ABI engine (include/kwok_engine.h).

`Engine` drives libkwok_engine.so (HIP kernels on gfx950).  The class is
written against the ABI only, parameterised by the symbol prefix, so test
infrastructure can point the same driver at the CPU oracle
(oracle/oracle.py); the product never does.

Mirrors the reference's controller-facing calls (hezhizhen/kwok,
pkg/kwok/controllers): ingest_nodes ~ WatchNodes/ListNodes event handling
(node_controller.go:256-295), ingest_pods ~ WatchPods/ListPods
(pod_controller.go:301-367), tick ~ one heartbeat interval of KeepNodeHeartbeat
+ LockNodes + LockPods + DeletePods (node_controller.go:175-204,301-354;
pod_controller.go:155-250), has/size ~ NodeController.Has/Size (:403-409).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libkwok_engine.so")


class KwokError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__("%s (%d)%s" % (abi.ERRNAMES.get(code, "?"), code, (": " + msg) if msg else ""))
        self.code = code


_LIB = None


def load_engine_lib(path=None):
    """Load the in-tree HIP engine library.  Fails loudly when it is missing:
    there is no CPU fallback for the product path."""
    global _LIB
    if _LIB is None or path:
        p = path or os.environ.get("KWOK_ENGINE_LIB") or LIB_PATH  # KWOK_ENGINE_LIB: A/B builds (diagnostics)
        if not os.path.exists(p):
            raise ImportError("kwok_amd: %s is missing - run __graft_entry__.build() (make -C kwok_amd)" % p)
        lib = C.CDLL(p)
        declare(lib, "kwok_")
        if path:
            return lib
        _LIB = lib
    return _LIB


def declare(lib, pre):
    P, I32, U32, U64, SZ, VP = C.POINTER, C.c_int32, C.c_uint32, C.c_uint64, C.c_size_t, C.c_void_p
    sig = {
        "engine_create" if pre == "kwok_" else "create": (C.c_int, [P(abi.Config), P(VP)]),
        "engine_destroy" if pre == "kwok_" else "destroy": (None, [VP]),
        "last_error": (C.c_char_p, [VP]),
        "register_pod_spec": (C.c_int, [VP, P(abi.PodSpec), C.c_char_p, SZ, P(I32)]),
        "ingest_nodes": (C.c_int, [VP, VP, SZ, C.c_char_p, SZ, VP, VP]),
        "ingest_pods": (C.c_int, [VP, VP, SZ, C.c_char_p, SZ, VP, VP, VP]),
        "ingest_pods_packed": (C.c_int, [VP, VP, SZ, VP, VP, VP]),
        "ingest_pods_packed12": (C.c_int, [VP, VP, SZ, VP, SZ, VP, VP]),
        "ingest_pods_packed12_tick": (C.c_int, [VP, VP, SZ, VP, SZ, VP, VP, C.c_int64]),
        "pool_put": (C.c_int, [VP, VP, SZ]),
        "cni_pending": (C.c_int, [VP, VP, SZ, P(SZ)]),
        "cni_assign": (C.c_int, [VP, VP, VP, SZ, VP]),
        "tick": (C.c_int, [VP, C.c_int64, P(abi.TickResult)]),
        "read_outputs": (C.c_int, [VP, P(abi.Outputs)]),
        "read_arena": (C.c_int, [VP, U64, U64, VP]),
        "node_has": (C.c_int, [VP, C.c_char_p, SZ]),
        "node_size": (U64, [VP]),
        "dump_pods": (C.c_int, [VP, I32, U32, VP, VP, VP, VP]),
    }
    if pre == "kwok_":
        sig.update({
            "abi_version": (U32, []),
            "comm_id": (C.c_int, [VP]),
            "finalizer_patch": (C.c_char_p, [P(SZ)]),
            "device_outputs": (C.c_int, [VP, P(abi.DeviceView)]),
            "bucket_of": (U32, [C.c_char_p, SZ, U32]),
            "host_alloc": (VP, [SZ]),
            "pack_pod_events": (C.c_int, [VP, SZ, C.c_char_p, SZ, VP, VP]),
            "host_free": (None, [VP]),
            "rank_of_bucket": (I32, [U32, U32, I32]),
            "profile_enable": (C.c_int, [VP, C.c_int]),
            "profile_read": (C.c_int, [VP, VP, VP]),
            "profile_host": (C.c_int, [VP, C.c_int, VP, VP]),
            "tick_submit": (C.c_int, [VP, C.c_int64]),
            "tick_collect": (C.c_int, [VP, P(abi.TickResult)]),
            "codec_create": (C.c_int, [P(abi.CodecConfig), P(VP)]),
            "template_render": (C.c_int, [C.c_char_p, SZ, C.c_char_p, SZ, C.c_char_p, SZ, VP, SZ, P(SZ)]),
            "template_last_error": (C.c_char_p, []),
            "pod_template_patch": (C.c_int, [C.c_char_p, P(abi.PodSpec), C.c_char_p, SZ, C.c_int64, C.c_char_p,
                                             C.c_int64, U32, U32, I32, VP, SZ, P(SZ)]),
            "node_template_patch": (C.c_int, [C.c_char_p, C.c_char_p, P(abi.NodeEvent), C.c_char_p, SZ, C.c_int64,
                                              C.c_char_p, C.c_int64, VP, SZ, P(SZ)]),
            "heartbeat_template_patch": (C.c_int, [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64, VP, SZ, P(SZ)]),
            "codec_destroy": (None, [VP]),
            "codec_last_error": (C.c_char_p, []),
            "selector_matches": (C.c_int, [C.c_char_p, C.c_char_p, SZ, P(I32)]),
            "decode_node": (C.c_int, [VP, VP, SZ, SZ, SZ, P(abi.NodeEvent)]),
            "decode_pod": (C.c_int, [VP, VP, SZ, SZ, SZ, P(abi.PodDoc)]),
            "decode_nodes": (C.c_int, [VP, VP, SZ, VP, VP, SZ, C.c_int, VP, VP]),
            "decode_pods": (C.c_int, [VP, VP, SZ, VP, VP, SZ, C.c_int, VP, VP]),
            "engine_stats": (C.c_int, [VP, VP]),
            "spec_key": (U64, [P(abi.PodSpec), C.c_char_p, SZ]),
            "decode_pods_gpu": (C.c_int, [VP, VP, C.c_char_p, SZ, VP, VP, SZ, VP, VP, VP, VP, P(SZ)]),
            "ingest_pods_json": (C.c_int, [VP, VP, C.c_char_p, SZ, VP, VP, VP, VP, SZ, VP, VP, VP, P(SZ)]),
            "read_arena_async": (C.c_int, [VP, U64, U64, VP]),
            "ingest_nodes_json": (C.c_int, [VP, VP, C.c_char_p, SZ, VP, VP, VP, SZ, VP, VP, P(SZ)]),
            "decode_nodes_gpu": (C.c_int, [VP, VP, VP, SZ, VP, VP, SZ, VP, VP, P(SZ)]),
            "read_wait": (C.c_int, [VP]),
        })
    for name, (res, args) in sig.items():
        f = getattr(lib, pre + name, None)
        if f is None:  # an older build (KWOK_ENGINE_LIB A/B runs); tests/test_abi.py checks the real one
            continue
        f.restype = res
        f.argtypes = args


@dataclass
class TickOutput:
    counters: dict
    local_counters: dict
    heartbeat_nodes: np.ndarray
    heartbeat_len: int
    heartbeat_stride: int
    heartbeat_off: int
    node_inits: list = field(default_factory=list)   # [(handle, bytes)]
    pod_patches: list = field(default_factory=list)  # [(handle, bytes)]
    deletes: list = field(default_factory=list)      # [(handle, has_finalizers)]
    arena: bytes = b""

    def heartbeat_body(self, i=0):
        o = self.heartbeat_off + i * self.heartbeat_stride
        return self.arena[o:o + self.heartbeat_len]


def make_config(cidr="10.0.0.1/24", node_ip="196.168.0.1", start_time=1704067200, buckets=4096,
                node_slots_per_bucket=64, pod_slots_per_bucket=512, max_pod_specs=1024, rank=0, world_size=1,
                device=0, comm_id=None, allgather=None, enable_cni=False, pod_handle_stride=0,
                pod_status_template=None, node_init_template=None, node_heartbeat_template=None, heartbeat_once=False):
    cfg = abi.Config()
    cfg.abi_version = abi.ABI_VERSION
    cfg.cidr = cidr.encode()
    cfg.node_ip = node_ip.encode()
    cfg.start_time_unix = start_time
    cfg.buckets = buckets
    cfg.node_slots_per_bucket = node_slots_per_bucket
    cfg.pod_slots_per_bucket = pod_slots_per_bucket
    cfg.max_pod_specs = max_pod_specs
    cfg.rank, cfg.world_size, cfg.device = rank, world_size, device
    cfg.enable_cni = 1 if enable_cni else 0
    cfg.pod_handle_stride = pod_handle_stride
    cfg.flags = abi.CFG_HEARTBEAT_ONCE if heartbeat_once else 0
    keep = []
    if pod_status_template is not None:
        b = C.create_string_buffer(pod_status_template.encode())
        keep.append(b)
        cfg.custom_templates |= 1
        cfg.pod_status_template = C.cast(b, C.c_char_p)
    if node_init_template is not None:
        b = C.create_string_buffer(node_init_template.encode())
        keep.append(b)
        cfg.custom_templates |= 2
        cfg.node_init_template = C.cast(b, C.c_char_p)
    if node_heartbeat_template is not None:
        b = C.create_string_buffer(node_heartbeat_template.encode())
        keep.append(b)
        cfg.custom_templates |= 4
        cfg.node_heartbeat_template = C.cast(b, C.c_char_p)
    if comm_id is not None:
        b = C.create_string_buffer(bytes(comm_id), abi.COMM_ID_BYTES)
        keep.append(b)
        cfg.comm_id = C.cast(b, C.c_void_p)
    if allgather is not None:
        cb = abi.ALLGATHER_FN(allgather)
        keep.append(cb)
        cfg.allgather = cb
    cfg._keep = keep  # keep buffers / callbacks alive with the struct
    return cfg


class EngineBase:
    """Driver over one ABI implementation (lib + symbol prefix)."""

    PREFIX = "kwok_"

    def __init__(self, lib, cfg: abi.Config):
        self._lib = lib
        self._cfg = cfg
        self._fn = lambda n: getattr(lib, self.PREFIX + n)
        h = C.c_void_p()
        create = self._fn("engine_create" if self.PREFIX == "kwok_" else "create")
        rc = create(C.byref(cfg), C.byref(h))
        if rc != 0:
            msg = self._fn("last_error")(None)
            raise KwokError(rc, "create: %s" % (msg or b"").decode())
        self._h = h
        self.last = None
        self.node_ip = abi.ip4(cfg.node_ip.decode())  # Config.NodeIP (kwok_pod_rec12's hostIP flag)

    def close(self):
        if getattr(self, "_h", None):
            self._fn("engine_destroy" if self.PREFIX == "kwok_" else "destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc < 0:
            err = self._fn("last_error")(self._h)
            raise KwokError(rc, "%s: %s" % (what, (err or b"").decode()))
        return rc

    # -- specs ----------------------------------------------------------------
    def register_pod_spec(self, containers=(), init_containers=(), readiness_gates=()):
        ar = abi.Arena()
        cs = (abi.Container * max(1, len(containers)))(
            *[abi.Container(ar.kstr(n), ar.kstr(i)) for n, i in containers])
        ics = (abi.Container * max(1, len(init_containers)))(
            *[abi.Container(ar.kstr(n), ar.kstr(i)) for n, i in init_containers])
        gs = (abi.KwokStr * max(1, len(readiness_gates)))(*[ar.kstr(g) for g in readiness_gates])
        spec = abi.PodSpec(cs, len(containers), ics, len(init_containers), gs, len(readiness_gates))
        buf, n = ar.cbuf()
        out = C.c_int32()
        self._check(self._fn("register_pod_spec")(self._h, C.byref(spec), buf, n, C.byref(out)), "register_pod_spec")
        return out.value

    # -- ingest ---------------------------------------------------------------
    def ingest_nodes_raw(self, events: np.ndarray, arena, out=None):
        """arena: bytes or a uint8 array; out: optional (handles, status)
        arrays of len(events) (e.g. page-locked, host_array)"""
        n = len(events)
        if out is None:
            hs, st = np.empty(n, np.int32), np.empty(n, np.int32)
        else:
            hs, st = (o[:n] for o in out)
        ev = np.ascontiguousarray(events, dtype=abi.NODE_EVENT_DTYPE)
        if isinstance(arena, np.ndarray):
            ar, alen = C.cast(arena.ctypes.data, C.c_char_p), arena.nbytes
        else:
            ar, alen = arena or b"\0", len(arena)
        rc = self._fn("ingest_nodes")(self._h, ev.ctypes.data, n, ar, alen, hs.ctypes.data, st.ctypes.data)
        self._check(rc, "ingest_nodes")
        return hs, st

    def ingest_pods_raw(self, events: np.ndarray, arena, out=None):
        """arena: bytes or a uint8 array; out: optional (handles, status,
        released) arrays of len(events) (e.g. page-locked, host_array)"""
        n = len(events)
        if out is None:
            hs, st, rel = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.uint32)
        else:
            hs, st, rel = (o[:n] for o in out)
        ev = np.ascontiguousarray(events, dtype=abi.POD_EVENT_DTYPE)
        if isinstance(arena, np.ndarray):
            ar, alen = C.cast(arena.ctypes.data, C.c_char_p), arena.nbytes
        else:
            ar, alen = arena or b"\0", len(arena)
        rc = self._fn("ingest_pods")(self._h, ev.ctypes.data, n, ar, alen, hs.ctypes.data, st.ctypes.data,
                                     rel.ctypes.data)
        self._check(rc, "ingest_pods")
        return hs, st, rel

    def ingest_pods_packed(self, recs: np.ndarray, out=None, released=True):
        """kwok_ingest_pods_packed over POD_REC_DTYPE rows; out: optional
        (handles, status int8, released) arrays (e.g. page-locked, host_array)"""
        n = len(recs)
        if out is None:
            hs, st = np.empty(n, np.int32), np.empty(n, np.int8)
            rel = np.empty(n, np.uint32) if released else None
        else:
            hs, st, rel = (o[:n] if o is not None else None for o in out)
        r = recs if recs.flags.c_contiguous and recs.dtype == abi.POD_REC_DTYPE else \
            np.ascontiguousarray(recs, dtype=abi.POD_REC_DTYPE)
        rc = self._fn("ingest_pods_packed")(self._h, r.ctypes.data, n, hs.ctypes.data, st.ctypes.data,
                                            rel.ctypes.data if rel is not None else None)
        self._check(rc, "ingest_pods_packed")
        return hs, st, rel

    def ingest_pods_packed12(self, recs: np.ndarray, new_cap=None, out=None, released=True, tick_now=None):
        """kwok_ingest_pods_packed12 over POD_REC12_DTYPE rows -> (handles of the
        creates in create order, status int8 per record, released).  new_cap: the
        room for create handles (default: the number of REC_NEW rows); out:
        optional (new handles, status, released) arrays (e.g. page-locked).
        tick_now: kwok_ingest_pods_packed12_tick - the tick at tick_now queued
        behind the batch's apply passes (collect it with tick_collect)"""
        n = len(recs)
        r = recs if recs.flags.c_contiguous and recs.dtype == abi.POD_REC12_DTYPE else \
            np.ascontiguousarray(recs, dtype=abi.POD_REC12_DTYPE)
        if new_cap is None:
            new_cap = int(np.count_nonzero(r["op"] & abi.REC_NEW))
        if out is None:
            nh, st = np.empty(max(new_cap, 1), np.int32), np.empty(n, np.int8)
            rel = np.empty(n, np.uint32) if released else None
        else:
            nh, st, rel = out[0], out[1][:n], (out[2][:n] if out[2] is not None else None)
            assert len(nh) >= new_cap
        if tick_now is None:
            rc = self._fn("ingest_pods_packed12")(self._h, r.ctypes.data, n, nh.ctypes.data, new_cap, st.ctypes.data,
                                                  rel.ctypes.data if rel is not None else None)
        else:
            rc = self._fn("ingest_pods_packed12_tick")(self._h, r.ctypes.data, n, nh.ctypes.data, new_cap,
                                                       st.ctypes.data, rel.ctypes.data if rel is not None else None,
                                                       int(tick_now))
        self._check(rc, "ingest_pods_packed12")
        return nh[:new_cap], st, rel

    def pool_put(self, ips):
        a = np.ascontiguousarray(ips, dtype=np.uint32)
        self._check(self._fn("pool_put")(self._h, a.ctypes.data, len(a)), "pool_put")

    # -- EnableCNI (configurePod's cni.Setup, pod_controller.go:383-389) --------
    def cni_pending(self):
        """handles (canonical order) of the pods the next tick evaluates without a podIP"""
        n = C.c_size_t()
        rc = self._fn("cni_pending")(self._h, None, 0, C.byref(n))
        if rc != 0 and n.value == 0:
            self._check(rc, "cni_pending")
        out = np.empty(max(1, n.value), np.int32)
        self._check(self._fn("cni_pending")(self._h, out.ctypes.data, out.size, C.byref(n)), "cni_pending")
        return out[:n.value]

    def cni_assign(self, handles, ips):
        h = np.ascontiguousarray(handles, dtype=np.int32)
        a = np.ascontiguousarray(ips, dtype=np.uint32)
        st = np.empty(len(h), np.int32)
        self._check(self._fn("cni_assign")(self._h, h.ctypes.data, a.ctypes.data, len(h), st.ctypes.data), "cni_assign")
        return st

    # -- tick -------------------------------------------------------------------
    def tick_raw(self, now_unix):
        res = abi.TickResult()
        self._check(self._fn("tick")(self._h, now_unix, C.byref(res)), "tick")
        self.last = res
        return res

    def tick(self, now_unix, read=True):
        res = self.tick_raw(now_unix)
        if not read:
            return res
        return self.read_outputs(res)

    def read_outputs(self, res=None, heartbeat_once=False):
        """The tick's outputs on the host.  heartbeat_once: the arena holds ONE
        heartbeat body (kwok_outputs KWOK_READ_HEARTBEAT_ONCE) - what a caller
        that sends the same body to every node needs."""
        res = res or self.last
        hb = np.empty(res.n_heartbeat, np.int32)
        ini = np.empty(res.n_node_init, np.int32)
        ini_off = np.empty(res.n_node_init, np.uint64)
        ini_len = np.empty(res.n_node_init, np.uint32)
        pp = np.empty(res.n_pod_patch, np.int32)
        pp_off = np.empty(res.n_pod_patch, np.uint64)
        pp_len = np.empty(res.n_pod_patch, np.uint32)
        dl = np.empty(res.n_delete, np.int32)
        dlf = np.empty(res.n_delete, np.uint8)
        arena = np.empty(max(1, res.arena_bytes), np.uint8)
        out = abi.Outputs(hb.ctypes.data, 0, ini.ctypes.data, ini_off.ctypes.data, ini_len.ctypes.data,
                          pp.ctypes.data, pp_off.ctypes.data, pp_len.ctypes.data, dl.ctypes.data, dlf.ctypes.data,
                          arena.ctypes.data, arena.nbytes, abi.READ_HEARTBEAT_ONCE if heartbeat_once else 0)
        self._check(self._fn("read_outputs")(self._h, C.byref(out)), "read_outputs")
        ab = arena[:out.arena_copied].tobytes()
        sh = out.arena_shift
        return TickOutput(
            counters=dict(zip(abi.COUNTERS, list(res.counters))),
            local_counters=dict(zip(abi.COUNTERS, list(res.local_counters))),
            heartbeat_nodes=hb, heartbeat_len=res.heartbeat_len,
            heartbeat_stride=0 if heartbeat_once else res.heartbeat_stride,
            heartbeat_off=out.heartbeat_off,
            node_inits=[(int(h), ab[o - sh:o - sh + n]) for h, o, n in zip(ini, ini_off, ini_len)],
            pod_patches=[(int(h), ab[o - sh:o - sh + n]) for h, o, n in zip(pp, pp_off, pp_len)],
            deletes=[(int(h), int(f)) for h, f in zip(dl, dlf)],
            arena=ab)

    def read_arrays(self, res=None, heartbeat_once=False):
        """The tick's outputs as numpy arrays (no per-patch Python objects): for
        fleets of millions of objects.  Offsets index `arena` directly."""
        res = res or self.last
        a = {"heartbeat_nodes": np.empty(res.n_heartbeat, np.int32),
             "node_init_nodes": np.empty(res.n_node_init, np.int32),
             "node_init_off": np.empty(res.n_node_init, np.uint64),
             "node_init_len": np.empty(res.n_node_init, np.uint32),
             "pod_patch_pods": np.empty(res.n_pod_patch, np.int32),
             "pod_patch_off": np.empty(res.n_pod_patch, np.uint64),
             "pod_patch_len": np.empty(res.n_pod_patch, np.uint32),
             "delete_pods": np.empty(res.n_delete, np.int32),
             "delete_has_finalizers": np.empty(res.n_delete, np.uint8)}
        arena = np.empty(max(1, res.arena_bytes), np.uint8)
        out = abi.Outputs(*[a[k].ctypes.data if k != "heartbeat_off" else 0 for k in
                            ("heartbeat_nodes", "heartbeat_off", "node_init_nodes", "node_init_off", "node_init_len",
                             "pod_patch_pods", "pod_patch_off", "pod_patch_len", "delete_pods",
                             "delete_has_finalizers")],
                          arena.ctypes.data, arena.nbytes, abi.READ_HEARTBEAT_ONCE if heartbeat_once else 0)
        self._check(self._fn("read_outputs")(self._h, C.byref(out)), "read_outputs")
        a["arena"] = arena[:out.arena_copied]
        a["node_init_off"] -= np.uint64(out.arena_shift)
        a["pod_patch_off"] -= np.uint64(out.arena_shift)
        a["heartbeat_off"] = out.heartbeat_off
        a["heartbeat_len"] = res.heartbeat_len
        a["heartbeat_stride"] = 0 if heartbeat_once else res.heartbeat_stride
        a["counters"] = dict(zip(abi.COUNTERS, list(res.counters)))
        return a

    def read_arena(self, off, n, out=None):
        """kwok_read_arena: bytes [off, off + n) of the collected tick's arena
        (the offsets read_outputs reports without heartbeat_once)"""
        buf = out if out is not None else np.empty(max(1, n), np.uint8)
        self._check(self._fn("read_arena")(self._h, off, n, buf.ctypes.data), "read_arena")
        return buf[:n]

    # -- queries ----------------------------------------------------------------
    def node_has(self, name: str) -> bool:
        b = name.encode()
        return bool(self._fn("node_has")(self._h, b, len(b)))

    def node_size(self) -> int:
        return int(self._fn("node_size")(self._h))

    def dump_pods(self, first, count):
        used = np.zeros(count, np.uint8)
        phase = np.zeros(count, np.uint8)
        hip = np.zeros(count, np.uint32)
        pip = np.zeros(count, np.uint32)
        self._check(self._fn("dump_pods")(self._h, first, count, used.ctypes.data, phase.ctypes.data,
                                          hip.ctypes.data, pip.ctypes.data), "dump_pods")
        return used, phase, hip, pip


class Engine(EngineBase):
    """The MI355X engine (libkwok_engine.so)."""

    PREFIX = "kwok_"

    def __init__(self, cfg=None, **kw):
        super().__init__(load_engine_lib(), cfg if cfg is not None else make_config(**kw))

    # kwok_tick in two halves: tick N+1 runs on the device while tick N is collected
    def tick_submit(self, now_unix):
        self._check(self._lib.kwok_tick_submit(self._h, now_unix), "tick_submit")

    def tick_collect(self, read=True):
        res = abi.TickResult()
        self._check(self._lib.kwok_tick_collect(self._h, C.byref(res)), "tick_collect")
        self.last = res
        return self.read_outputs(res) if read else res

    PHASES = ("classify", "stream", "header", "exchange", "pool", "emit", "kernel", "emit_kernel")  # KWOK_T_* order
    HOST = ("enqueue", "wait", "post", "total")  # KWOK_H_* order

    def profile_enable(self, on=True):
        self._check(self._lib.kwok_profile_enable(self._h, 1 if on else 0), "profile_enable")

    def profile_read(self):
        ms = (C.c_double * len(self.PHASES))()
        n = C.c_uint64()
        self._check(self._lib.kwok_profile_read(self._h, ms, C.byref(n)), "profile_read")
        return dict(zip(self.PHASES, list(ms))), n.value

    def profile_host(self, reset=False):
        ms = (C.c_double * len(self.HOST))()
        n = C.c_uint64()
        self._check(self._lib.kwok_profile_host(self._h, 1 if reset else 0, ms, C.byref(n)), "profile_host")
        return dict(zip(self.HOST, list(ms))), n.value

    # ---- the pod codec on the GPU (kwok_decode_pods_gpu / kwok_ingest_pods_json) ----
    @staticmethod
    def _docs(docs):
        """concatenated documents (bytes or JSON-able values) -> (arena, offsets, lengths)"""
        import json as _json
        raws = [d if isinstance(d, (bytes, bytearray)) else _json.dumps(d).encode() for d in docs]
        lens = np.fromiter((len(r) for r in raws), np.uint32, len(raws))
        offs = np.zeros(len(raws), np.uint64)
        if len(raws):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        return b"".join(raws), offs, lens

    def decode_pods_gpu(self, codec, docs=None, arena=None, offs=None, lens=None):
        """kwok_decode_pods_gpu: per document its kwok_pod_event (POD_EVENT_DTYPE),
        (name, namespace) spans, spec key and status, and the number the host decided.
        Documents as a list, or as (arena, offs, lens)."""
        if docs is not None:
            arena, offs, lens = self._docs(docs)
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        n = len(offs)
        ev = np.zeros(n, abi.POD_EVENT_DTYPE)
        names = np.zeros((n, 2, 2), np.uint32)
        keys = np.zeros(n, np.uint64)
        st = np.zeros(n, np.int32)
        nh = C.c_size_t()
        ar, alen = self._arena_arg(arena)
        rc = self._lib.kwok_decode_pods_gpu(self._h, codec._h, ar, alen, offs.ctypes.data, lens.ctypes.data, n,
                                            ev.ctypes.data, names.ctypes.data, keys.ctypes.data, st.ctypes.data,
                                            C.byref(nh))
        self._check(rc, "decode_pods_gpu")
        return ev, names, keys, st, nh.value

    def ingest_nodes_json(self, codec, arena, offs, lens, ops, out=None):
        """kwok_ingest_nodes_json: (handles, statuses, documents the host decided)"""
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        ops = np.ascontiguousarray(ops, np.uint8)
        n = len(offs)
        if out is None:
            hs, st = np.empty(n, np.int32), np.empty(n, np.int32)
        else:
            hs, st = (o[:n] for o in out)
        nh = C.c_size_t()
        ar, alen = self._arena_arg(arena)
        rc = self._lib.kwok_ingest_nodes_json(self._h, codec._h, ar, alen, offs.ctypes.data, lens.ctypes.data,
                                              ops.ctypes.data, n, hs.ctypes.data, st.ctypes.data, C.byref(nh))
        self._check(rc, "ingest_nodes_json")
        return hs, st, nh.value

    def decode_nodes_gpu(self, codec, docs=None, arena=None, offs=None, lens=None):
        """kwok_decode_nodes_gpu: per document its kwok_node_event (NODE_EVENT_DTYPE) and
        status, the number the host decided, and the arena (the host codec rewrites the
        listed documents' blobs in place).  Documents as a list, or as (arena, offs, lens)."""
        if docs is not None:
            arena, offs, lens = self._docs(docs)
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        n = len(offs)
        buf = np.frombuffer(bytearray(bytes(arena) + b"\0"), np.uint8)
        ev = np.zeros(n, abi.NODE_EVENT_DTYPE)
        st = np.zeros(n, np.int32)
        nh = C.c_size_t()
        rc = self._lib.kwok_decode_nodes_gpu(self._h, codec._h, buf.ctypes.data, len(arena), offs.ctypes.data,
                                             lens.ctypes.data, n, ev.ctypes.data, st.ctypes.data, C.byref(nh))
        self._check(rc, "decode_nodes_gpu")
        return ev, st, nh.value, bytes(buf[:len(arena)])

    def ingest_pods_json(self, codec, arena, offs, lens, ops, handles, out=None):
        """kwok_ingest_pods_json: (handles, statuses, released, documents the host decided)"""
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        ops = np.ascontiguousarray(ops, np.uint8)
        handles = np.ascontiguousarray(handles, np.int32)
        n = len(offs)
        if out is None:
            hs, st, rel = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.uint32)
        else:
            hs, st, rel = (o[:n] for o in out)
        nh = C.c_size_t()
        ar, alen = self._arena_arg(arena)
        rc = self._lib.kwok_ingest_pods_json(self._h, codec._h, ar, alen, offs.ctypes.data, lens.ctypes.data,
                                             ops.ctypes.data, handles.ctypes.data, n, hs.ctypes.data, st.ctypes.data,
                                             rel.ctypes.data, C.byref(nh))
        self._check(rc, "ingest_pods_json")
        return hs, st, rel, nh.value

    @staticmethod
    def _arena_arg(arena):
        if isinstance(arena, np.ndarray):
            return C.cast(arena.ctypes.data, C.c_char_p), arena.nbytes
        return (arena or b"\0"), len(arena or b"")

    def read_arena_async(self, off, n, out):
        """kwok_read_arena_async: bytes [off, off + n) of the collected tick's arena
        queued into `out` (page-locked: host_array); read_wait() waits for them"""
        self._check(self._lib.kwok_read_arena_async(self._h, off, n, out.ctypes.data), "read_arena_async")

    def read_wait(self):
        self._check(self._lib.kwok_read_wait(self._h), "read_wait")

    STATS = ("ticks_full", "ticks_once", "once_redo", "once_summary")  # KWOK_STAT_* order

    def stats(self):
        """kwok_engine_stats: ticks run by k_tick / completed by k_once / k_once ticks redone / k_once
        launches that read the per-bucket summaries"""
        out = (C.c_uint64 * len(self.STATS))()
        self._check(self._lib.kwok_engine_stats(self._h, out), "engine_stats")
        return dict(zip(self.STATS, list(out)))

    def device_outputs(self):
        v = abi.DeviceView()
        self._check(self._lib.kwok_device_outputs(self._h, C.byref(v)), "device_outputs")
        return v


def host_array(shape, dtype):
    """A numpy array over page-locked host memory (kwok_host_alloc), freed
    with the array: batch buffers that move to and from the GPU by DMA."""
    import weakref
    lib = load_engine_lib()
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    p = lib.kwok_host_alloc(max(n, 1))
    if not p:
        raise MemoryError("kwok_host_alloc(%d)" % n)
    buf = (C.c_uint8 * max(n, 1)).from_address(p)
    weakref.finalize(buf, lib.kwok_host_free, p)
    return np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)


def comm_id() -> bytes:
    lib = load_engine_lib()
    b = C.create_string_buffer(abi.COMM_ID_BYTES)
    rc = lib.kwok_comm_id(b)
    if rc != 0:
        raise KwokError(rc, "comm_id")
    return b.raw


def spec_key(containers, init_containers=(), gates=()) -> int:
    """kwok_spec_key: the key the GPU codec finds a registered pod spec by"""
    lib = load_engine_lib()
    ar = abi.Arena()
    cs = (abi.Container * max(1, len(containers)))(*[abi.Container(ar.ref(n), ar.ref(i)) for n, i in containers])
    ics = (abi.Container * max(1, len(init_containers)))(*[abi.Container(ar.ref(n), ar.ref(i))
                                                            for n, i in init_containers])
    gs = (abi.KwokStr * max(1, len(gates)))(*[ar.ref(g) for g in gates])
    sp = abi.PodSpec(cs, len(containers), ics, len(init_containers), gs, len(gates))
    buf = bytes(ar.buf) or b"\0"
    return int(lib.kwok_spec_key(C.byref(sp), buf, len(ar.buf)))


def finalizer_patch() -> bytes:
    lib = load_engine_lib()
    n = C.c_size_t()
    p = lib.kwok_finalizer_patch(C.byref(n))
    return p[: n.value]


def template_render(tpl: str, doc, funcs=None) -> str:
    """kwok_template_render: renderToJSON of `tpl` over the document (a JSON
    string or a JSON-able value) with zero-argument template funcs
    {"Now": "...", ...}.  Host only."""
    import json as _json
    lib = load_engine_lib()
    t = tpl.encode()
    d = (doc if isinstance(doc, str) else _json.dumps(doc)).encode()
    f = _json.dumps(funcs or {}).encode()
    n = C.c_size_t()
    cap = 1 << 16
    while True:
        out = C.create_string_buffer(cap)
        rc = lib.kwok_template_render(t, len(t), d, len(d), f, len(f), out, cap, C.byref(n))
        if rc == abi.EINVAL and n.value > cap:
            cap = n.value + 1
            continue
        if rc != 0:
            raise KwokError(rc, (lib.kwok_template_last_error() or b"").decode())
        return out.raw[:n.value].decode()


def pod_template_patch(tpl: str, containers=(), init_containers=(), readiness_gates=(), start=1704067200,
                       node_ip="196.168.0.1", creation=1704067140, host_ip=0, pod_ip=0, status_nonempty=True) -> bytes:
    """kwok_pod_template_patch: the patch the engine emits for a pod with this
    spec under the custom pod status template (compiled + assembled on the host)."""
    lib = load_engine_lib()
    ar = abi.Arena()
    cs = (abi.Container * max(1, len(containers)))(*[abi.Container(ar.kstr(n), ar.kstr(i)) for n, i in containers])
    ics = (abi.Container * max(1, len(init_containers)))(
        *[abi.Container(ar.kstr(n), ar.kstr(i)) for n, i in init_containers])
    gs = (abi.KwokStr * max(1, len(readiness_gates)))(*[ar.kstr(g) for g in readiness_gates])
    spec = abi.PodSpec(cs, len(containers), ics, len(init_containers), gs, len(readiness_gates))
    buf, n = ar.cbuf()
    out = C.create_string_buffer(1 << 16)
    m = C.c_size_t()
    rc = lib.kwok_pod_template_patch(tpl.encode(), C.byref(spec), buf, n, start, node_ip.encode(), creation, host_ip,
                                     pod_ip, 1 if status_nonempty else 0, out, 1 << 16, C.byref(m))
    if rc != 0:
        raise KwokError(rc, (lib.kwok_template_last_error() or b"").decode())
    return out.raw[:m.value]


def node_template_patch(tpl: str, event, arena: bytes, start=1704067200, node_ip="196.168.0.1",
                        now=1704067230, heartbeat_tpl=None) -> bytes:
    """kwok_node_template_patch: the init patch of the node record `event` (a
    NODE_EVENT_DTYPE row) under a custom node initialization template."""
    lib = load_engine_lib()
    ev = np.ascontiguousarray(np.asarray([event], dtype=abi.NODE_EVENT_DTYPE))
    out = C.create_string_buffer(1 << 16)
    m = C.c_size_t()
    rc = lib.kwok_node_template_patch(tpl.encode(), heartbeat_tpl.encode() if heartbeat_tpl else None,
                                      C.cast(ev.ctypes.data, C.POINTER(abi.NodeEvent)), arena or b"\0",
                                      len(arena), start, node_ip.encode(), now, out, 1 << 16, C.byref(m))
    if rc != 0:
        raise KwokError(rc, (lib.kwok_template_last_error() or b"").decode())
    return out.raw[:m.value]


def heartbeat_template_patch(tpl=None, start=1704067200, node_ip="196.168.0.1", now=1704067230) -> bytes:
    """kwok_heartbeat_template_patch: the heartbeat body under a custom heartbeat
    template (None: the default)."""
    lib = load_engine_lib()
    out = C.create_string_buffer(1 << 16)
    m = C.c_size_t()
    rc = lib.kwok_heartbeat_template_patch(tpl.encode() if tpl else None, start, node_ip.encode(), now, out, 1 << 16,
                                           C.byref(m))
    if rc != 0:
        raise KwokError(rc, (lib.kwok_template_last_error() or b"").decode())
    return out.raw[:m.value]


def pack_pod_events(events: np.ndarray, arena) -> tuple[np.ndarray, np.ndarray]:
    """kwok_pack_pod_events: kwok_pod_event rows + their string arena -> the
    compact records and a status per row (host only)"""
    lib = load_engine_lib()
    ev = np.ascontiguousarray(events, dtype=abi.POD_EVENT_DTYPE)
    out = np.zeros(len(ev), abi.POD_REC_DTYPE)
    st = np.empty(len(ev), np.int32)
    a = bytes(arena) if arena is not None else b""
    rc = lib.kwok_pack_pod_events(ev.ctypes.data, len(ev), a or b"\0", len(a), out.ctypes.data, st.ctypes.data)
    if rc < 0:
        raise KwokError(rc, "pack_pod_events")
    return out, st
