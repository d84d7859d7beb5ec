"""ctypes / numpy mirrors of include/kwok_engine.h (the C-ABI boundary).

Everything here is layout only; the structs must stay byte-identical to the
header (tests/test_abi.py checks sizes and offsets against the compiled
library's expectations)."""
from __future__ import annotations

import ctypes as C

import numpy as np

ABI_VERSION = 5
COMM_ID_BYTES = 128

OK, EINVAL, ENOMEM, EDOMAIN, EFULL, EDEVICE, ECOMM, ENOTFOUND, ENOTMINE, EBUSY = 0, -1, -2, -3, -4, -5, -6, -7, -8, -9
ERRNAMES = {0: "OK", -1: "EINVAL", -2: "ENOMEM", -3: "EDOMAIN", -4: "EFULL", -5: "EDEVICE",
            -6: "ECOMM", -7: "ENOTFOUND", -8: "ENOTMINE", -9: "EBUSY"}

OP_UPSERT, OP_DELETE = 1, 2
PHASE_NONE, PHASE_PENDING, PHASE_RUNNING, PHASE_SUCCEEDED, PHASE_FAILED, PHASE_UNKNOWN, PHASE_OTHER = range(7)
POD_PHASES = {"": PHASE_NONE, "Pending": PHASE_PENDING, "Running": PHASE_RUNNING, "Succeeded": PHASE_SUCCEEDED,
              "Failed": PHASE_FAILED, "Unknown": PHASE_UNKNOWN}
PHASE_NAMES = {v: k for k, v in POD_PHASES.items()}

POD_DISREGARD, POD_DELETING, POD_STATUS_NONEMPTY, POD_CONFORMS, POD_HAS_FINALIZERS = 1, 2, 4, 8, 16

NODEINFO_KEYS = ["architecture", "bootID", "containerRuntimeVersion", "kernelVersion", "kubeProxyVersion",
                 "kubeletVersion", "machineID", "operatingSystem", "osImage", "systemUUID"]
NI_COUNT = len(NODEINFO_KEYS)

COUNTERS = ["heartbeat", "node_init", "pod_patch", "delete", "alloc", "release", "evaluated", "lock_checked",
            "nodes_managed", "nodes_ready", "pods_total", "pods_pending", "pods_running"]
COUNTER_COUNT = len(COUNTERS)


class KwokStr(C.Structure):
    _fields_ = [("off", C.c_uint32), ("len", C.c_uint32)]


class NodeEvent(C.Structure):
    _fields_ = [("op", C.c_uint8), ("managed", C.c_uint8), ("lockable", C.c_uint8), ("phase", C.c_uint8),
                ("name", KwokStr), ("addresses", KwokStr), ("allocatable", KwokStr), ("capacity", KwokStr),
                ("node_info", KwokStr * NI_COUNT)]


class PodEvent(C.Structure):
    _fields_ = [("op", C.c_uint8), ("phase", C.c_uint8), ("flags", C.c_uint8), ("reserved0", C.c_uint8),
                ("handle", C.c_int32), ("spec_id", C.c_int32), ("node_handle", C.c_int32),
                ("creation_unix", C.c_int64), ("node_name", KwokStr), ("host_ip", KwokStr), ("pod_ip", KwokStr)]


class PodRec(C.Structure):
    """kwok_pod_rec: the compact wire form of a pod event (kwok_ingest_pods_packed)"""
    _fields_ = [("op", C.c_uint8), ("flags", C.c_uint8), ("spec_id", C.c_uint16), ("target", C.c_int32),
                ("creation", C.c_uint32), ("host_ip", C.c_uint32), ("pod_ip", C.c_uint32)]


class PodRec12(C.Structure):
    """kwok_pod_rec12 (kwok_ingest_pods_packed12): REC_HOST_NODE_IP in op stands for
    hostIP = the engine's node_ip; value = a create's creationTimestamp, any other
    record's podIP"""
    _fields_ = [("op", C.c_uint8), ("flags", C.c_uint8), ("spec_id", C.c_uint16), ("target", C.c_int32),
                ("value", C.c_uint32)]


REC_NEW = 0x80
REC_HOST_NODE_IP = 0x40
REC_PHASE_SHIFT = 5


class Container(C.Structure):
    _fields_ = [("name", KwokStr), ("image", KwokStr)]


class PodSpec(C.Structure):
    _fields_ = [("containers", C.POINTER(Container)), ("n_containers", C.c_uint32),
                ("init_containers", C.POINTER(Container)), ("n_init_containers", C.c_uint32),
                ("readiness_gates", C.POINTER(KwokStr)), ("n_readiness_gates", C.c_uint32)]


DOC_MAX_CONTAINERS, DOC_MAX_GATES = 32, 16


class CodecConfig(C.Structure):
    _fields_ = [("manage_all_nodes", C.c_int32), ("manage_nodes_with_annotation_selector", C.c_char_p),
                ("manage_nodes_with_label_selector", C.c_char_p),
                ("disregard_status_with_annotation_selector", C.c_char_p),
                ("disregard_status_with_label_selector", C.c_char_p)]


class PodDoc(C.Structure):
    _fields_ = [("ev", PodEvent), ("name", KwokStr), ("namespace_", KwokStr), ("n_containers", C.c_uint32),
                ("n_init_containers", C.c_uint32), ("n_readiness_gates", C.c_uint32), ("reserved0", C.c_uint32),
                ("containers", Container * DOC_MAX_CONTAINERS), ("init_containers", Container * DOC_MAX_CONTAINERS),
                ("readiness_gates", KwokStr * DOC_MAX_GATES)]


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


class Config(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("cidr", C.c_char_p), ("node_ip", C.c_char_p),
                ("start_time_unix", C.c_int64), ("enable_cni", C.c_int32), ("custom_templates", C.c_int32),
                ("buckets", C.c_uint32), ("node_slots_per_bucket", C.c_uint32),
                ("pod_slots_per_bucket", C.c_uint32), ("max_pod_specs", C.c_uint32),
                ("rank", C.c_int32), ("world_size", C.c_int32), ("device", C.c_int32),
                ("comm_id", C.c_void_p), ("allgather", ALLGATHER_FN), ("allgather_user", C.c_void_p),
                ("pod_handle_stride", C.c_uint32), ("flags", C.c_uint32),
                ("pod_status_template", C.c_char_p), ("node_init_template", C.c_char_p),
                ("node_heartbeat_template", C.c_char_p)]


class TickResult(C.Structure):
    _fields_ = [("n_heartbeat", C.c_uint32), ("heartbeat_len", C.c_uint32), ("heartbeat_stride", C.c_uint64),
                ("n_node_init", C.c_uint32), ("n_pod_patch", C.c_uint32), ("n_delete", C.c_uint32),
                ("heartbeat_epoch", C.c_uint32), ("arena_bytes", C.c_uint64),
                ("counters", C.c_uint64 * COUNTER_COUNT), ("local_counters", C.c_uint64 * COUNTER_COUNT)]


class Outputs(C.Structure):
    _fields_ = [("heartbeat_nodes", C.c_void_p), ("heartbeat_off", C.c_uint64),
                ("node_init_nodes", C.c_void_p), ("node_init_off", C.c_void_p), ("node_init_len", C.c_void_p),
                ("pod_patch_pods", C.c_void_p), ("pod_patch_off", C.c_void_p), ("pod_patch_len", C.c_void_p),
                ("delete_pods", C.c_void_p), ("delete_has_finalizers", C.c_void_p),
                ("arena", C.c_void_p), ("arena_cap", C.c_uint64), ("flags", C.c_uint32), ("reserved0", C.c_uint32),
                ("arena_shift", C.c_uint64), ("arena_copied", C.c_uint64)]

READ_HEARTBEAT_ONCE = 1
CFG_HEARTBEAT_ONCE = 1


class DeviceView(C.Structure):
    _fields_ = [("arena", C.c_void_p), ("heartbeat_nodes", C.c_void_p), ("pod_patch_pods", C.c_void_p),
                ("pod_patch_off", C.c_void_p), ("pod_patch_len", C.c_void_p), ("stream", C.c_void_p)]


def _np_dtype(st):
    """numpy structured dtype with the exact ctypes layout (for bulk batches)."""
    names, formats, offsets = [], [], []
    for name, ty in st._fields_:
        names.append(name)
        offsets.append(getattr(st, name).offset)
        if ty is KwokStr:
            formats.append(np.dtype([("off", "<u4"), ("len", "<u4")]))
        elif isinstance(ty, type) and issubclass(ty, C.Array):
            formats.append((np.dtype([("off", "<u4"), ("len", "<u4")]), (ty._length_,)))
        else:
            formats.append(np.dtype(ty))
    return np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": C.sizeof(st)})


NODE_EVENT_DTYPE = _np_dtype(NodeEvent)
POD_EVENT_DTYPE = _np_dtype(PodEvent)
POD_REC_DTYPE = _np_dtype(PodRec)
POD_REC12_DTYPE = _np_dtype(PodRec12)


def ip4(s: str) -> int:
    if not s:
        return 0
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def ip4s(v: int) -> str:
    return "" if not v else "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)


def fnv1a32(s: str) -> int:
    h = 0x811C9DC5
    for b in s.encode():
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


class Arena:
    """Growing byte arena + kwok_str refs for one ingest batch."""

    def __init__(self):
        self.buf = bytearray()
        self._intern = {}

    def ref(self, s) -> tuple[int, int]:
        if s is None or s == "" or s == b"":
            return (0, 0)
        b = s.encode() if isinstance(s, str) else bytes(s)
        r = self._intern.get(b)
        if r is None:
            r = (len(self.buf), len(b))
            self.buf += b
            self._intern[b] = r
        return r

    def kstr(self, s) -> KwokStr:
        o, n = self.ref(s)
        return KwokStr(o, n)

    def cbuf(self):
        b = bytes(self.buf) or b"\0"
        return C.create_string_buffer(b, len(b)), len(self.buf)


def pack_pod_events(ev: np.ndarray, ips_host: np.ndarray | None = None, ips_pod: np.ndarray | None = None):
    """kwok_pod_event rows (POD_EVENT_DTYPE) whose IPs are given as integers
    (ips_*: per row, 0 = empty) -> POD_REC_DTYPE rows, vectorised: what
    kwok_pack_pod_events computes from the strings"""
    n = len(ev)
    out = np.zeros(n, POD_REC_DTYPE)
    create = (ev["op"] == OP_UPSERT) & (ev["handle"] < 0)
    out["op"] = ev["op"] | np.where(create, REC_NEW, 0).astype(np.uint8)
    out["flags"] = (ev["flags"] & 31) | (ev["phase"].astype(np.uint8) << REC_PHASE_SHIFT)
    out["spec_id"] = np.where(ev["op"] == OP_UPSERT, ev["spec_id"], 0)
    out["target"] = np.where(create, ev["node_handle"], ev["handle"])
    out["creation"] = np.where(ev["op"] == OP_UPSERT, ev["creation_unix"], 0)
    if ips_host is not None:
        out["host_ip"] = np.where(ev["op"] == OP_UPSERT, ips_host, 0)
    if ips_pod is not None:
        out["pod_ip"] = ips_pod
    return out


def pack12(recs: np.ndarray, node_ip: int, out: np.ndarray | None = None) -> np.ndarray:
    """POD_REC_DTYPE rows -> POD_REC12_DTYPE rows (every hostIP empty or node_ip,
    no create holding a podIP; ValueError otherwise: such a record goes through
    kwok_ingest_pods_packed)"""
    hip = recs["host_ip"]
    new = (recs["op"] & REC_NEW) != 0
    if ((hip != 0) & (hip != node_ip)).any():
        raise ValueError("a hostIP other than the node IP: not expressible as kwok_pod_rec12")
    if (new & (recs["pod_ip"] != 0)).any():
        raise ValueError("a create holding a podIP: not expressible as kwok_pod_rec12")
    o = np.empty(len(recs), POD_REC12_DTYPE) if out is None else out[:len(recs)]
    o["op"] = recs["op"] | np.where(hip != 0, REC_HOST_NODE_IP, 0).astype(np.uint8)
    for f in ("flags", "spec_id", "target"):
        o[f] = recs[f]
    o["value"] = np.where(new, recs["creation"], recs["pod_ip"])
    return o
