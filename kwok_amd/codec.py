"""Host watch-event codec: Kubernetes Node / Pod JSON -> the ingest records of
include/kwok_engine.h (kwok_decode_node / kwok_decode_pod, csrc/codec.cpp).

This is the Python face of the C codec, mirroring what the reference's
WatchNodes / WatchPods do per object before queueing it
(pkg/kwok/controllers/node_controller.go:206-270, pod_controller.go:252-343)
and computePatchData's no-op test (pod_controller.go:404-439).  Decoded string
references point into one shared arena (the concatenated documents), which is
exactly the arena kwok_ingest_nodes / kwok_ingest_pods take."""
from __future__ import annotations

import ctypes as C
import json

from . import abi
from .engine import KwokError, load_engine_lib


def _b(s):
    return None if s is None else (s.encode() if isinstance(s, str) else s)


def selector_matches(selector: str, labels: dict | None) -> bool:
    """labels.Parse(selector).Matches(labels.Set(labels)); "" is the nil selector (never matches)."""
    lib = load_engine_lib()
    js = json.dumps(labels).encode()
    out = C.c_int32()
    rc = lib.kwok_selector_matches(_b(selector), js, len(js), C.byref(out))
    if rc:
        raise KwokError(rc, lib.kwok_codec_last_error().decode())
    return bool(out.value)


class Batch:
    """Decoded records of one ingest batch plus their shared arena."""

    def __init__(self):
        self.buf = bytearray()
        self.nodes: list[abi.NodeEvent] = []
        self.pods: list[abi.PodDoc] = []
        self.status: list[int] = []

    def text(self, r: abi.KwokStr) -> str:
        return bytes(self.buf[r.off:r.off + r.len]).decode()

    def arena(self):
        b = bytes(self.buf) or b"\0"
        return C.create_string_buffer(b, len(b)), len(self.buf)


class Codec:
    def __init__(self, manage_all_nodes=True, manage_nodes_with_annotation_selector="",
                 manage_nodes_with_label_selector="", disregard_status_with_annotation_selector="",
                 disregard_status_with_label_selector=""):
        self._lib = load_engine_lib()
        cfg = abi.CodecConfig(int(bool(manage_all_nodes)), _b(manage_nodes_with_annotation_selector),
                              _b(manage_nodes_with_label_selector), _b(disregard_status_with_annotation_selector),
                              _b(disregard_status_with_label_selector))
        h = C.c_void_p()
        rc = self._lib.kwok_codec_create(C.byref(cfg), C.byref(h))
        if rc:
            raise KwokError(rc, "codec: %s" % self._lib.kwok_codec_last_error().decode())
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.kwok_codec_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _decode(self, kind, docs, strict, threads=1):
        b = Batch()
        offs, lens = [], []
        for d in docs:
            raw = d if isinstance(d, (bytes, bytearray)) else json.dumps(d).encode()
            offs.append(len(b.buf))
            lens.append(len(raw))
            b.buf += raw
        n = len(offs)
        cbuf = C.create_string_buffer(bytes(b.buf) or b"\0", max(1, len(b.buf)))
        off_a, len_a = (C.c_uint64 * max(1, n))(*offs), (C.c_uint32 * max(1, n))(*lens)
        recs = ((abi.NodeEvent if kind == "node" else abi.PodDoc) * max(1, n))()
        st = (C.c_int32 * max(1, n))()
        fn = self._lib.kwok_decode_nodes if kind == "node" else self._lib.kwok_decode_pods
        bad = fn(self._h, cbuf, len(b.buf), off_a, len_a, n, threads, recs, st)
        if bad < 0 or (bad and strict):
            raise KwokError(bad if bad < 0 else st[[x for x in range(n) if st[x]][0]],
                            "decode_%ss: %s" % (kind, self._lib.kwok_codec_last_error().decode()))
        b.status = list(st[:n])
        (b.nodes if kind == "node" else b.pods).extend(recs[:n])
        b.buf = bytearray(cbuf.raw[:len(b.buf)])  # node blobs were canonicalised in place
        return b

    def decode_nodes(self, docs, strict=True, threads=1) -> Batch:
        return self._decode("node", docs, strict, threads)

    def decode_pods(self, docs, strict=True, threads=1) -> Batch:
        return self._decode("pod", docs, strict, threads)
