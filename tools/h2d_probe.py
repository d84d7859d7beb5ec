#!/usr/bin/env python3
"""Host-to-device copy rate of a 96 MB batch (2M kwok_pod_event records), as
kwok_ingest_pods issues it: page-locked (kwok_host_alloc) vs pageable source,
with and without the CPU rewriting the buffer before each copy (the bench's
Churn generator does), one copy per round.  Diagnostics for DESIGN.md §14."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (the HIP runtime the engine binds)

torch.cuda.init()
hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
from kwok_amd import engine as keng  # noqa: E402

N = 96 << 20
dev = C.c_void_p()
assert hip.hipMalloc(C.byref(dev), N) == 0
st = C.c_void_p()
assert hip.hipStreamCreate(C.byref(st)) == 0
pinned = keng.host_array((N,), np.uint8)
pageable = np.zeros(N, np.uint8)


big = torch.empty(6 << 30, dtype=torch.uint8, device="cuda")


dsrc = C.c_void_p()
assert hip.hipMalloc(C.byref(dsrc), 100 << 20) == 0
dump_pinned = keng.host_array((100 << 20,), np.uint8)


def d2h(kind):
    """a 100 MB device -> host read between copies, as the bench's dump_pods does"""
    dst = np.zeros(100 << 20, np.uint8) if kind == "fresh" else dump_pinned
    assert hip.hipMemcpyAsync(dst.ctypes.data, dsrc, 100 << 20, 2, st) == 0
    assert hip.hipStreamSynchronize(st) == 0


def run(buf, write, rounds=10, sleep=0.0, thrash=False, dump=None):
    out = []
    for r in range(rounds):
        if dump:
            d2h(dump)
        if thrash:  # touch 6 GiB of device memory between copies (as a tick's arena writes do)
            big.fill_(r & 255)
            torch.cuda.synchronize()
        if write:
            buf[::4096] = r & 255  # touch every page
            buf[: N // 2] = r  # rewrite half the buffer
        if sleep:
            time.sleep(sleep)
        t0 = time.perf_counter()
        assert hip.hipMemcpyAsync(dev, buf.ctypes.data, N, 1, st) == 0
        assert hip.hipStreamSynchronize(st) == 0
        out.append(N / (time.perf_counter() - t0) / 1e9)
    return " ".join("%.0f" % x for x in out)


tag = "SDMA=%s alloc=%s" % (os.environ.get("HSA_ENABLE_SDMA", "default"), os.environ.get("KWOK_HOST_ALLOC", "thp"))
print("[h2d %s] pinned           GB/s: %s" % (tag, run(pinned, False)))
print("[h2d %s] pinned + writes  GB/s: %s" % (tag, run(pinned, True)))
print("[h2d %s] pinned + idle    GB/s: %s" % (tag, run(pinned, True, sleep=0.2)))
print("[h2d %s] pinned + thrash   GB/s: %s" % (tag, run(pinned, True, thrash=True)))
print("[h2d %s] pinned + D2H into fresh pageable GB/s: %s" % (tag, run(pinned, True, dump="fresh")))
print("[h2d %s] pinned + D2H into pinned         GB/s: %s" % (tag, run(pinned, True, dump="pinned")))
print("[h2d %s] pageable         GB/s: %s" % (tag, run(pageable, False)))
print("[h2d %s] pageable + writes GB/s: %s" % (tag, run(pageable, True)))
