#!/usr/bin/env python3
"""Latency of the first small GPU operation (a 64-byte memset + stream sync)
after the host has left the GPU idle for a while, as the bench's churn leg does
between steps (event generation).  Diagnostics for DESIGN.md §11."""
import ctypes as C
import time

import torch  # noqa: F401  (the HIP runtime)

torch.cuda.init()
hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
dev = C.c_void_p()
assert hip.hipMalloc(C.byref(dev), 1 << 20) == 0
st = C.c_void_p()
assert hip.hipStreamCreate(C.byref(st)) == 0


def op():
    t0 = time.perf_counter()
    assert hip.hipMemsetAsync(dev, 0, 64, st) == 0
    assert hip.hipStreamSynchronize(st) == 0
    return (time.perf_counter() - t0) * 1e3


for idle in (0.0, 0.01, 0.05, 0.1, 0.2, 0.4, 1.0):
    out = []
    for _ in range(8):
        time.sleep(idle)
        out.append(op())
    print("[idle %.2fs] first op after idle, ms: %s" % (idle, " ".join("%.2f" % x for x in out)))
