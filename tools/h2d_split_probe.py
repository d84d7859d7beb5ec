#!/usr/bin/env python3
"""Host-to-device rate of one C4 batch's records (24 MB of kwok_pod_rec12, page-locked)
copied as one hipMemcpyAsync or split over 2 / 4 streams (copy engines) at once.
Diagnostics for DESIGN.md §11 (the C4 ingest is link-bound)."""
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
hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
from kwok_amd import engine as keng  # noqa: E402

for mb in (24, 96):
    N = mb << 20
    dev = C.c_void_p()
    assert hip.hipMalloc(C.byref(dev), N) == 0
    src = keng.host_array((N,), np.uint8)
    src[:] = 1
    sts = []
    for _ in range(4):
        s = C.c_void_p()
        assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0
        sts.append(s)
    for ways in (1, 2, 4):
        best = 1e9
        for rep in range(12):
            t0 = time.perf_counter()
            for w in range(ways):
                lo, hi = N * w // ways, N * (w + 1) // ways
                assert hip.hipMemcpyAsync(C.c_void_p(dev.value + lo), C.c_void_p(src.ctypes.data + lo), hi - lo, 1,
                                          sts[w]) == 0
            for w in range(ways):
                assert hip.hipStreamSynchronize(sts[w]) == 0
            dt = time.perf_counter() - t0
            if rep >= 2:
                best = min(best, dt)
        print("%3d MB, %d way(s): best %.3f ms -> %.1f GB/s" % (mb, ways, best * 1e3, N / best / 1e9), flush=True)
