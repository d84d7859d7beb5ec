"""kwok_amd - MI355X-native engine for kwok's fake-kubelet tick.

The product is the C-ABI library kwok_amd/lib/libkwok_engine.so (HIP kernels
for gfx950 + C++ host runtime, include/kwok_engine.h).  This package holds its
Python binding (engine.py), the ABI mirror (abi.py), the host-side mirror of
the reference controller interface (controllers.py) and the synthetic
workload generator used by bench.py (workload.py).
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
