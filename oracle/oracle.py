"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It reuses the ABI-generic driver with the oracle's symbol
prefix; the oracle library is built from oracle/kwok_oracle.c (oracle/Makefile).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

from kwok_amd import engine as _eng

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libkwok_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _eng.declare(_lib, "kwok_oracle_")
        _lib.kwok_oracle_set_threads.restype = C.c_int
        _lib.kwok_oracle_set_threads.argtypes = [C.c_void_p, C.c_int]
    return _lib


class Oracle(_eng.EngineBase):
    PREFIX = "kwok_oracle_"

    def __init__(self, cfg=None, threads=1, **kw):
        super().__init__(load(), cfg if cfg is not None else _eng.make_config(**kw))
        self.threads = self.set_threads(threads)

    def set_threads(self, n):
        """host threads of the tick's sweeps (OpenMP; <= 0: all cores); the
        outputs are the same for every count"""
        self.threads = self._lib.kwok_oracle_set_threads(self._h, n)
        return self.threads
