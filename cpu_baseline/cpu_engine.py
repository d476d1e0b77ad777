"""ctypes view of the CPU baseline engine (cpu_baseline/jc_cpu_engine.cpp).

BENCHMARK BASELINE ONLY: bench.py's cpu_baseline leg and tests/test_cpu_baseline.py use it; the
product path (janus_amd) never loads it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libjc_cpu_engine.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        L.jc_helper_prep_aggregate.argtypes = [ctypes.c_int] * 4 + [vp, ctypes.c_uint64] + [vp] * 8 + [vp, ctypes.c_int]
        L.jc_helper_prep_aggregate.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else np.ascontiguousarray(a).ctypes.data_as(ctypes.c_void_p)


def helper_prep_aggregate(algo, bits, length, chunk, vk: bytes, nonces, ps, his, lps, nthreads: int = 1):
    """Returns dict(verdicts, prep_msgs, agg, count, checksum) for n fixed-stride reports."""
    n = int(nonces.shape[0])
    verdicts = np.zeros(max(n, 1), np.uint8)
    msgs = np.zeros((max(n, 1), 16), np.uint8)
    agg = np.zeros(length * 16, np.uint8)
    cs = np.zeros(32, np.uint8)
    cnt = ctypes.c_uint64()
    keep = [np.ascontiguousarray(x) for x in (nonces, ps, his, lps)]
    vkb = np.frombuffer(vk, np.uint8).copy()
    rc = lib().jc_helper_prep_aggregate(algo, bits, length, chunk, _p(vkb), n, *[_p(x) for x in keep], _p(verdicts),
                                        _p(msgs), _p(agg), ctypes.byref(cnt), _p(cs), nthreads)
    if rc:
        raise ValueError("unsupported parameters for the CPU baseline engine")
    return {"verdicts": verdicts[:n], "prep_msgs": msgs[:n], "agg": agg.tobytes(), "count": cnt.value,
            "checksum": cs.tobytes()}
