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
        L.jc_leader_prep_init.argtypes = [ctypes.c_int] * 4 + [vp, ctypes.c_uint64] + [vp] * 6 + [ctypes.c_int]
        L.jc_leader_prep_init.restype = ctypes.c_int
        L.jc_leader_finish_aggregate.argtypes = [ctypes.c_int] * 4 + [ctypes.c_uint64] + [vp] * 10 + [ctypes.c_int]
        L.jc_leader_finish_aggregate.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else np.ascontiguousarray(a).ctypes.data_as(ctypes.c_void_p)


def helper_prep_aggregate(algo, bits, length, chunk, vk: bytes, nonces, ps, his, lps, nthreads: int = 1):
    """Returns dict(verdicts, prep_msgs, agg, count, checksum) for n fixed-stride reports."""
    n = int(nonces.shape[0])
    verdicts = np.zeros(max(n, 1), np.uint8)
    msgs = np.zeros((max(n, 1), 16), np.uint8)
    out_len, fb = (1, 8) if algo == 0 else (1, 16) if algo == 1 else (length, 16)
    agg = np.zeros(out_len * fb, np.uint8)
    cs = np.zeros(32, np.uint8)
    cnt = ctypes.c_uint64()
    keep = [np.ascontiguousarray(x) if x is not None and x.size else np.zeros(1, np.uint8)
            for x in (nonces, ps, his, lps)]
    vkb = np.frombuffer(vk, np.uint8).copy()
    rc = lib().jc_helper_prep_aggregate(algo, bits, length, chunk, _p(vkb), n, *[_p(x) for x in keep], _p(verdicts),
                                        _p(msgs), _p(agg), ctypes.byref(cnt), _p(cs), nthreads)
    if rc:
        raise ValueError("unsupported parameters for the CPU baseline engine")
    return {"verdicts": verdicts[:n], "prep_msgs": msgs[:n], "agg": agg.tobytes(), "count": cnt.value,
            "checksum": cs.tobytes()}


def leader_prep_init(algo, bits, length, chunk, vk: bytes, nonces, ps, lis, lps_len: int, nthreads: int = 1):
    """Leader prepare_init: dict(verdicts, prep_shares [n, lps_len], seeds [n, 16])."""
    n = int(nonces.shape[0])
    verdicts = np.zeros(max(n, 1), np.uint8)
    shares = np.zeros((max(n, 1), lps_len), np.uint8)
    seeds = np.zeros((max(n, 1), 16), np.uint8)
    keep = [np.ascontiguousarray(x) for x in (nonces, ps, lis)]
    vkb = np.frombuffer(vk, np.uint8).copy()
    rc = lib().jc_leader_prep_init(algo, bits, length, chunk, _p(vkb), n, *[_p(x) for x in keep], _p(shares),
                                   _p(seeds), _p(verdicts), nthreads)
    if rc:
        raise ValueError("unsupported parameters for the CPU baseline leader")
    return {"verdicts": verdicts[:n], "prep_shares": shares[:n], "seeds": seeds[:n]}


def leader_finish_aggregate(algo, bits, length, chunk, nonces, lis, seeds, init_verdicts, prep_msgs,
                            peer_verdicts=None, nthreads: int = 1):
    """Leader prepare_next + accumulate: dict(verdicts, agg, count, checksum)."""
    n = int(nonces.shape[0])
    out_len = 1 if algo == 1 else length
    verdicts = np.zeros(max(n, 1), np.uint8)
    agg = np.zeros(out_len * 16, np.uint8)
    cs = np.zeros(32, np.uint8)
    cnt = ctypes.c_uint64()
    keep = [np.ascontiguousarray(x) for x in (nonces, lis, seeds, init_verdicts, prep_msgs)]
    pv = None if peer_verdicts is None else np.ascontiguousarray(peer_verdicts, dtype=np.uint8)
    rc = lib().jc_leader_finish_aggregate(algo, bits, length, chunk, n, *[_p(x) for x in keep], _p(pv), _p(verdicts),
                                          _p(agg), ctypes.byref(cnt), _p(cs), nthreads)
    if rc:
        raise ValueError("unsupported parameters for the CPU baseline leader")
    return {"verdicts": verdicts[:n], "agg": agg.tobytes(), "count": cnt.value, "checksum": cs.tobytes()}
