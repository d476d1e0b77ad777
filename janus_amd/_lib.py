"""Loader for the in-tree HIP engine library (libjanus_prio3.so, C ABI in include/jx_prio3.h).

There is no CPU fallback: if the library is missing or no HIP device is present,
every engine entry point raises. Build with ``python -m janus_amd.build``.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libjanus_prio3.so")

# Every symbol include/jx_prio3.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "jx_engine_create", "jx_engine_create_ex", "jx_engine_destroy", "jx_engine_sizes", "jx_engine_set_capacity",
    "jx_helper_prep_batch", "jx_engine_batch_id", "jx_engine_batches", "jx_batch_release",
    "jx_batch_aggregate_records", "jx_batch_aggregate_records_device", "jx_engine_leader_sizes", "jx_leader_prep_init_batch",
    "jx_leader_prep_finish_batch", "jx_leader_prep_init_device", "jx_leader_prep_finish_device",
    "jx_accumulate", "jx_accumulate_device", "jx_helper_prep_aggregate", "jx_helper_prep_aggregate_device",
    "jx_aggregate_read", "jx_aggregate_checksum", "jx_aggregate_reset", "jx_aggregate_export_device",
    "jx_aggregate_combine_device", "jx_shard_record_bytes", "jx_shard_record_export_device",
    "jx_shard_record_combine_device", "jx_engine_sync", "jx_engine_stream", "jx_engine_timing",
    "jx_engine_timing_read", "jx_engine_debug", "jx_status_str", "jx_last_error",
    "jx_engine_wait_stream", "jx_engine_join_stream", "jx_engine_wait_event", "jx_engine_record_event",
    "jx_engine_memory", "jx_engine_coalesce", "jx_leader_prep_init_device_ex", "jx_helper_prep_encrypted_batch",
)

_lib = None


class JxParams(ctypes.Structure):
    _fields_ = [("algo_id", ctypes.c_uint32), ("bits", ctypes.c_uint32), ("length", ctypes.c_uint32),
                ("chunk_length", ctypes.c_uint32), ("num_proofs", ctypes.c_uint32)]


class JxMemoryStats(ctypes.Structure):
    _fields_ = [(name, ctypes.c_uint64) for name in (
        "resident_batches", "batch_bytes", "arena_budget", "arena_allocated", "arena_in_use", "arena_peak",
        "arena_allocs", "arena_reuses", "arena_waits", "arena_engines", "last_pipelines", "coalesced_launches",
        "coalesced_jobs", "coalesced_reports", "coalesce_window_us", "coalesce_gather_us", "coalesce_copy_us",
        "coalesce_enqueue_us", "coalesce_device_us", "arena_cross_stream_waits", "coalesce_pinned_bytes",
        "coalesced_helper_launches", "coalesced_helper_jobs", "coalesced_leader_launches", "coalesced_leader_jobs",
        "coalesced_encrypted_jobs", "arena_frees")]


class EngineError(RuntimeError):
    pass


def load():
    """Load the shared library and declare exact argument types (fails loudly)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"{LIB_PATH} is missing: build it with `python -m janus_amd.build` "
                          "(there is no CPU fallback)")
    # One HIP runtime per process: torch bundles libamdhip64.so (soname libamdhip64.so.7).
    # Loading torch first makes our NEEDED libamdhip64.so.7 resolve to that same runtime;
    # loading ours first would put two HSA runtimes in the process and break torch.cuda.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, u8p = ctypes.c_void_p, ctypes.c_void_p
    i32, u32, u64 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64
    P = ctypes.POINTER
    sig = {
        "jx_engine_create": (i32, [P(JxParams), u8p, i32, P(vp)]),
        "jx_engine_create_ex": (i32, [P(JxParams), u8p, u32, i32, P(vp)]),
        "jx_engine_destroy": (None, [vp]),
        "jx_engine_sizes": (i32, [vp, P(u32), P(u32), P(u32), P(u32), P(u32), P(u32)]),
        "jx_engine_set_capacity": (i32, [vp, u64]),
        "jx_helper_prep_batch": (i32, [vp, u64, u8p, u8p, u8p, u8p, u8p, u8p, u8p, P(u64)]),
        "jx_helper_prep_encrypted_batch": (i32, [vp, u64, u8p, P(u64), u8p, u8p, P(vp), u32, u8p, u8p, u8p, P(u64),
                                                  u32, u8p, u8p, u8p, u8p, P(u64)]),
        "jx_engine_batch_id": (i32, [vp, P(u64)]),
        "jx_engine_batches": (i32, [vp, P(u64), P(u64)]),
        "jx_batch_release": (i32, [vp, u64]),
        "jx_batch_aggregate_records": (i32, [vp, u64, u64, u8p, u8p, u32, u8p]),
        "jx_batch_aggregate_records_device": (i32, [vp, u64, u64, vp, vp, u32, vp]),
        "jx_engine_leader_sizes": (i32, [vp, P(u32)]),
        "jx_leader_prep_init_batch": (i32, [vp, u64, u8p, u8p, u8p, u8p, u8p, P(u64)]),
        "jx_leader_prep_finish_batch": (i32, [vp, u64, u64, u8p, u8p, u8p]),
        "jx_leader_prep_init_device": (i32, [vp, u64, vp, vp, vp, vp, vp, P(u64)]),
        "jx_leader_prep_init_device_ex": (i32, [vp, u64, vp, vp, vp, u64, vp, vp, P(u64)]),
        "jx_engine_memory": (i32, [vp, P(JxMemoryStats)]),
        "jx_engine_coalesce": (i32, [vp, i32, u32]),
        "jx_leader_prep_finish_device": (i32, [vp, u64, u64, vp, vp, vp]),
        "jx_accumulate": (i32, [vp, u64, u64, u8p, u8p]),
        "jx_accumulate_device": (i32, [vp, u64, u64, vp, vp, P(u32), u32]),
        "jx_helper_prep_aggregate": (i32, [vp, u64, u8p, u8p, u8p, u8p, u32, u8p, u8p]),
        "jx_helper_prep_aggregate_device": (i32, [vp, u64, vp, vp, vp, vp, vp, P(u32), u32, vp, vp]),
        "jx_aggregate_read": (i32, [vp, u32, u8p, P(u64)]),
        "jx_aggregate_checksum": (i32, [vp, u32, u8p]),
        "jx_aggregate_reset": (i32, [vp]),
        "jx_aggregate_export_device": (i32, [vp, u32, vp]),
        "jx_aggregate_combine_device": (i32, [vp, vp, u32, vp]),
        "jx_shard_record_bytes": (i32, [vp, P(u32)]),
        "jx_shard_record_export_device": (i32, [vp, u32, vp]),
        "jx_shard_record_combine_device": (i32, [vp, vp, u32, vp]),
        "jx_engine_sync": (i32, [vp]),
        "jx_engine_stream": (i32, [vp, P(vp)]),
        "jx_engine_wait_stream": (i32, [vp, vp]),
        "jx_engine_join_stream": (i32, [vp, vp]),
        "jx_engine_wait_event": (i32, [vp, vp]),
        "jx_engine_record_event": (i32, [vp, vp]),
        "jx_engine_timing": (i32, [vp, i32]),
        "jx_engine_timing_read": (i32, [vp, P(ctypes.c_float), P(u64)]),
        "jx_engine_debug": (i32, [vp, i32, ctypes.c_int64]),
        "jx_status_str": (ctypes.c_char_p, [i32]),
        "jx_last_error": (ctypes.c_char_p, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(status: int, engine_ptr=None, what: str = "") -> None:
    if status == 0:
        return
    L = load()
    msg = L.jx_status_str(status).decode()
    detail = L.jx_last_error(engine_ptr).decode() if engine_ptr else ""
    raise EngineError(f"{what}: {msg} ({status}) {detail}".strip())
