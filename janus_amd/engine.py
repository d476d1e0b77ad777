"""Batched Prio3 helper preparation + aggregation on one MI355X (wrapper of include/jx_prio3.h).

This is the host-side mirror of the prio `vdaf::Aggregator` + ping-pong surface that
Janus calls per report at /root/reference/aggregator/src/aggregator.rs:1945-1967:

    vdaf.helper_initialized(verify_key, agg_param, nonce, public_share, input_share,
                            leader_message).and_then(|t| t.evaluate(&vdaf))

`HelperEngine.helper_initialized_batch` does that for a whole batch and returns, per
report, either the outbound `PingPongMessage::Finish{prep_msg}` or a verdict naming the
`PingPongError` variant (labels of aggregator/src/aggregator/error.rs:379-424), plus the
handle of the new resident batch (one per aggregation job in flight; any number can be
resident). `aggregate_records` turns a batch into per-batch-identifier deltas
(BatchAggregation rows to merge with `merged_with`, aggregator_core/src/datastore/
models.rs:1275-1330) without changing the engine, so a retried datastore transaction can
recompute them; `accumulate` merges a batch into the engine's running aggregations (the
engine as one shard) and releases it.

Device-pointer methods (`*_device`) order themselves against a torch stream (default: the current
stream of the engine's device): the engine's work waits for everything queued on that stream before
the call (the producer of the inputs), and work queued on that stream afterwards waits for the
engine's (the consumer of the outputs, and torch's allocator reusing the inputs). So tensors produced
and consumed on torch's current stream need no `sync()`. Pass `stream=False` to order by hand
(`wait_stream` / `join_stream` / events), e.g. to keep two engines' jobs overlapping.

Resident batches hold device memory until released: `helper_initialized_batch(keep=False)` drops the
batch at once, `resident(batch_id)` is a context manager that releases it on exit, and the aggregator
paths release in `finally`.

All compute runs in the HIP kernels of libjanus_prio3.so; nothing here falls back to the CPU.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import EngineError, JxParams, check
from .vdaf import Prio3

FINISHED = 0
PREPARE_INIT_FAILURE = 1
PREP_SHARE_DECODE_FAILURE = 2
PREPARE_MESSAGE_FAILURE = 3
PREPARE_NEXT_FAILURE = 4
HELPER_STEP_FAILURE = 5  # leader only: the helper rejected the report
OPEN_FAILURE = 6  # encrypted inputs: the report never reached helper_initialized (see open_status)
VERDICT_LABELS = {
    FINISHED: "finished",
    PREPARE_INIT_FAILURE: "prepare_init_failure",
    PREP_SHARE_DECODE_FAILURE: "leader_prep_share_decode_failure",
    PREPARE_MESSAGE_FAILURE: "prepare_message_failure",
    PREPARE_NEXT_FAILURE: "prepare_next_failure",
    HELPER_STEP_FAILURE: "helper_step_failure",
}
# open status of an encrypted input share (include/jx_prio3.h JX_OPEN_*; aggregator.rs:1781-1910):
# (janus_step_failures label, PrepareError value)
OPEN_OK = 0
KEY_NONE, KEY_MALFORMED = 0xFF, 0xFE
ENC_REQUIRE_TASKPROV = 1
OPEN_STATUS = {
    1: ("decrypt_failure", 4),                           # HpkeDecryptError
    2: ("plaintext_input_share_decode_failure", 8),      # InvalidMessage
    3: ("duplicate_extension", 8),
    4: ("unexpected_taskprov_extension", 8),
    5: ("missing_or_malformed_taskprov_extension", 8),
    6: ("input_share_decode_failure", 8),
    7: ("unknown_hpke_config_id", 3),                    # HpkeUnknownConfigId
}


def _ptr(a: np.ndarray | None):
    if a is None:
        return None
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data_as(ctypes.c_void_p)


def _u8(a, n: int, width: int, what: str) -> np.ndarray:
    arr = np.ascontiguousarray(np.frombuffer(a, np.uint8) if isinstance(a, (bytes, bytearray)) else a,
                               dtype=np.uint8)
    if width == 0:
        return np.zeros((max(n, 1), 1), np.uint8)
    arr = arr.reshape(n, width) if arr.size == n * width else None
    if arr is None:
        raise ValueError(f"{what}: expected {n} x {width} bytes")
    return arr


def _seg_table(segment_ids):
    ids = np.ascontiguousarray(np.asarray(segment_ids, dtype=np.uint32).reshape(-1))
    if ids.size == 0:
        raise ValueError("at least one segment id")
    return ids, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


@dataclass
class LeaderInit:
    verdicts: np.ndarray       # uint8[n]: 0 initialized, 1 prepare_init_failure
    prep_shares: np.ndarray    # uint8[n, LPS]: payloads of PingPongMessage::Initialize
    batch_id: int = 0          # the resident leader batch (finish / records / accumulate / release)


@dataclass
class BatchResult:
    verdicts: np.ndarray       # uint8[n]
    prep_msgs: np.ndarray      # uint8[n, PM]
    out_shares: np.ndarray | None  # uint8[n, OUT*FB]
    batch_id: int = 0          # the resident batch these results belong to (records / accumulate / release)

    def finished(self) -> np.ndarray:
        return self.verdicts == FINISHED


@dataclass
class EncryptedResult:
    verdicts: np.ndarray       # uint8[n]: as BatchResult, OPEN_FAILURE where the share did not open / decode
    prep_msgs: np.ndarray      # uint8[n, PM]
    open_status: np.ndarray    # uint8[n]: OPEN_OK or an OPEN_STATUS key
    batch_id: int = 0


class HelperEngine:
    """One engine per (Prio3 instance, verify key, GPU). Serves the helper role (the north-star
    path) and the leader role of the same ping-pong exchange."""

    _leader_n = 0
    _leader_id = 0

    def __init__(self, vdaf: Prio3, verify_key: bytes, device: int = 0):
        # guards the per-instance defaults (last leader batch) when threads share the engine; the
        # C engine serializes the calls themselves
        self._lock = threading.Lock()
        if len(verify_key) != vdaf.verify_key_len:
            raise ValueError(f"verify key must be {vdaf.verify_key_len} bytes for {vdaf.name()} "
                             "(VERIFY_KEY_LENGTH / VERIFY_KEY_LENGTH_HMACSHA256_AES128, core/src/vdaf.rs:16,24)")
        self.vdaf = vdaf
        self.device = device
        L = _lib.load()
        self._L = L
        p = JxParams(vdaf.algo_id, vdaf.bits, vdaf.length, vdaf.chunk_length, vdaf.num_proofs)
        h = ctypes.c_void_p()
        vk = (ctypes.c_uint8 * len(verify_key)).from_buffer_copy(verify_key)
        st = L.jx_engine_create_ex(ctypes.byref(p), ctypes.cast(vk, ctypes.c_void_p), len(verify_key), device,
                                   ctypes.byref(h))
        check(st, None, f"jx_engine_create({vdaf.name()})")
        self._h = h
        sizes = [ctypes.c_uint32() for _ in range(6)]
        check(L.jx_engine_sizes(h, *[ctypes.byref(s) for s in sizes]), h, "jx_engine_sizes")
        self.public_share_len, self.helper_input_share_len, self.prep_share_len, self.prep_msg_len, \
            self.output_len, self.field_bytes = (s.value for s in sizes)
        lis = ctypes.c_uint32()
        check(L.jx_engine_leader_sizes(h, ctypes.byref(lis)), h, "jx_engine_leader_sizes")
        self.leader_input_share_len = lis.value

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None):
            self._L.jx_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------------ stream ordering
    def _stream_handle(self, stream):
        """hipStream_t of `stream` (None: torch's current stream on the engine's device; a torch
        stream; or an integer handle); None when the caller orders by hand (stream=False)."""
        if stream is False:
            return None
        if stream is None:
            try:
                import torch
            except ImportError:  # raw device pointers without torch: the caller orders by hand
                return None
            stream = torch.cuda.current_stream(self.device)
        return int(getattr(stream, "cuda_stream", stream))

    def wait_stream(self, stream=None):
        """Engine work queued from now on waits for all work queued on `stream` so far."""
        h = self._stream_handle(stream)
        check(self._L.jx_engine_wait_stream(self._h, h or None), self._h, "jx_engine_wait_stream")

    def join_stream(self, stream=None):
        """Work queued on `stream` from now on waits for all engine work queued so far."""
        h = self._stream_handle(stream)
        check(self._L.jx_engine_join_stream(self._h, h or None), self._h, "jx_engine_join_stream")

    def wait_event(self, event):
        """The engine stream waits on a torch.cuda.Event (or hipEvent_t handle) recorded by the caller."""
        check(self._L.jx_engine_wait_event(self._h, int(getattr(event, "cuda_event", event))), self._h,
              "jx_engine_wait_event")

    def record_event(self, event):
        """Record a torch.cuda.Event (or hipEvent_t handle) on the engine stream."""
        h = int(getattr(event, "cuda_event", event))
        if h == 0 and hasattr(event, "record"):  # torch creates its event on the first record
            event.record()
            h = int(event.cuda_event)
        check(self._L.jx_engine_record_event(self._h, h), self._h, "jx_engine_record_event")

    @contextlib.contextmanager
    def _ordered(self, stream):
        h = self._stream_handle(stream)
        if h is None:  # stream=False (ordered by hand), or no torch to order against
            yield
            return
        check(self._L.jx_engine_wait_stream(self._h, h or None), self._h, "jx_engine_wait_stream")
        try:
            yield
        except BaseException:
            # the join still orders whatever the failed call queued; its own error must not hide the call's
            self._L.jx_engine_join_stream(self._h, h or None)
            raise
        check(self._L.jx_engine_join_stream(self._h, h or None), self._h, "jx_engine_join_stream")

    # ------------------------------------------------------------------ prepare
    def helper_initialized_batch(self, nonces, public_shares, helper_input_shares, leader_prep_shares,
                                 want_out_shares: bool = False, keep: bool = True) -> BatchResult:
        """prio ping-pong helper_initialized + evaluate for n reports (host buffers).

        leader_prep_shares are the prep_share payloads of the leaders'
        PingPongMessage::Initialize (fixed length; the aggregator layer rejects other
        lengths as leader_prep_share_decode_failure before calling this). keep=False releases the
        new resident batch before returning (callers that want only verdicts / prep messages /
        output shares); the result's batch_id is then 0."""
        n = len(nonces) // 16 if isinstance(nonces, (bytes, bytearray)) else int(np.asarray(nonces).shape[0])
        nn = _u8(nonces, n, 16, "nonces")
        ps = _u8(public_shares, n, self.public_share_len, "public_shares")
        his = _u8(helper_input_shares, n, self.helper_input_share_len, "helper_input_shares")
        lps = _u8(leader_prep_shares, n, self.prep_share_len, "leader_prep_shares")
        verdicts = np.zeros(max(n, 1), np.uint8)
        msgs = np.zeros((max(n, 1), max(self.prep_msg_len, 1)), np.uint8)
        outs = np.zeros((max(n, 1), self.output_len * self.field_bytes), np.uint8) if want_out_shares else None
        bid = ctypes.c_uint64()
        st = self._L.jx_helper_prep_batch(self._h, n, _ptr(nn), _ptr(ps) if self.public_share_len else None,
                                          _ptr(his), _ptr(lps), _ptr(msgs) if self.prep_msg_len else None,
                                          _ptr(verdicts), _ptr(outs), ctypes.byref(bid))
        check(st, self._h, "jx_helper_prep_batch")
        if not keep:
            self.release(bid.value)
            bid.value = 0
        return BatchResult(verdicts[:n], msgs[:n, : self.prep_msg_len], outs[:n] if outs is not None else None,
                           bid.value)

    def helper_initialized_encrypted_batch(self, nonces, times, public_shares, task_id: bytes, keypairs,
                                           key_index, encs, payloads: list[bytes], leader_prep_shares,
                                           require_taskprov: bool = False, keep: bool = True) -> "EncryptedResult":
        """The helper's per-report loop from the encrypted report share to helper_initialized + evaluate
        (aggregator.rs:1763-1967), on the GPU for the whole job (jx_helper_prep_encrypted_batch): report i
        is opened with keypairs[key_index[i][0]] (then keypairs[key_index[i][1]] if that fails to decrypt;
        KEY_NONE: none; KEY_MALFORMED: an encapsulated key that is not 32 bytes), its PlaintextInputShare
        decoded and checked, and prepared. keypairs: janus_amd.hpke.HpkeOpener contexts on this engine's
        device. Returns verdicts (OPEN_FAILURE where the share did not open / decode), prep messages, the
        open status per report (OPEN_STATUS) and the batch handle."""
        n = int(np.asarray(nonces).reshape(-1, 16).shape[0])
        nn = _u8(nonces, n, 16, "nonces")
        ps = _u8(public_shares, n, self.public_share_len, "public_shares")
        lps = _u8(leader_prep_shares, n, self.prep_share_len, "leader_prep_shares")
        tm = np.ascontiguousarray(np.asarray(times, dtype=np.uint64).reshape(n)) if n else np.zeros(1, np.uint64)
        ki = np.ascontiguousarray(np.asarray(key_index, dtype=np.uint8).reshape(n, 2)) if n else np.zeros((1, 2), np.uint8)
        en = _u8(encs, n, 32, "encs") if n else np.zeros((1, 32), np.uint8)
        if len(task_id) != 32 or len(payloads) != n:
            raise ValueError("task id is 32 bytes; one payload per report")
        off = np.zeros(n + 1, np.uint64)
        if n:
            off[1:] = np.cumsum([len(p) for p in payloads])
        ct = np.frombuffer(b"".join(payloads) or b"\0", np.uint8).copy()
        task = np.frombuffer(task_id, np.uint8).copy()
        hs = (ctypes.c_void_p * max(1, len(keypairs)))(*[k.handle for k in keypairs])
        verdicts = np.zeros(max(n, 1), np.uint8)
        status = np.zeros(max(n, 1), np.uint8)
        msgs = np.zeros((max(n, 1), max(self.prep_msg_len, 1)), np.uint8)
        bid = ctypes.c_uint64()
        st = self._L.jx_helper_prep_encrypted_batch(
            self._h, n, _ptr(nn), tm.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            _ptr(ps) if self.public_share_len else None, _ptr(task), hs, len(keypairs), _ptr(ki), _ptr(en), _ptr(ct),
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), ENC_REQUIRE_TASKPROV if require_taskprov else 0,
            _ptr(lps), _ptr(msgs) if self.prep_msg_len else None, _ptr(verdicts), _ptr(status), ctypes.byref(bid))
        check(st, self._h, "jx_helper_prep_encrypted_batch")
        if not keep:
            self.release(bid.value)
            bid.value = 0
        return EncryptedResult(verdicts[:n], msgs[:n, : self.prep_msg_len], status[:n], bid.value)

    def batch_id(self) -> int:
        """Handle of the most recently prepared batch if still resident (0 otherwise)."""
        b = ctypes.c_uint64()
        check(self._L.jx_engine_batch_id(self._h, ctypes.byref(b)), self._h, "jx_engine_batch_id")
        return b.value

    def resident_batches(self) -> tuple[int, int]:
        """(resident batches, device bytes they hold)."""
        n, b = ctypes.c_uint64(), ctypes.c_uint64()
        check(self._L.jx_engine_batches(self._h, ctypes.byref(n), ctypes.byref(b)), self._h, "jx_engine_batches")
        return n.value, b.value

    def release(self, batch_id: int, missing_ok: bool = False):
        """Drop a resident batch (an aggregation job that is done or abandoned). missing_ok: a batch
        that is no longer resident (already accumulated or released) is not an error."""
        st = self._L.jx_batch_release(self._h, batch_id)
        if st == -5 and missing_ok:  # JX_E_STATE
            return
        check(st, self._h, "jx_batch_release")

    @contextlib.contextmanager
    def resident(self, batch_id: int):
        """Scope of a resident batch: released on exit unless accumulate already consumed it."""
        try:
            yield batch_id
        finally:
            if batch_id:
                self.release(batch_id, missing_ok=True)

    def aggregate_records(self, batch_id: int, n: int, accept_mask: np.ndarray | None = None,
                          segment_index: np.ndarray | None = None, nsegments: int = 1) -> list[tuple[bytes, int, bytes]]:
        """Per-batch-identifier deltas of a resident batch: for each of nsegments aggregations, the
        (encoded aggregate share, report count, checksum) of the finished reports i with
        accept_mask[i] and segment_index[i] == that index. Changes nothing on the engine: repeatable
        (a retried transaction recomputes the same rows), the batch stays resident."""
        m = None if accept_mask is None else np.ascontiguousarray(accept_mask, dtype=np.uint8)
        s = None if segment_index is None else np.ascontiguousarray(segment_index, dtype=np.uint32)
        rb = self.record_bytes()
        out = np.zeros(nsegments * rb, np.uint8)
        check(self._L.jx_batch_aggregate_records(self._h, batch_id, n, _ptr(m), _ptr(s), nsegments, _ptr(out)),
              self._h, "jx_batch_aggregate_records")
        from .distributed import unpack_record
        return [unpack_record(out[k * rb:(k + 1) * rb], self.field_bytes) for k in range(nsegments)]

    def aggregate_records_device(self, batch_id: int, n: int, d_accept_mask: int | None, d_segment_index: int | None,
                                 nsegments: int, d_out_records: int, stream=None):
        """aggregate_records with device arrays; asynchronous on the engine stream, ordered against
        `stream`."""
        with self._ordered(stream):
            check(self._L.jx_batch_aggregate_records_device(self._h, batch_id, n, d_accept_mask, d_segment_index,
                                                            nsegments, d_out_records),
                  self._h, "jx_batch_aggregate_records_device")

    # ------------------------------------------------------------------ leader role
    def leader_initialized_batch(self, nonces, public_shares, leader_input_shares) -> "LeaderInit":
        """prio ping-pong leader_initialized for n reports (aggregation_job_driver.rs:344-362):
        prepare_init with agg_id 0 on the explicit leader input shares. Returns the verdicts
        (0 = initialized, 1 = prepare_init_failure) and the prep shares that go into each
        PingPongMessage::Initialize. The prepare states stay on the device for
        leader_continued_batch."""
        n = int(np.asarray(nonces).reshape(-1, 16).shape[0])
        nn = _u8(nonces, n, 16, "nonces")
        ps = _u8(public_shares, n, self.public_share_len, "public_shares")
        lis = _u8(leader_input_shares, n, self.leader_input_share_len, "leader_input_shares")
        verdicts = np.zeros(max(n, 1), np.uint8)
        shares = np.zeros((max(n, 1), self.prep_share_len), np.uint8)
        bid = ctypes.c_uint64()
        st = self._L.jx_leader_prep_init_batch(self._h, n, _ptr(nn), _ptr(ps) if self.public_share_len else None,
                                               _ptr(lis), _ptr(shares), _ptr(verdicts), ctypes.byref(bid))
        check(st, self._h, "jx_leader_prep_init_batch")
        with self._lock:
            self._leader_n, self._leader_id = n, bid.value
        return LeaderInit(verdicts[:n], shares[:n], bid.value)

    def leader_continued_batch(self, prep_msgs, want_out_shares: bool = False,
                               init: "LeaderInit | None" = None) -> BatchResult:
        """prio ping-pong leader_continued on the helper's Finish{prep_msg} (aggregation_job_driver.rs:
        588-602): prepare_next for the batch of `init` (default: the last leader_initialized_batch).
        Raises EngineError (JX_E_STATE) if that batch was released or already finished."""
        if init is None:  # the last leader batch: callers sharing the engine across threads pass `init`
            with self._lock:
                n, bid = self._leader_n, self._leader_id
        else:
            n, bid = len(init.verdicts), init.batch_id
        msgs = None
        if self.prep_msg_len:
            msgs = _u8(prep_msgs, n, self.prep_msg_len, "prep_msgs") if n else np.zeros((1, self.prep_msg_len), np.uint8)
        verdicts = np.zeros(max(n, 1), np.uint8)
        outs = np.zeros((max(n, 1), self.output_len * self.field_bytes), np.uint8) if want_out_shares else None
        st = self._L.jx_leader_prep_finish_batch(self._h, bid, n, _ptr(msgs), _ptr(verdicts), _ptr(outs))
        check(st, self._h, "jx_leader_prep_finish_batch")
        return BatchResult(verdicts[:n], msgs[:n] if msgs is not None else np.zeros((n, 0), np.uint8),
                           outs[:n] if outs is not None else None, bid)

    def accumulate(self, n: int, accept_mask: np.ndarray | None = None, segments: np.ndarray | None = None,
                   batch_id: int | None = None):
        """Merge the finished output shares of a prepared batch into the engine's running batch
        aggregations and release the batch (at most once per batch). segments[i]: the
        batch-aggregation id (any u32) of report i. batch_id defaults to the last prepared batch,
        which is only meaningful on an engine one thread uses: threads sharing an engine pass it."""
        m = None if accept_mask is None else np.ascontiguousarray(accept_mask, dtype=np.uint8)
        s = None if segments is None else np.ascontiguousarray(segments, dtype=np.uint32)
        bid = self.batch_id() if batch_id is None else batch_id
        check(self._L.jx_accumulate(self._h, bid, n, _ptr(m), _ptr(s)), self._h, "jx_accumulate")

    # ------------------------------------------------------------------ device-pointer paths (inputs in HBM)
    def leader_init_device(self, n: int, d_nonces: int, d_public_shares: int | None, d_leader_input_shares: int,
                           d_out_prep_shares: int, d_out_verdicts: int | None = None, stream=None,
                           lis_stride: int = 0) -> int:
        """leader_initialized for n reports resident in HBM; returns the batch id. Asynchronous,
        ordered against `stream` (module docstring). lis_stride: the row stride of the leader input
        shares (0: packed rows of leader_input_share_len; a multiple of 128 lets the in-place FLP
        kernels read whole cache lines)."""
        bid = ctypes.c_uint64()
        with self._ordered(stream):
            st = self._L.jx_leader_prep_init_device_ex(self._h, n, d_nonces, d_public_shares, d_leader_input_shares,
                                                       lis_stride, d_out_prep_shares, d_out_verdicts, ctypes.byref(bid))
            check(st, self._h, "jx_leader_prep_init_device_ex")
        return bid.value

    def leader_finish_device(self, batch_id: int, n: int, d_prep_msgs: int | None, d_peer_verdicts: int | None = None,
                             d_out_verdicts: int | None = None, stream=None):
        """leader_continued on the helper's prep messages in HBM; reports the helper rejected
        (d_peer_verdicts != 0) fail with helper_step_failure. Asynchronous, ordered against `stream`."""
        with self._ordered(stream):
            check(self._L.jx_leader_prep_finish_device(self._h, batch_id, n, d_prep_msgs, d_peer_verdicts,
                                                       d_out_verdicts),
                  self._h, "jx_leader_prep_finish_device")

    def accumulate_device(self, batch_id: int, n: int, d_accept_mask: int | None = None, d_segments: int | None = None,
                          segment_ids=(0,), stream=None):
        """accumulate with device arrays: d_segments[i] indexes segment_ids. Asynchronous, ordered
        against `stream`."""
        ids, ptr = _seg_table(segment_ids)
        with self._ordered(stream):
            check(self._L.jx_accumulate_device(self._h, batch_id, n, d_accept_mask, d_segments, ptr, ids.size),
                  self._h, "jx_accumulate_device")

    def prep_and_aggregate(self, nonces, public_shares, helper_input_shares, leader_prep_shares,
                           segment: int = 0, want_results: bool = True):
        """Fused prep_init + aggregate of n reports (the benchmark's unit of work), host buffers."""
        n = int(np.asarray(nonces).reshape(-1, 16).shape[0])
        nn = _u8(nonces, n, 16, "nonces")
        ps = _u8(public_shares, n, self.public_share_len, "public_shares")
        his = _u8(helper_input_shares, n, self.helper_input_share_len, "helper_input_shares")
        lps = _u8(leader_prep_shares, n, self.prep_share_len, "leader_prep_shares")
        verdicts = np.zeros(max(n, 1), np.uint8) if want_results else None
        msgs = np.zeros((max(n, 1), self.prep_msg_len), np.uint8) if (want_results and self.prep_msg_len) else None
        st = self._L.jx_helper_prep_aggregate(self._h, n, _ptr(nn), _ptr(ps) if self.public_share_len else None,
                                              _ptr(his), _ptr(lps), segment, _ptr(msgs), _ptr(verdicts))
        check(st, self._h, "jx_helper_prep_aggregate")
        if want_results:
            return verdicts[:n], (msgs[:n] if msgs is not None else np.zeros((n, 0), np.uint8))
        return None

    def prep_and_aggregate_device(self, d_nonces: int, d_public_shares: int | None, d_helper_input_shares: int,
                                  d_leader_prep_shares: int, n: int, segment: int = 0,
                                  d_out_prep_msgs: int | None = None, d_out_verdicts: int | None = None,
                                  d_segments: int | None = None, segment_ids=None, stream=None):
        """Same, with inputs already resident in HBM (device pointers, e.g. tensor.data_ptr()).
        Every report goes to `segment`, or, with d_segments, report i to segment_ids[d_segments[i]].
        Asynchronous, ordered against `stream` (default: torch's current stream), so outputs read on
        that stream need no sync(); with stream=False call sync() (or join_stream) first."""
        ids, ptr = _seg_table([segment] if segment_ids is None else segment_ids)
        with self._ordered(stream):
            st = self._L.jx_helper_prep_aggregate_device(self._h, n, d_nonces, d_public_shares, d_helper_input_shares,
                                                         d_leader_prep_shares, d_segments, ptr, ids.size,
                                                         d_out_prep_msgs, d_out_verdicts)
            check(st, self._h, "jx_helper_prep_aggregate_device")

    # ------------------------------------------------------------------ aggregation state
    def aggregate_share(self, segment: int = 0) -> tuple[bytes, int, bytes]:
        """(encoded aggregate share, report count, checksum) of one batch aggregation."""
        out = np.zeros(self.output_len * self.field_bytes, np.uint8)
        cnt = ctypes.c_uint64()
        check(self._L.jx_aggregate_read(self._h, segment, _ptr(out), ctypes.byref(cnt)), self._h,
              "jx_aggregate_read")
        cs = np.zeros(32, np.uint8)
        check(self._L.jx_aggregate_checksum(self._h, segment, _ptr(cs)), self._h, "jx_aggregate_checksum")
        return out.tobytes(), cnt.value, cs.tobytes()

    def reset_aggregates(self):
        check(self._L.jx_aggregate_reset(self._h), self._h, "jx_aggregate_reset")

    def export_aggregate_device(self, segment: int, d_dst: int, stream=None):
        with self._ordered(stream):
            check(self._L.jx_aggregate_export_device(self._h, segment, d_dst), self._h, "jx_aggregate_export_device")

    def combine_device(self, d_parts: int, nparts: int, d_out: int, stream=None):
        with self._ordered(stream):
            check(self._L.jx_aggregate_combine_device(self._h, d_parts, nparts, d_out), self._h,
                  "jx_aggregate_combine_device")

    def record_bytes(self) -> int:
        b = ctypes.c_uint32()
        check(self._L.jx_shard_record_bytes(self._h, ctypes.byref(b)), self._h, "jx_shard_record_bytes")
        return b.value

    def export_record_device(self, segment: int, d_dst: int, stream=None):
        """Write this engine's shard record (agg share || count || checksum) to device memory."""
        with self._ordered(stream):
            check(self._L.jx_shard_record_export_device(self._h, segment, d_dst), self._h,
                  "jx_shard_record_export_device")

    def combine_records_device(self, d_records: int, nrecords: int, d_out: int, stream=None):
        """Merge nrecords back-to-back shard records on the device (compute_aggregate_share)."""
        with self._ordered(stream):
            check(self._L.jx_shard_record_combine_device(self._h, d_records, nrecords, d_out), self._h,
                  "jx_shard_record_combine_device")

    def set_capacity(self, reports: int):
        check(self._L.jx_engine_set_capacity(self._h, reports), self._h, "jx_engine_set_capacity")

    def sync(self):
        check(self._L.jx_engine_sync(self._h), self._h, "jx_engine_sync")

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(self._L.jx_engine_stream(self._h, ctypes.byref(s)), self._h, "jx_engine_stream")
        return s.value or 0

    # ------------------------------------------------------------------ coalescing and memory
    def coalesce(self, enable: bool = True, window_us: int = 0):
        """Coalesced prepares: helper_initialized_batch / leader_initialized_batch of small jobs join the
        device's next shared launch with the concurrent jobs of every coalescing engine of this Prio3
        instance on the device (each report keeps its own engine's verify key). window_us = 0: automatic."""
        check(self._L.jx_engine_coalesce(self._h, int(bool(enable)), int(window_us)), self._h, "jx_engine_coalesce")

    def memory(self) -> dict:
        """This engine's resident batches and the device arena / coalescer counters (jx_engine_memory)."""
        m = _lib.JxMemoryStats()
        check(self._L.jx_engine_memory(self._h, ctypes.byref(m)), self._h, "jx_engine_memory")
        return {name: int(getattr(m, name)) for name, _ in m._fields_}

    # ------------------------------------------------------------------ instrumentation
    def timing(self, enable: bool):
        check(self._L.jx_engine_timing(self._h, int(enable)), self._h, "jx_engine_timing")

    def timing_read(self) -> dict:
        ms = (ctypes.c_float * 4)()
        ln = (ctypes.c_uint64 * 4)()
        check(self._L.jx_engine_timing_read(self._h, ms, ln), self._h, "jx_engine_timing_read")
        names = ("xof", "flp", "accumulate", "slow")
        return {k: {"ms": float(ms[i]), "launches": int(ln[i])} for i, k in enumerate(names)}

    def debug(self, option: int, value: int):
        check(self._L.jx_engine_debug(self._h, option, value), self._h, "jx_engine_debug")


Prio3Engine = HelperEngine

__all__ = ["HelperEngine", "Prio3Engine", "BatchResult", "EncryptedResult", "LeaderInit", "EngineError",
           "VERDICT_LABELS", "FINISHED", "OPEN_STATUS"]
