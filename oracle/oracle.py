"""TEST INFRASTRUCTURE ONLY — ctypes view of the C Prio3 restatement (prio3_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline. The product path
(janus_amd) never imports it. Parity vs prio 0.16.1 is UNPINNED (see
prio3_oracle.h and DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libprio3_oracle.so")
_lib = None

COUNT, SUM, SUMVEC, HISTOGRAM = 0, 1, 2, 3
# Prio3SumVecField64MultiproofHmacSha256Aes128 (core/src/vdaf.rs:173-199)
SUMVEC_F64_MULTIPROOF = 4
# Prio3FixedPointBoundedL2VecSum{bitsize, length} (core/src/vdaf.rs:86-91; bits = 16 or 32)
FIXEDPOINT_L2 = 5
NSIZES = 21
VERDICT_NAMES = {
    0: "finished",
    1: "prepare_init_failure",
    2: "leader_prep_share_decode_failure",
    3: "prepare_message_failure",
    4: "prepare_next_failure",
}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        L.jo_sizes.argtypes = [ctypes.c_int] * 5 + [u8p]
        i5 = [ctypes.c_int] * 5
        sz, u64 = ctypes.c_size_t, ctypes.c_uint64
        L.jo_shard.argtypes = i5 + [u8p] * 6
        L.jo_prep_init.argtypes = i5 + [u8p, ctypes.c_int] + [u8p] * 6
        L.jo_prep_shares_to_prep.argtypes = i5 + [u8p, sz, u8p, sz, u8p]
        L.jo_helper_prep.argtypes = i5 + [u8p] * 5 + [sz, u8p, u8p]
        L.jo_helper_prep_batch.argtypes = i5 + [u8p, u64] + [u8p] * 10 + [ctypes.c_int]
        L.jo_client_leader_batch.argtypes = i5 + [u8p, u64] + [u8p] * 7 + [ctypes.c_int]
        L.jo_aggregate.argtypes = i5 + [u64, u8p, u8p]
        for name in ("jo_shard", "jo_prep_init", "jo_prep_shares_to_prep", "jo_helper_prep",
                     "jo_helper_prep_batch", "jo_client_leader_batch", "jo_aggregate"):
            getattr(L, name).restype = ctypes.c_int
        L.jo_turboshake128.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint8, u8p, ctypes.c_size_t]
        L.jo_xof_expand.argtypes = [u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        L.jo_xof_hmac_aes.argtypes = [u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        L.jo_aes128_encrypt.argtypes = [u8p, u8p, u8p]
        L.jo_keccak_p1600.argtypes = [u8p, ctypes.c_int]
        L.jo_field_op.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p, u8p]
        L.jo_sha256.argtypes = [u8p, ctypes.c_size_t, u8p]
        _lib = L
    return _lib


def _buf(b: bytes | bytearray | np.ndarray | None):
    if b is None:
        return None
    if isinstance(b, np.ndarray):
        return b.ctypes.data_as(ctypes.c_void_p)
    if isinstance(b, bytearray):
        return ctypes.cast((ctypes.c_char * len(b)).from_buffer(b), ctypes.c_void_p)
    return ctypes.cast(ctypes.c_char_p(bytes(b)), ctypes.c_void_p)


def turboshake128(msg: bytes, D: int, outlen: int) -> bytes:
    out = bytearray(outlen)
    lib().jo_turboshake128(_buf(msg), len(msg), D, _buf(out), outlen)
    return bytes(out)


def keccak_p1600(state: list[int], rounds: int) -> list[int]:
    a = np.array(state, dtype=np.uint64)
    lib().jo_keccak_p1600(_buf(a), rounds)
    return [int(x) for x in a]


def xof_expand(seed: bytes, dst: bytes, binder: bytes, outlen: int) -> bytes:
    out = bytearray(outlen)
    lib().jo_xof_expand(_buf(seed), _buf(dst), len(dst), _buf(binder), len(binder), _buf(out), outlen)
    return bytes(out)


def xof_hmac_aes(seed: bytes, dst: bytes, binder: bytes, outlen: int) -> bytes:
    out = bytearray(outlen)
    lib().jo_xof_hmac_aes(_buf(seed), _buf(dst), len(dst), _buf(binder), len(binder), _buf(out), outlen)
    return bytes(out)


def aes128_encrypt(key: bytes, block: bytes) -> bytes:
    out = bytearray(16)
    lib().jo_aes128_encrypt(_buf(key), _buf(block), _buf(out))
    return bytes(out)


def sha256(msg: bytes) -> bytes:
    out = bytearray(32)
    lib().jo_sha256(_buf(msg), len(msg), _buf(out))
    return bytes(out)


def field_op(field64: bool, op: int, a: int | None, b: int | None = None) -> int:
    enc = 8 if field64 else 16
    ab = a.to_bytes(enc, "little") if a is not None else None
    if op == 4:
        ab = bytes([a]) + bytes(enc - 1)
    bb = b.to_bytes(enc, "little") if b is not None else None
    out = bytearray(enc)
    rc = lib().jo_field_op(int(field64), op, _buf(ab), _buf(bb), _buf(out))
    if rc:
        raise ValueError("field decode failure")
    return int.from_bytes(out, "little")


@dataclass
class Sizes:
    meas_len: int
    output_len: int
    joint_rand_len: int
    proof_len: int
    verifier_len: int
    public_share: int
    leader_input_share: int
    helper_input_share: int
    prep_share: int
    prep_msg: int
    field_bytes: int
    client_rand: int
    arity: int
    calls: int
    P: int
    seed: int
    verify_key: int
    chunk: int          # first gadget's chunk length
    arity1: int         # second gadget (FixedPoint norm): arity, calls, P; 0 if none
    calls1: int
    P1: int


class Prio3Oracle:
    """CPU restatement of one Prio3 instance (the `vdaf` object of core/src/vdaf.rs:203-262)."""

    def __init__(self, algo: int, bits: int = 0, length: int = 0, chunk: int = 0, proofs: int = 1):
        self.params = (algo, bits, length, chunk, proofs)
        out = (ctypes.c_uint32 * NSIZES)()
        if lib().jo_sizes(*self.params, ctypes.cast(out, ctypes.c_void_p)) != 0:
            raise ValueError(f"bad Prio3 params {self.params}")
        self.sizes = Sizes(*list(out))
        self.algo = algo

    @property
    def meas_stride(self) -> int:
        return self.params[2] if self.algo in (SUMVEC, SUMVEC_F64_MULTIPROOF, FIXEDPOINT_L2) else 1

    def shard(self, measurement, nonce: bytes, rand: bytes):
        s = self.sizes
        m = np.asarray(measurement if isinstance(measurement, (list, tuple, np.ndarray)) else [measurement],
                       dtype=np.uint64)
        ps, lin, hin = bytearray(s.public_share), bytearray(s.leader_input_share), bytearray(s.helper_input_share)
        rc = lib().jo_shard(*self.params, _buf(m), _buf(nonce), _buf(rand), _buf(ps), _buf(lin), _buf(hin))
        assert rc == 0
        return bytes(ps), bytes(lin), bytes(hin)

    def prep_init(self, vk: bytes, agg_id: int, nonce: bytes, public_share: bytes, input_share: bytes):
        s = self.sizes
        prep_share, out, corr = bytearray(s.prep_share), bytearray(s.output_len * s.field_bytes), bytearray(s.seed)
        rc = lib().jo_prep_init(*self.params, _buf(vk), agg_id, _buf(nonce), _buf(public_share),
                                _buf(input_share), _buf(prep_share), _buf(out), _buf(corr))
        return rc, bytes(prep_share), bytes(out), bytes(corr)

    def prep_shares_to_prep(self, leader_share: bytes, helper_share: bytes):
        msg = bytearray(self.sizes.seed)
        rc = lib().jo_prep_shares_to_prep(*self.params, _buf(leader_share), len(leader_share),
                                          _buf(helper_share), len(helper_share), _buf(msg))
        return rc, bytes(msg[: self.sizes.prep_msg])

    def helper_prep(self, vk: bytes, nonce: bytes, public_share: bytes, helper_input_share: bytes,
                    leader_prep_share: bytes):
        s = self.sizes
        msg, out = bytearray(s.seed), bytearray(s.output_len * s.field_bytes)
        v = lib().jo_helper_prep(*self.params, _buf(vk), _buf(nonce), _buf(public_share),
                                 _buf(helper_input_share), _buf(leader_prep_share), len(leader_prep_share),
                                 _buf(msg), _buf(out))
        return v, bytes(msg[: s.prep_msg]), bytes(out) if v == 0 else None

    def helper_prep_batch(self, vk, nonces, public_shares, helper_input_shares, leader_prep_shares,
                          nthreads: int = 1, want_out_shares: bool = False):
        """Arrays are uint8 numpy arrays of shape (n, size). Returns dict."""
        s = self.sizes
        n = nonces.shape[0]
        msgs = np.zeros((n, max(s.prep_msg, 1)), np.uint8)
        verdicts = np.zeros(n, np.uint8)
        outs = np.zeros((n, s.output_len * s.field_bytes), np.uint8) if want_out_shares else None
        agg = np.zeros(s.output_len * s.field_bytes, np.uint8)
        count = ctypes.c_uint64(0)
        cs = np.zeros(32, np.uint8)
        ps = public_shares if s.public_share else np.zeros((n, 1), np.uint8)
        rc = lib().jo_helper_prep_batch(*self.params, _buf(vk), ctypes.c_uint64(n), _buf(np.ascontiguousarray(nonces)),
                                        _buf(np.ascontiguousarray(ps)),
                                        _buf(np.ascontiguousarray(helper_input_shares)),
                                        _buf(np.ascontiguousarray(leader_prep_shares)),
                                        _buf(msgs) if s.prep_msg else None, _buf(verdicts), _buf(outs), _buf(agg),
                                        ctypes.byref(count), _buf(cs), nthreads)
        assert rc == 0
        return {"verdicts": verdicts, "prep_msgs": msgs[:, : s.prep_msg], "out_shares": outs,
                "agg": agg.tobytes(), "count": count.value, "checksum": cs.tobytes()}

    def client_leader_batch(self, vk, measurements, nonces, rands, nthreads: int = 1, want_leader_out=False):
        s = self.sizes
        n = nonces.shape[0]
        ps = np.zeros((n, max(s.public_share, 1)), np.uint8)
        his = np.zeros((n, s.helper_input_share), np.uint8)
        lps = np.zeros((n, s.prep_share), np.uint8)
        lout = np.zeros((n, s.output_len * s.field_bytes), np.uint8) if want_leader_out else None
        m = np.ascontiguousarray(measurements, dtype=np.uint64)
        rc = lib().jo_client_leader_batch(*self.params, _buf(vk), ctypes.c_uint64(n), _buf(m),
                                          _buf(np.ascontiguousarray(nonces)), _buf(np.ascontiguousarray(rands)),
                                          _buf(ps), _buf(his), _buf(lps), _buf(lout), nthreads)
        assert rc == 0
        return ps[:, : s.public_share], his, lps, lout

    def aggregate(self, out_shares: list[bytes]) -> bytes:
        s = self.sizes
        arr = np.frombuffer(b"".join(out_shares), np.uint8) if out_shares else np.zeros(1, np.uint8)
        agg = bytearray(s.output_len * s.field_bytes)
        rc = lib().jo_aggregate(*self.params, ctypes.c_uint64(len(out_shares)), _buf(arr), _buf(agg))
        assert rc == 0
        return bytes(agg)
