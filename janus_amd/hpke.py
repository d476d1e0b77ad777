"""Batched HPKE open of report shares on the GPU (wrapper of include/jx_hpke.h).

Mirror of janus_core::hpke::open (core/src/hpke.rs:200-230) as the helper calls it once per
report in its aggregate-init loop (aggregator/src/aggregator.rs:1772-1832): RFC 9180 base
mode with DHKEM(X25519, HKDF-SHA256) / HKDF-SHA256 / AES-128-GCM, application info
HpkeApplicationInfo::new(&Label::InputShare, &Role::Client, &Role::Helper) (core/src/hpke.rs:
69-84), associated data the encoded InputShareAad (messages/src/lib.rs:1854-1858). Here the
whole request's ciphertexts are opened in one launch. There is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import EngineError

# Role (messages/src/lib.rs:512-517) and Label (core/src/hpke.rs:56-66)
ROLE_COLLECTOR, ROLE_CLIENT, ROLE_LEADER, ROLE_HELPER = 0, 1, 2, 3
LABEL_INPUT_SHARE = b"dap-09 input share"
LABEL_AGGREGATE_SHARE = b"dap-09 aggregate share"

EXPORTED_SYMBOLS = ("jx_hpke_create", "jx_hpke_destroy", "jx_hpke_open_batch", "jx_hpke_open_batch_device",
                    "jx_hpke_last_error")


def application_info(label: bytes = LABEL_INPUT_SHARE, sender: int = ROLE_CLIENT, recipient: int = ROLE_HELPER) -> bytes:
    """HpkeApplicationInfo::new (core/src/hpke.rs:74-84)."""
    return label + bytes([sender, recipient])


def input_share_aad(task_id: bytes, report_id: bytes, time: int, public_share: bytes) -> bytes:
    """InputShareAad encoding: task_id || ReportMetadata(id, time) || u32-prefixed public share
    (messages/src/lib.rs:1854-1858)."""
    if len(task_id) != 32 or len(report_id) != 16:
        raise ValueError("task id is 32 bytes, report id 16")
    return task_id + report_id + time.to_bytes(8, "big") + len(public_share).to_bytes(4, "big") + public_share


def _declare(L):
    if getattr(L, "_jx_hpke_declared", False):
        return L
    vp, u64, i32, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint32
    L.jx_hpke_create.restype = i32
    L.jx_hpke_create.argtypes = [vp, vp, vp, u32, i32, ctypes.POINTER(vp)]
    L.jx_hpke_destroy.restype = None
    L.jx_hpke_destroy.argtypes = [vp]
    L.jx_hpke_open_batch.restype = i32
    L.jx_hpke_open_batch.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp, vp]
    L.jx_hpke_open_batch_device.restype = i32
    L.jx_hpke_open_batch_device.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp, vp]
    L.jx_hpke_last_error.restype = ctypes.c_char_p
    L.jx_hpke_last_error.argtypes = [vp]
    L._jx_hpke_declared = True
    return L


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class HpkeOpener:
    """One recipient key pair + application info on one GPU."""

    def __init__(self, private_key: bytes, public_key: bytes, info: bytes, device: int = 0):
        if len(private_key) != 32 or len(public_key) != 32:
            raise ValueError("X25519 keys are 32 bytes")
        self._L = _declare(_lib.load())
        h = ctypes.c_void_p()
        sk = np.frombuffer(private_key, np.uint8).copy()
        pk = np.frombuffer(public_key, np.uint8).copy()
        inf = np.frombuffer(info, np.uint8).copy() if info else np.zeros(1, np.uint8)
        st = self._L.jx_hpke_create(_p(sk), _p(pk), _p(inf), len(info), device, ctypes.byref(h))
        if st != 0:
            raise EngineError(f"jx_hpke_create: status {st}")
        self._h = h

    @property
    def handle(self):
        """The jx_hpke context (for jx_helper_prep_encrypted_batch)."""
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            self._L.jx_hpke_destroy(self._h)
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

    def open_batch(self, encs: list[bytes], ciphertexts: list[bytes], aads: list[bytes]) -> list[bytes | None]:
        """Open n HPKE ciphertexts; None where opening fails (PrepareError::HpkeDecryptError)."""
        n = len(encs)
        if not (len(ciphertexts) == len(aads) == n):
            raise ValueError("one enc, ciphertext and aad per report")
        if n == 0:
            return []
        # a malformed share fails alone (HpkeDecryptError for that report, aggregator.rs:1772-1831):
        # a wrong-length encapsulated key or a ciphertext shorter than the GCM tag never reaches the GPU
        idx = [i for i in range(n) if len(encs[i]) == 32 and len(ciphertexts[i]) >= 16]
        out: list[bytes | None] = [None] * n
        if not idx:
            return out
        enc = np.frombuffer(b"".join(encs[i] for i in idx), np.uint8).copy()
        cts = np.frombuffer(b"".join(ciphertexts[i] for i in idx) or b"\0", np.uint8).copy()
        aad = np.frombuffer(b"".join(aads[i] for i in idx) or b"\0", np.uint8).copy()
        co = np.zeros(len(idx) + 1, np.uint64)
        ao = np.zeros(len(idx) + 1, np.uint64)
        co[1:] = np.cumsum([len(ciphertexts[i]) for i in idx])
        ao[1:] = np.cumsum([len(aads[i]) for i in idx])
        pts = np.zeros(max(1, int(co[-1]) - 16 * len(idx)), np.uint8)
        ok = np.zeros(len(idx), np.uint8)
        st = self._L.jx_hpke_open_batch(self._h, len(idx), _p(enc), _p(cts), _p(co), _p(aad), _p(ao), _p(pts), _p(ok))
        if st != 0:
            raise EngineError(f"jx_hpke_open_batch: status {st} {self._L.jx_hpke_last_error(self._h).decode()}")
        for j, i in enumerate(idx):
            if ok[j]:
                a = int(co[j]) - 16 * j
                out[i] = pts[a:a + len(ciphertexts[i]) - 16].tobytes()
        return out
