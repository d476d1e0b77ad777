"""DAP message codecs on the hot path (subset of /root/reference/messages/src/lib.rs).

Only what the helper's aggregate-init loop touches: PingPongMessage (prio's
topology::ping_pong framing, KATs at messages/src/lib.rs:4232-4240, 4289-4297,
4321-4333), PrepareInit (:2114-2228), PrepareResp / PrepareStepResult / PrepareError
(:2237-2349). Encodings are big-endian length-prefixed as in the DAP codec.
"""
from __future__ import annotations

import enum
import struct
from dataclasses import dataclass


class CodecError(ValueError):
    pass


class _Reader:
    def __init__(self, b: bytes):
        self.b, self.i = memoryview(b), 0

    def take(self, n: int) -> bytes:
        if self.i + n > len(self.b):
            raise CodecError("short read")
        v = bytes(self.b[self.i:self.i + n])
        self.i += n
        return v

    def u8(self) -> int:
        return self.take(1)[0]

    def u16(self) -> int:
        return struct.unpack(">H", self.take(2))[0]

    def u32(self) -> int:
        return struct.unpack(">I", self.take(4))[0]

    def u64(self) -> int:
        return struct.unpack(">Q", self.take(8))[0]

    def opaque16(self) -> bytes:
        return self.take(self.u16())

    def opaque32(self) -> bytes:
        return self.take(self.u32())

    def done(self):
        if self.i != len(self.b):
            raise CodecError("trailing bytes")


def _o16(b: bytes) -> bytes:
    return struct.pack(">H", len(b)) + b


def _o32(b: bytes) -> bytes:
    return struct.pack(">I", len(b)) + b


# ----------------------------------------------------------------------------- PingPongMessage


@dataclass(frozen=True)
class PingPongMessage:
    """Initialize{prep_share} (0), Continue{prep_msg, prep_share} (1), Finish{prep_msg} (2)."""

    kind: int
    prep_msg: bytes = b""
    prep_share: bytes = b""

    INITIALIZE, CONTINUE, FINISH = 0, 1, 2

    @classmethod
    def initialize(cls, prep_share: bytes) -> "PingPongMessage":
        return cls(cls.INITIALIZE, prep_share=prep_share)

    @classmethod
    def finish(cls, prep_msg: bytes) -> "PingPongMessage":
        return cls(cls.FINISH, prep_msg=prep_msg)

    def encode(self) -> bytes:
        if self.kind == self.INITIALIZE:
            return b"\x00" + _o32(self.prep_share)
        if self.kind == self.CONTINUE:
            return b"\x01" + _o32(self.prep_msg) + _o32(self.prep_share)
        return b"\x02" + _o32(self.prep_msg)

    @classmethod
    def decode(cls, b: bytes) -> "PingPongMessage":
        r = _Reader(b)
        k = r.u8()
        if k == 0:
            m = cls(0, prep_share=r.opaque32())
        elif k == 1:
            pm = r.opaque32()
            m = cls(1, prep_msg=pm, prep_share=r.opaque32())
        elif k == 2:
            m = cls(2, prep_msg=r.opaque32())
        else:
            raise CodecError("unexpected PingPongMessage type")
        r.done()
        return m


# ----------------------------------------------------------------------------- Prepare*


class PrepareError(enum.IntEnum):  # messages/src/lib.rs:2338-2349
    BatchCollected = 0
    ReportReplayed = 1
    ReportDropped = 2
    HpkeUnknownConfigId = 3
    HpkeDecryptError = 4
    VdafPrepError = 5
    BatchSaturated = 6
    TaskExpired = 7
    InvalidMessage = 8
    ReportTooEarly = 9


@dataclass(frozen=True)
class ReportMetadata:
    report_id: bytes
    time: int

    def encode(self) -> bytes:
        return self.report_id + struct.pack(">Q", self.time)


@dataclass(frozen=True)
class HpkeCiphertext:
    config_id: int
    encapsulated_key: bytes
    payload: bytes

    def encode(self) -> bytes:
        return bytes([self.config_id]) + _o16(self.encapsulated_key) + _o32(self.payload)


@dataclass(frozen=True)
class ReportShare:
    metadata: ReportMetadata
    public_share: bytes
    encrypted_input_share: HpkeCiphertext

    def encode(self) -> bytes:
        return self.metadata.encode() + _o32(self.public_share) + self.encrypted_input_share.encode()

    @classmethod
    def decode_from(cls, r: _Reader) -> "ReportShare":
        md = ReportMetadata(r.take(16), r.u64())
        ps = r.opaque32()
        cfg = r.u8()
        enc = r.opaque16()
        payload = r.opaque32()
        return cls(md, ps, HpkeCiphertext(cfg, enc, payload))


@dataclass(frozen=True)
class PrepareInit:
    report_share: ReportShare
    message: PingPongMessage

    def encode(self) -> bytes:
        return self.report_share.encode() + _o32(self.message.encode())

    @classmethod
    def decode(cls, b: bytes) -> "PrepareInit":
        r = _Reader(b)
        rs = ReportShare.decode_from(r)
        msg = PingPongMessage.decode(r.opaque32())
        r.done()
        return cls(rs, msg)


@dataclass(frozen=True)
class PrepareStepResult:
    """Continue{message} (0), Finished (1), Reject(PrepareError) (2)."""

    kind: int
    message: PingPongMessage | None = None
    error: PrepareError | None = None

    def encode(self) -> bytes:
        if self.kind == 0:
            return b"\x00" + _o32(self.message.encode())
        if self.kind == 1:
            return b"\x01"
        return b"\x02" + bytes([int(self.error)])


@dataclass(frozen=True)
class PrepareResp:
    report_id: bytes
    result: PrepareStepResult

    def encode(self) -> bytes:
        return self.report_id + self.result.encode()

    @classmethod
    def decode(cls, b: bytes) -> "PrepareResp":
        r = _Reader(b)
        rid = r.take(16)
        k = r.u8()
        if k == 0:
            res = PrepareStepResult(0, message=PingPongMessage.decode(r.opaque32()))
        elif k == 1:
            res = PrepareStepResult(1)
        elif k == 2:
            res = PrepareStepResult(2, error=PrepareError(r.u8()))
        else:
            raise CodecError("unexpected PrepareStepResult")
        r.done()
        return cls(rid, res)


# ----------------------------------------------------------------------------- PlaintextInputShare

EXTENSION_TBD, EXTENSION_TASKPROV = 0x0000, 0xFF00  # messages/src/lib.rs:924-927


@dataclass(frozen=True)
class Extension:
    extension_type: int
    extension_data: bytes = b""

    def encode(self) -> bytes:
        return struct.pack(">H", self.extension_type) + _o16(self.extension_data)


@dataclass(frozen=True)
class PlaintextInputShare:
    """extensions (u16-length-prefixed list) || payload (u32-length-prefixed), the HPKE plaintext
    of a report share (messages/src/lib.rs:1323-1326)."""

    extensions: tuple = ()
    payload: bytes = b""

    def encode(self) -> bytes:
        ext = b"".join(e.encode() for e in self.extensions)
        return _o16(ext) + _o32(self.payload)

    @classmethod
    def decode(cls, b: bytes) -> "PlaintextInputShare":
        r = _Reader(b)
        er = _Reader(r.opaque16())
        exts = []
        while er.i < len(er.b):
            t = er.u16()
            if t not in (EXTENSION_TBD, EXTENSION_TASKPROV):
                raise CodecError("unknown extension type")
            exts.append(Extension(t, er.opaque16()))
        payload = r.opaque32()
        r.done()
        return cls(tuple(exts), payload)
