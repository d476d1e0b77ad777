"""VDAF instances handled by the engine — mirror of janus_core::vdaf::VdafInstance.

Reference: /root/reference/core/src/vdaf.rs:65-108 (enum) and :203-262 (the prio
constructors `Prio3::new_count(2)`, `new_sum(2, bits)`, `new_sum_vec_multithreaded(2,
bits, length, chunk_length)`, `new_histogram(2, length, chunk_length)`). Sizes follow
VDAF-08 / prio 0.16.1.
"""
from __future__ import annotations

from dataclasses import dataclass

VERIFY_KEY_LENGTH = 16  # core/src/vdaf.rs:16
VERIFY_KEY_LENGTH_HMACSHA256_AES128 = 32  # core/src/vdaf.rs:24

# Prio3 algorithm ids (== taskprov VDAF type codes, messages/src/taskprov.rs:358-363), plus the
# engine's id for Prio3SumVecField64MultiproofHmacSha256Aes128 (core/src/vdaf.rs:173-199, whose
# private-use DST algorithm id is 0xFFFF1003)
PRIO3_COUNT, PRIO3_SUM, PRIO3_SUMVEC, PRIO3_HISTOGRAM = 0, 1, 2, 3
PRIO3_SUMVEC_F64_MULTIPROOF = 4
# Prio3FixedPointBoundedL2VecSum{bitsize, length} (core/src/vdaf.rs:86-91, aggregator.rs:916-932;
# prio's private-use DST algorithm id 0xFFFF0000)
PRIO3_FIXEDPOINT_L2 = 5
FIXEDPOINT_BITSIZES = {"BitSize16": 16, "BitSize32": 32}  # Prio3FixedPointBoundedL2VecSumBitSize


def _next_pow2(v: int) -> int:
    p = 1
    while p < v:
        p <<= 1
    return p


def _isqrt(v: int) -> int:
    import math
    return max(1, math.isqrt(v))


@dataclass(frozen=True)
class Prio3:
    """One Prio3 instance (2 aggregators). XofTurboShake128 and one proof, except
    Prio3SumVecField64MultiproofHmacSha256Aes128 (Field64, num_proofs >= 2, XofHmacSha256Aes128)."""

    algo_id: int
    bits: int = 0
    length: int = 0
    chunk_length: int = 0
    num_proofs: int = 1

    # -- constructors named like VdafInstance variants
    @staticmethod
    def count() -> "Prio3":
        return Prio3(PRIO3_COUNT)

    @staticmethod
    def sum(bits: int) -> "Prio3":
        return Prio3(PRIO3_SUM, bits=bits)

    @staticmethod
    def sum_vec(bits: int, length: int, chunk_length: int) -> "Prio3":
        return Prio3(PRIO3_SUMVEC, bits=bits, length=length, chunk_length=chunk_length)

    @staticmethod
    def histogram(length: int, chunk_length: int) -> "Prio3":
        return Prio3(PRIO3_HISTOGRAM, length=length, chunk_length=chunk_length)

    @staticmethod
    def sum_vec_field64_multiproof_hmacsha256_aes128(proofs: int, bits: int, length: int,
                                                     chunk_length: int) -> "Prio3":
        """new_prio3_sum_vec_field64_multiproof_hmacsha256_aes128 (core/src/vdaf.rs:176-199)."""
        if proofs < 2:
            raise ValueError("Must use at least two proofs with Field64")
        return Prio3(PRIO3_SUMVEC_F64_MULTIPROOF, bits=bits, length=length, chunk_length=chunk_length,
                     num_proofs=proofs)

    @staticmethod
    def fixedpoint_boundedl2_vec_sum(bitsize, length: int) -> "Prio3":
        """Prio3::new_fixedpoint_boundedl2_vec_sum_multithreaded(2, length) with FixedI16<U15>
        (bitsize 16 / "BitSize16") or FixedI32<U31> (32 / "BitSize32"), core/src/vdaf.rs:313-334.
        Measurements are the entries' two's-complement bit patterns; the DP strategy is a
        collection-time step (add_noise_to_agg_share) and not part of preparation."""
        bits = FIXEDPOINT_BITSIZES.get(bitsize, bitsize)
        if bits not in (16, 32):
            raise ValueError("bitsize must be 16 or 32 (BitSize16 / BitSize32)")
        return Prio3(PRIO3_FIXEDPOINT_L2, bits=bits, length=length)

    # -- FixedPointBoundedL2VecSum gadget sizes (prio 0.16.1 FixedPointBoundedL2VecSum::new)
    @property
    def norm_bits(self) -> int:
        return 2 * self.bits - 2 if self.algo_id == PRIO3_FIXEDPOINT_L2 else 0

    @property
    def gadget_chunk(self) -> int:
        return _isqrt(self.meas_len) if self.algo_id == PRIO3_FIXEDPOINT_L2 else self.chunk_length

    @property
    def norm_chunk(self) -> int:
        return _isqrt(self.length)

    @property
    def norm_calls(self) -> int:
        return -(-self.length // self.norm_chunk)

    # -- derived sizes
    @property
    def seed_size(self) -> int:
        return 32 if self.algo_id == PRIO3_SUMVEC_F64_MULTIPROOF else 16

    @property
    def verify_key_len(self) -> int:
        return VERIFY_KEY_LENGTH_HMACSHA256_AES128 if self.algo_id == PRIO3_SUMVEC_F64_MULTIPROOF \
            else VERIFY_KEY_LENGTH

    @property
    def field_bytes(self) -> int:
        return 8 if self.algo_id in (PRIO3_COUNT, PRIO3_SUMVEC_F64_MULTIPROOF) else 16

    @property
    def meas_len(self) -> int:
        return {PRIO3_COUNT: 1, PRIO3_SUM: self.bits, PRIO3_SUMVEC: self.bits * self.length,
                PRIO3_SUMVEC_F64_MULTIPROOF: self.bits * self.length,
                PRIO3_FIXEDPOINT_L2: self.bits * self.length + 2 * self.bits - 2,
                PRIO3_HISTOGRAM: self.length}[self.algo_id]

    @property
    def output_len(self) -> int:
        return 1 if self.algo_id in (PRIO3_COUNT, PRIO3_SUM) else self.length

    @property
    def joint_rand_len(self) -> int:
        return {PRIO3_COUNT: 0, PRIO3_SUM: 1, PRIO3_SUMVEC: 1, PRIO3_SUMVEC_F64_MULTIPROOF: 1,
                PRIO3_HISTOGRAM: 2, PRIO3_FIXEDPOINT_L2: 2}[self.algo_id]

    @property
    def arity(self) -> int:
        """Arity of the first (range-check) gadget."""
        return {PRIO3_COUNT: 2, PRIO3_SUM: 1}.get(self.algo_id, 2 * self.gadget_chunk)

    @property
    def calls(self) -> int:
        if self.algo_id == PRIO3_COUNT:
            return 1
        if self.algo_id == PRIO3_SUM:
            return self.bits
        return -(-self.meas_len // self.gadget_chunk)

    @property
    def P(self) -> int:
        return _next_pow2(1 + self.calls)

    @property
    def proof_len(self) -> int:
        n = self.arity + 2 * (self.P - 1) + 1
        if self.algo_id == PRIO3_FIXEDPOINT_L2:  # + the norm gadget's [seeds || gadget poly]
            n += self.norm_chunk + 2 * (_next_pow2(1 + self.norm_calls) - 1) + 1
        return n

    @property
    def verifier_len(self) -> int:
        n = self.arity + 2
        if self.algo_id == PRIO3_FIXEDPOINT_L2:
            n += self.norm_chunk + 1
        return n

    @property
    def public_share_len(self) -> int:
        return 2 * self.seed_size if self.joint_rand_len else 0

    @property
    def helper_input_share_len(self) -> int:
        return (3 if self.joint_rand_len else 2) * self.seed_size

    @property
    def prep_share_len(self) -> int:
        return self.num_proofs * self.verifier_len * self.field_bytes + (self.seed_size if self.joint_rand_len else 0)

    @property
    def leader_input_share_len(self) -> int:
        return (self.meas_len + self.num_proofs * self.proof_len) * self.field_bytes + \
            (self.seed_size if self.joint_rand_len else 0)

    @property
    def prep_msg_len(self) -> int:
        return self.seed_size if self.joint_rand_len else 0

    def name(self) -> str:
        return {PRIO3_COUNT: "Prio3Count", PRIO3_SUM: f"Prio3Sum{{bits={self.bits}}}",
                PRIO3_SUMVEC: f"Prio3SumVec{{bits={self.bits},length={self.length},chunk_length={self.chunk_length}}}",
                PRIO3_HISTOGRAM: f"Prio3Histogram{{length={self.length},chunk_length={self.chunk_length}}}",
                PRIO3_SUMVEC_F64_MULTIPROOF: "Prio3SumVecField64MultiproofHmacSha256Aes128"
                f"{{proofs={self.num_proofs},bits={self.bits},length={self.length},chunk_length={self.chunk_length}}}",
                PRIO3_FIXEDPOINT_L2: f"Prio3FixedPointBoundedL2VecSum{{bitsize=BitSize{self.bits},length={self.length}}}",
                }[self.algo_id]

    # -- FixedPointBoundedL2VecSum measurement / result codecs (host side; collection is out of scope)
    def encode_fixedpoint(self, values) -> list[int]:
        """f64 entries in [-1, 1) -> FixedI{n}<U{n-1}> bit patterns (round to nearest, like fixed!)."""
        n = self.bits
        out = []
        for v in values:
            q = int(round(float(v) * (1 << (n - 1))))
            if not -(1 << (n - 1)) <= q < (1 << (n - 1)):
                raise ValueError(f"fixed-point entry {v} outside [-1, 1)")
            out.append(q & ((1 << n) - 1))
        return out

    def decode_fixedpoint_result(self, agg_share: bytes, num_measurements: int) -> list[float]:
        """FixedPointBoundedL2VecSum::decode_result on an aggregate (the sum of both aggregators'
        shares): CompatibleFloat::to_float(d, c) = d * 2^(1-n) - c per entry."""
        P = 2**128 - 28 * 2**64 + 1
        vals = [int.from_bytes(agg_share[i:i + 16], "little") % P for i in range(0, len(agg_share), 16)]
        return [x * 2.0 ** (1 - self.bits) - num_measurements for x in vals]
