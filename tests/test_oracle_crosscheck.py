"""C oracle vs the independent pure-Python restatement (oracle/pyref.py), small configs.

Also the semantic invariants Janus's integration tests rely on
(integration_tests/tests/integration/common.rs:298-510): honest reports are accepted and
leader + helper output shares sum to the encoded measurement; tampered leader shares are
rejected with the same verdict by both restatements."""
import random

import pytest

from oracle import oracle as O
from oracle import pyref

CFGS = [
    ("count", O.COUNT, {}, (0, 0, 0)),
    ("sum", O.SUM, dict(bits=5), (5, 0, 0)),
    ("histogram", O.HISTOGRAM, dict(length=7, chunk=3), (0, 7, 3)),
    ("sumvec", O.SUMVEC, dict(bits=3, length=4, chunk=5), (3, 4, 5)),
    ("sumvec_padded", O.SUMVEC, dict(bits=2, length=5, chunk=4), (2, 5, 4)),
]


def _meas(name, rng, kw):
    if name == "count":
        return rng.randrange(2)
    if name == "sum":
        return rng.randrange(1 << kw["bits"])
    if name == "histogram":
        return rng.randrange(kw["length"])
    return [rng.randrange(1 << kw["bits"]) for _ in range(kw["length"])]


@pytest.mark.parametrize("name,algo,kw,args", CFGS, ids=[c[0] for c in CFGS])
def test_c_oracle_equals_pyref(name, algo, kw, args):
    rng = random.Random(hash(name) & 0xFFFF)
    C = O.Prio3Oracle(algo, *args)
    Py = pyref.Prio3(name.replace("_padded", ""), **kw)
    vk = bytes(rng.randrange(256) for _ in range(16))
    for _ in range(3):
        nonce = bytes(rng.randrange(256) for _ in range(16))
        rand = bytes(rng.randrange(256) for _ in range(C.sizes.client_rand))
        m = _meas(name, rng, kw)
        shard = C.shard(m, nonce, rand)
        assert shard == Py.shard(m, nonce, rand)
        ps, lin, hin = shard
        rc, lshare, lout, _ = C.prep_init(vk, 0, nonce, ps, lin)
        _, lshare_py = Py.prep_init(vk, 0, nonce, ps, lin)
        assert rc == 0 and lshare == lshare_py
        got = C.helper_prep(vk, nonce, ps, hin, lshare)
        assert got == Py.helper_prep(vk, nonce, ps, hin, lshare)
        assert got[0] == 0
        # leader + helper output shares == truncate(encode(measurement))
        agg = C.aggregate([lout, got[2]])
        E = C.sizes.field_bytes
        vals = [int.from_bytes(agg[i:i + E], "little") for i in range(0, len(agg), E)]
        assert vals == Py.valid.truncate(Py.valid.encode(m))
        # every single-bit flip of the leader prep share is rejected identically
        for byte in range(0, len(lshare), max(1, len(lshare) // 9)):
            t = bytearray(lshare)
            t[byte] ^= 1 << rng.randrange(8)
            v_c = C.helper_prep(vk, nonce, ps, hin, bytes(t))[0]
            assert v_c == Py.helper_prep(vk, nonce, ps, hin, bytes(t))[0]
            assert v_c in (2, 3, 4)


def test_invalid_measurement_rejected():
    """A client that shards an out-of-range value (bit = 2) fails decide (prepare_message_failure)."""
    C = O.Prio3Oracle(O.SUMVEC, 1, 3, 2)
    Py = pyref.Prio3("sumvec", bits=1, length=3, chunk=2)
    vk, nonce, rand = bytes(16), bytes(range(16)), bytes(range(80))
    # encode [1, 0, 1] -> meas bits; leader adds 1 to element 1 making it 1 -> still valid; add 2 -> invalid
    ps, lin, hin = Py.shard([1, 0, 1], nonce, rand)
    p = Py.F.p
    lmeas = Py.F.decode_vec(lin[:48])
    lmeas[1] = (lmeas[1] + 2) % p
    bad_lin = Py.F.encode_vec(lmeas) + lin[48:]
    # leader recomputes its prep share from the bad share (its joint-rand part changes too)
    _, lshare = Py.prep_init(vk, 0, nonce, ps, bad_lin)
    assert Py.helper_prep(vk, nonce, ps, hin, lshare)[0] in (3, 4)
    assert C.helper_prep(vk, nonce, ps, hin, lshare)[0] == Py.helper_prep(vk, nonce, ps, hin, lshare)[0]


# ---- Prio3SumVecField64MultiproofHmacSha256Aes128 (core/src/vdaf.rs:173-199)

MP_CFGS = [(2, 16, 15, 16), (2, 8, 12, 14), (3, 1, 7, 3), (2, 2, 5, 3)]


def test_xof_hmac_sha256_aes128_c_equals_python():
    """The two restatements of XofHmacSha256Aes128 agree (C: own SHA-256/HMAC/AES; Python:
    hashlib/hmac + the AES of oracle/hpke_oracle.py, itself pinned by RFC 9180's AES-GCM vector),
    including a counter that wraps its low 64 bits (Ctr64BE)."""
    rng = random.Random(4)
    for n in (0, 1, 16, 17, 100, 1000):
        seed, dst, binder = rng.randbytes(32), rng.randbytes(8), rng.randbytes(rng.randrange(40))
        assert O.xof_hmac_aes(seed, dst, binder, n) == pyref.XofHmacSha256Aes128(seed, dst, binder).next(n)
    # Ctr64BE: the low 64 bits of the counter block wrap without carrying into the high half
    x = pyref.XofHmacSha256Aes128(bytes(32), b"d", b"")
    x.ctr = 2**64 - 1
    hi = x.iv_hi
    a = x.next(32)
    assert x.ctr == 1 and x.iv_hi == hi and len(a) == 32


@pytest.mark.parametrize("cfg", MP_CFGS, ids=[f"p{c[0]}_{c[1]}x{c[2]}_{c[3]}" for c in MP_CFGS])
def test_multiproof_c_oracle_equals_pyref(cfg):
    proofs, bits, length, chunk = cfg
    rng = random.Random(sum(cfg))
    C = O.Prio3Oracle(O.SUMVEC_F64_MULTIPROOF, bits, length, chunk, proofs)
    Py = pyref.Prio3("sumvec_f64_multiproof", proofs=proofs, bits=bits, length=length, chunk=chunk)
    assert (C.sizes.seed, C.sizes.verify_key, C.sizes.field_bytes) == (32, 32, 8)
    vk = rng.randbytes(32)
    for _ in range(2):
        nonce = rng.randbytes(16)
        rand = rng.randbytes(C.sizes.client_rand)
        m = [rng.randrange(1 << bits) for _ in range(length)]
        shard = C.shard(m, nonce, rand)
        assert shard == Py.shard(m, nonce, rand)
        ps, lin, hin = shard
        rc, lshare, lout, _ = C.prep_init(vk, 0, nonce, ps, lin)
        assert rc == 0 and lshare == Py.prep_init(vk, 0, nonce, ps, lin)[1]
        got = C.helper_prep(vk, nonce, ps, hin, lshare)
        assert got == Py.helper_prep(vk, nonce, ps, hin, lshare) and got[0] == 0
        agg = C.aggregate([lout, got[2]])
        assert [int.from_bytes(agg[i:i + 8], "little") for i in range(0, len(agg), 8)] == m
        for byte in range(0, len(lshare), max(1, len(lshare) // 7)):
            t = bytearray(lshare)
            t[byte] ^= 1 << rng.randrange(8)
            v = C.helper_prep(vk, nonce, ps, hin, bytes(t))[0]
            assert v == Py.helper_prep(vk, nonce, ps, hin, bytes(t))[0] and v in (2, 3, 4)


def test_multiproof_rejects_single_proof():
    with pytest.raises(ValueError):
        O.Prio3Oracle(O.SUMVEC_F64_MULTIPROOF, 8, 12, 14, 1)


# ---- Prio3FixedPointBoundedL2VecSum (core/src/vdaf.rs:86-91; aggregator.rs:916-932)

FP_CFGS = [(16, 3), (32, 3), (16, 10), (16, 5)]


def _fx(v: float, bits: int) -> int:
    """FixedI{bits}<U{bits-1}> bit pattern of v in [-1, 1) (two's complement, as u{bits})."""
    return int(round(v * (1 << (bits - 1)))) & ((1 << bits) - 1)


def _decode_fp(vals, bits, num_measurements):
    """prio CompatibleFloat::to_float (fixedpoint_l2/compatible_float.rs): f * 2^(1-n) - c."""
    return [x * 2.0 ** (1 - bits) - num_measurements for x in vals]


@pytest.mark.parametrize("cfg", FP_CFGS, ids=[f"fp{c[0]}_len{c[1]}" for c in FP_CFGS])
def test_fixedpoint_c_oracle_equals_pyref(cfg):
    bits, length = cfg
    rng = random.Random(bits * 100 + length)
    C = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, length, 0)
    Py = pyref.Prio3("fixedpoint", bits=bits, length=length)
    s = C.sizes
    assert (s.meas_len, s.output_len, s.joint_rand_len, s.proof_len, s.verifier_len) == \
        (Py.valid.MEAS_LEN, length, 2, Py.valid.PROOF_LEN, Py.valid.VERIFIER_LEN)
    vk = rng.randbytes(16)
    for trial in range(3):
        nonce, rand = rng.randbytes(16), rng.randbytes(s.client_rand)
        lim = 1.0 / (2 * length)
        m = [_fx(rng.uniform(-lim, lim), bits) for _ in range(length)]
        shard = C.shard(m, nonce, rand)
        assert shard == Py.shard(m, nonce, rand)
        ps, lin, hin = shard
        rc, lshare, lout, _ = C.prep_init(vk, 0, nonce, ps, lin)
        assert rc == 0 and lshare == Py.prep_init(vk, 0, nonce, ps, lin)[1]
        got = C.helper_prep(vk, nonce, ps, hin, lshare)
        assert got == Py.helper_prep(vk, nonce, ps, hin, lshare) and got[0] == 0
        agg = C.aggregate([lout, got[2]])
        vals = [int.from_bytes(agg[i:i + 16], "little") for i in range(0, len(agg), 16)]
        assert vals == [(x ^ (1 << (bits - 1))) for x in m]  # the offset encodings of the entries
        for byte in range(0, len(lshare), max(1, len(lshare) // 7)):
            t = bytearray(lshare)
            t[byte] ^= 1 << rng.randrange(8)
            v = C.helper_prep(vk, nonce, ps, hin, bytes(t))[0]
            assert v == Py.helper_prep(vk, nonce, ps, hin, bytes(t))[0] and v in (2, 3, 4)


@pytest.mark.parametrize("bits", [16, 32])
def test_fixedpoint_norm_violation_rejected(bits):
    """A vector of squared norm >= 1 cannot be encoded honestly (prio refuses); a client that
    claims the low 2n-2 bits of its norm is rejected by the norm check (prepare_message_failure)."""
    length = 4
    C = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, length, 0)
    Py = pyref.Prio3("fixedpoint", bits=bits, length=length)
    vk, nonce, rand = bytes(range(16)), bytes(16), bytes(range(80))
    for m in ([_fx(0.75, bits)] * length, [_fx(-1.0, bits)] + [0] * (length - 1)):
        ps, lin, hin = C.shard(m, nonce, rand)
        rc, lshare, _, _ = C.prep_init(vk, 0, nonce, ps, lin)
        assert rc == 0
        v = C.helper_prep(vk, nonce, ps, hin, lshare)[0]
        assert v == 3 == Py.helper_prep(vk, nonce, ps, hin, lshare)[0]
    # the largest honest vector: squared norm just below 1
    m = [_fx(0.49, bits)] * length
    ps, lin, hin = C.shard(m, nonce, rand)
    assert C.helper_prep(vk, nonce, ps, hin, C.prep_init(vk, 0, nonce, ps, lin)[1])[0] == 0


@pytest.mark.parametrize("bits", [16, 32])
def test_fixedpoint_reference_e2e_vectors(bits):
    """The reference's own end-to-end expectation (interop_binaries/tests/end_to_end.rs:689-765,
    e2e_prio3_fixed16vec / e2e_prio3_fixed32vec): these four measurements aggregate and decode
    to [0.5, 0.5, 0.6875]; collector/src/lib.rs:1141-1213 decodes one [1/16, 1/8, 1/4]."""
    q, e, s = 0.25, 0.125, 0.0625
    meas = [[q, e, e], [s, e, s], [e, e, q], [s, e, q]]
    C = O.Prio3Oracle(O.FIXEDPOINT_L2, bits, 3, 0)
    vk = bytes(range(16))
    outs = []
    for i, m in enumerate(meas):
        nonce, rand = bytes([i]) * 16, bytes([i + 7]) * 80
        ps, lin, hin = C.shard([_fx(v, bits) for v in m], nonce, rand)
        rc, lshare, lout, _ = C.prep_init(vk, 0, nonce, ps, lin)
        v, _, hout = C.helper_prep(vk, nonce, ps, hin, lshare)
        assert rc == 0 and v == 0
        outs += [lout, hout]
    agg = C.aggregate(outs)
    vals = [int.from_bytes(agg[i:i + 16], "little") for i in range(0, len(agg), 16)]
    assert _decode_fp(vals, bits, len(meas)) == [0.5, 0.5, 0.6875]
    # collector/src/lib.rs:1141-1213: a single measurement decodes to itself
    nonce, rand = bytes(16), bytes(80)
    ps, lin, hin = C.shard([_fx(v, bits) for v in (s, e, q)], nonce, rand)
    _, lshare, lout, _ = C.prep_init(vk, 0, nonce, ps, lin)
    hout = C.helper_prep(vk, nonce, ps, hin, lshare)[2]
    agg = C.aggregate([lout, hout])
    vals = [int.from_bytes(agg[i:i + 16], "little") for i in range(0, len(agg), 16)]
    assert _decode_fp(vals, bits, 1) == [0.0625, 0.125, 0.25]
