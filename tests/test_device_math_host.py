"""The device arithmetic headers (janus_amd/csrc/jx_field.h, jx_keccak.h, jx_sha256.h),
compiled for the host, against Python integers / hashlib / the oracle's Keccak."""
import ctypes
import hashlib
import os
import random
import subprocess

import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
P128 = 2**128 - 28 * 2**64 + 1
P64 = 2**64 - 2**32 + 1
R = 2**128


@pytest.fixture(scope="module")
def ht():
    src = os.path.join(HERE, "csrc", "hosttest.cpp")
    so = os.path.join(HERE, "csrc", "libjx_hosttest.so")
    hdrs = [os.path.join(HERE, "..", "janus_amd", "csrc", h) for h in ("jx_field.h", "jx_keccak.h", "jx_sha256.h",
                                                                         "jx_hpke.h", "jx_sha_aes.h")]
    if not os.path.exists(so) or any(os.path.getmtime(h) > os.path.getmtime(so) for h in hdrs + [src]):
        tmp = f"{so}.{os.getpid()}.tmp"  # atomic: pytest-xdist workers may build concurrently
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", tmp, src], check=True)
        os.replace(tmp, so)
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.ht_f128.argtypes = [ctypes.c_int, vp, vp, vp]
    L.ht_reduce192.argtypes = [vp, vp]
    L.ht_reduce192_small.argtypes = [vp, vp]
    L.ht_wide_dot.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp]
    L.ht_wacc_reduce.argtypes = [vp, vp]
    L.ht_x25519.argtypes = [vp, vp, vp]
    L.ht_fe.argtypes = [ctypes.c_int, vp, vp, vp]
    L.ht_aes128.argtypes = [vp, vp, vp]
    L.ht_ghash_mul.argtypes = [vp, vp, vp]
    L.ht_hmac32.argtypes = [vp, vp, ctypes.c_int, vp]
    L.ht_mont_lazy.argtypes = [vp, vp, vp]
    L.ht_f64.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
    L.ht_f64.restype = ctypes.c_uint64
    L.ht_keccak_p12.argtypes = [vp]
    L.ht_sha256_16.argtypes = [vp, vp]
    L.ht_xof_block.argtypes = [ctypes.c_uint32, ctypes.c_uint32, vp, vp, ctypes.c_int, vp]
    L.ht_aes128_t.argtypes = [ctypes.c_int, vp, vp, vp]
    L.ht_be_word_shift16.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.ht_be_word_shift16.restype = ctypes.c_uint32
    L.ht_wacc64_dot.argtypes = [vp, vp, ctypes.c_int]
    L.ht_wacc64_dot.restype = ctypes.c_uint64
    L.ht_reduce192_p64.argtypes = [vp]
    L.ht_reduce192_p64.restype = ctypes.c_uint64
    return L


def _b(x, n=16):
    return ctypes.create_string_buffer(x.to_bytes(n, "little"), n)


def f128(L, op, a, b=None):
    out = ctypes.create_string_buffer(16)
    L.ht_f128(op, _b(a), _b(b) if b is not None else None, out)
    return int.from_bytes(out.raw, "little")


EDGE = [0, 1, 2, P128 - 1, P128 - 2, 2**127, 2**64, 2**64 - 1, 28 * 2**64 - 1, P128 // 2,
        # all-ones 32-bit limbs: every column sum and REDC add carries (mont128's carry chains)
        0xFFFFFFFFFFFFFFE3FFFFFFFFFFFFFFFF, 0xFFFFFFFFFFFFFFE3FFFFFFFF00000000, 2**96 - 1, 2**32 - 1,
        0xFFFFFFFF00000000FFFFFFFF, 0xFFFFFFFFFFFFFFE300000000FFFFFFFF]


def test_field128_add_sub(ht):
    rnd = random.Random(1)
    vals = EDGE + [rnd.randrange(P128) for _ in range(200)]
    for a in vals[:60]:
        for b in vals[:60]:
            assert f128(ht, 0, a, b) == (a + b) % P128
            assert f128(ht, 1, a, b) == (a - b) % P128


def test_field128_montgomery(ht):
    rnd = random.Random(2)
    rinv = pow(R, P128 - 2, P128)
    vals = EDGE + [rnd.randrange(P128) for _ in range(300)]
    for a in vals[:90]:
        for b in vals[:90]:
            assert f128(ht, 2, a, b) == a * b * rinv % P128
    for a in vals:
        assert f128(ht, 3, a) == a * R % P128
        assert f128(ht, 4, a) == a * rinv % P128


def test_field128_mont_lazy_bound(ht):
    rnd = random.Random(3)
    rinv = pow(R, P128 - 2, P128)
    for _ in range(500):
        a, b = rnd.choice(EDGE + [rnd.randrange(P128)]), rnd.randrange(P128)
        out = (ctypes.c_uint64 * 3)()
        ht.ht_mont_lazy(_b(a), _b(b), out)
        v = out[0] + (out[1] << 64) + (out[2] << 128)
        assert v < 2 * P128 and v % P128 == a * b * rinv % P128


def test_reduce192(ht):
    rnd = random.Random(4)
    cases = [0, 1, P128, 2**192 - 1, 2**128, 2**128 - 1, 64 * 2 * P128] + [rnd.randrange(2**192) for _ in range(500)]
    for v in cases:
        w = (ctypes.c_uint64 * 3)(v & (2**64 - 1), (v >> 64) & (2**64 - 1), v >> 128)
        out = ctypes.create_string_buffer(16)
        ht.ht_reduce192(w, out)
        assert int.from_bytes(out.raw, "little") == v % P128, hex(v)


def test_reduce192_small(ht):
    """The branch-free reduction of the output-share truncation (top word < 2^32)."""
    rnd = random.Random(14)
    cases = [0, 1, P128 - 1, P128, 2**128 - 1, 2**128, 2**160 - 1, 2**128 + 2**64 - 1, (2**32 - 1) << 128,
             ((2**32 - 1) << 128) + 2**128 - 1, ((2**32 - 1) << 128) | 1, P128 * 255, 2**136 - 1]
    cases += [rnd.randrange(2**(128 + rnd.randrange(0, 33))) for _ in range(3000)]
    # tops whose fold carries: w1 close to 2^64
    cases += [(rnd.randrange(1, 2**32) << 128) | ((2**64 - rnd.randrange(1, 2**40)) << 64) | rnd.randrange(2**64)
              for _ in range(500)]
    for v in cases:
        w = (ctypes.c_uint64 * 3)(v & (2**64 - 1), (v >> 64) & (2**64 - 1), v >> 128)
        out = ctypes.create_string_buffer(16)
        ht.ht_reduce192_small(w, out)
        assert int.from_bytes(out.raw, "little") == v % P128, hex(v)


def test_field64(ht):
    rnd = random.Random(5)
    vals = [0, 1, P64 - 1, P64 - 2, 2**32, 2**32 - 1, 2**63] + [rnd.randrange(P64) for _ in range(300)]
    for a in vals[:70]:
        for b in vals[:70]:
            assert ht.ht_f64(0, a, b) == (a + b) % P64
            assert ht.ht_f64(1, a, b) == (a - b) % P64
            assert ht.ht_f64(2, a, b) == a * b % P64


def test_keccak_p12_matches_oracle(ht):
    rnd = random.Random(6)
    for _ in range(10):
        st = [rnd.getrandbits(64) for _ in range(25)]
        arr = (ctypes.c_uint64 * 25)(*st)
        ht.ht_keccak_p12(arr)
        assert list(arr) == O.keccak_p1600(st, 12)


def test_sha256_16(ht):
    for _ in range(20):
        rid = os.urandom(16)
        out = ctypes.create_string_buffer(32)
        ht.ht_sha256_16(rid, out)
        assert out.raw == hashlib.sha256(rid).digest()


@pytest.mark.parametrize("usage,binder", [(1, b"\x01"), (2, b"\x01\x01"), (5, b"\x01" + bytes(range(16))),
                                          (6, bytes(range(32))), (3, b"\x01")])
def test_xof_block_builder(ht, usage, binder):
    """blk_xof_prefix + pad == the oracle's XofTurboShake128 message framing."""
    seed = os.urandom(16)
    for algo in (0, 2, 0xFFFF1003):
        w = (ctypes.c_uint32 * 42)()
        ht.ht_xof_block(algo, usage, seed, binder, len(binder), w)
        dst = bytes([8, 0]) + algo.to_bytes(4, "big") + usage.to_bytes(2, "big")
        msg = bytes([8]) + dst + seed + binder
        blk = bytearray(msg) + b"\x01" + bytes(168 - len(msg) - 1)
        blk[-1] ^= 0x80
        assert b"".join(x.to_bytes(4, "little") for x in w) == bytes(blk)


def test_wacc_reduce_columns(ht):
    """wacc_reduce's straight-line fold on raw column sums: every column up to 2^63 (the kernels' bound:
    <= 5 * 512 limb products < 2^52 per column between normalisations), zeros, and random mixes."""
    rnd = random.Random(11)
    cases = [[0] * 9, [2**63 - 1] * 9, [2**26 - 1] * 8 + [2**63 - 1], [0] * 8 + [2**63 - 1], [1] + [0] * 8,
             [2**63 - 1] + [0] * 8, [0, 0, 0, 0, 0, 2**63 - 1, 0, 0, 0]]
    cases += [[rnd.randrange(2**63) for _ in range(9)] for _ in range(300)]
    cases += [[rnd.choice([0, 2**26 - 1, 2**63 - 1, rnd.randrange(2**63)]) for _ in range(9)] for _ in range(300)]
    for cols in cases:
        out = ctypes.create_string_buffer(16)
        ht.ht_wacc_reduce((ctypes.c_uint64 * 9)(*cols), out)
        assert int.from_bytes(out.raw, "little") == sum(c << (26 * s) for s, c in enumerate(cols)) % P128, cols


@pytest.mark.parametrize("n,norm", [(1, 0), (91, 0), (700, 0), (2000, 512), (5000, 512)])
def test_wide_dot_accumulator(ht, n, norm):
    """The FLP wire sums: sum x_k c_k mod p with 26-bit limbs and deferred reduction,
    including worst-case operands (p - 1) at the term counts the kernel allows."""
    rnd = random.Random(n)
    for trial in range(3):
        if trial == 0:
            xs = [P128 - 1] * n
            cs = [P128 - 1] * n
        else:
            xs = [rnd.randrange(P128) for _ in range(n)]
            cs = [rnd.choice([rnd.randrange(P128), P128 - 1, 2**128 - 2**100]) % P128 for _ in range(n)]
        xb = b"".join(x.to_bytes(16, "little") for x in xs)
        cb = b"".join(c.to_bytes(16, "little") for c in cs)
        out = ctypes.create_string_buffer(16)
        ht.ht_wide_dot(xb, cb, n, norm, out)
        assert int.from_bytes(out.raw, "little") == sum(x * c for x, c in zip(xs, cs)) % P128


# ---------------------------------------------------------------------------- HPKE primitives (jx_hpke.h)
P25519 = 2**255 - 19


def _buf32(x: int) -> bytes:
    return x.to_bytes(32, "little")


def test_fe25519_ops(ht):
    from oracle import hpke_oracle as H  # noqa: F401
    rnd = random.Random(5)
    vals = [0, 1, 2, 19, P25519 - 1, P25519 - 19, 2**254, 2**255 - 20] + [rnd.randrange(P25519) for _ in range(40)]
    out = ctypes.create_string_buffer(32)
    for a in vals:
        for b in vals[:12]:
            for op, want in ((0, a * b), (2, a - b)):
                ht.ht_fe(op, _buf32(a), _buf32(b), out)
                assert int.from_bytes(out.raw, "little") == want % P25519, (op, a, b)
        ht.ht_fe(1, _buf32(a), _buf32(0), out)
        assert int.from_bytes(out.raw, "little") == a * a % P25519
        ht.ht_fe(4, _buf32(a), _buf32(0), out)
        assert int.from_bytes(out.raw, "little") == a * 121665 % P25519
        if a:
            ht.ht_fe(3, _buf32(a), _buf32(0), out)
            assert int.from_bytes(out.raw, "little") == pow(a, P25519 - 2, P25519)


def test_fe25519_reduction_bounds(ht):
    """The product reduction on the loosest inputs the ladder makes (every limb up to 2^28 - 1): the value is the
    product mod p, and the output limbs stay within what fe_sub's 2p needs (limb 0 <= 2^27 - 38, limbs 1..8 <=
    2^27 - 2, limb 9 <= 2^22 - 2) and small enough that a sum or difference of two stays under 2^28."""
    rnd = random.Random(25519)
    L = ctypes.c_uint32 * 10
    ht.ht_fe_limbs.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    top = (1 << 28) - 1
    cases = [[top] * 10, [0] * 10, [1] + [0] * 9] + [[rnd.randrange(1 << 28) for _ in range(10)] for _ in range(300)]
    cases += [[rnd.choice([0, top, 1 << 26, (1 << 26) - 1, 1 << 27]) for _ in range(10)] for _ in range(100)]

    def val(v):
        return sum(x << (26 * i) for i, x in enumerate(v))

    for i, a in enumerate(cases):
        b = cases[(7 * i + 3) % len(cases)]
        for op in (0, 1, 4):
            out = L()
            ht.ht_fe_limbs(op, L(*a), L(*b), out)
            want = val(a) * (val(b) if op == 0 else val(a) if op == 1 else 121665) % P25519
            assert val(out) % P25519 == want, (op, a, b)
            assert out[0] <= (1 << 27) - 38 and all(x <= (1 << 27) - 2 for x in out[1:9]) and out[9] <= (1 << 22) - 2
            assert max(out) < (1 << 26) + (1 << 17), list(out)


def test_x25519_vs_oracle(ht):
    from oracle import hpke_oracle as H
    rnd = random.Random(11)
    out = ctypes.create_string_buffer(32)
    cases = [(bytes.fromhex("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4"),
              bytes.fromhex("e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c"))]
    cases += [(rnd.randbytes(32), rnd.randbytes(32)) for _ in range(6)]
    cases += [(rnd.randbytes(32), (9).to_bytes(32, "little")), (rnd.randbytes(32), bytes(32)),
              (rnd.randbytes(32), b"\xff" * 32)]
    for k, u in cases:
        ht.ht_x25519(k, u, out)
        assert out.raw == H.x25519(k, u)


def test_aes_ghash_hmac_vs_oracle(ht):
    import hashlib
    import hmac as hm

    from oracle import hpke_oracle as H
    rnd = random.Random(3)
    out = ctypes.create_string_buffer(32)
    for _ in range(20):
        key, blk = rnd.randbytes(16), rnd.randbytes(16)
        ht.ht_aes128(key, blk, out)
        assert out.raw[:16] == H.aes128_encrypt_block(H.aes128_expand(key), blk)
        x, h = rnd.randbytes(16), rnd.randbytes(16)
        ht.ht_ghash_mul(x, h, out)
        want = H._ghash_mul(int.from_bytes(x, "big"), int.from_bytes(h, "big")).to_bytes(16, "big")
        assert out.raw[:16] == want
    for n in (0, 1, 23, 51, 55, 56, 63, 64, 92, 95, 119):
        key, msg = rnd.randbytes(32), rnd.randbytes(n)
        ht.ht_hmac32(key, msg, n, out)
        assert out.raw == hm.new(key, msg, hashlib.sha256).digest(), n


# ---- XofHmacSha256Aes128 / Field64 multiproof building blocks (jx_sha_aes.h, jx_field.h)

def test_aes128_ttable_fips197(ht):
    """T-table AES (both key-schedule forms) against the FIPS 197 Appendix C.1 vector and the oracle."""
    from oracle import oracle as O
    key, pt = bytes.fromhex("000102030405060708090a0b0c0d0e0f"), bytes.fromhex("00112233445566778899aabbccddeeff")
    rnd = random.Random(9)
    cases = [(key, pt, bytes.fromhex("69c4e0d86a7b0430d8cdb78070b4c55a"))]
    for _ in range(20):
        k, m = rnd.randbytes(16), rnd.randbytes(16)
        cases.append((k, m, O.aes128_encrypt(k, m)))
    for k, m, want in cases:
        for otf in (0, 1):
            out = ctypes.create_string_buffer(16)
            ht.ht_aes128_t(otf, k, m, out)
            assert out.raw == want, (otf, k.hex())


def test_be_word_shift16(ht):
    rnd = random.Random(3)
    for _ in range(100):
        lo, hi = rnd.getrandbits(32), rnd.getrandbits(32)
        b = lo.to_bytes(4, "little") + hi.to_bytes(4, "little")
        assert ht.ht_be_word_shift16(lo, hi) == int.from_bytes(b[2:6], "big")


@pytest.mark.parametrize("n", [1, 91, 1023, 1024, 1025, 3000])
def test_wacc64_dot(ht, n):
    rnd = random.Random(n)
    edge = [0, 1, P64 - 1, P64 - 2, 2**63, 2**32, 2**32 - 1]
    xs = [rnd.choice(edge) if rnd.random() < 0.3 else rnd.randrange(P64) for _ in range(n)]
    cs = [rnd.choice(edge) if rnd.random() < 0.3 else rnd.randrange(P64) for _ in range(n)]
    if n == 1024:  # worst case for the column bound
        xs, cs = [P64 - 1] * n, [P64 - 1] * n
    ax = (ctypes.c_uint64 * n)(*xs)
    ac = (ctypes.c_uint64 * n)(*cs)
    assert ht.ht_wacc64_dot(ax, ac, n) == sum(x * c for x, c in zip(xs, cs)) % P64


def test_reduce192_p64(ht):
    rnd = random.Random(5)
    for _ in range(200):
        w = [rnd.getrandbits(64) for _ in range(3)]
        if rnd.random() < 0.2:
            w = [2**64 - 1] * 3
        a = (ctypes.c_uint64 * 3)(*w)
        assert ht.ht_reduce192_p64(a) == (w[0] + (w[1] << 64) + (w[2] << 128)) % P64
