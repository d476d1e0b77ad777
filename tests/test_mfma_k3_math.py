"""Host replay of the matrix-core wire sums (flp_psum_mfma_kernel) with Python integers.

The kernel was built, parity-tested on MI355X and measured slower than the VALU ring (git 3299f0a); it is not
in the library. This test keeps its arithmetic pinned for a later revisit. The kernel computed gadget 0's
R-scaled wire sums  x_s = sum_k v_k x_{k,s}  (v_k = c_k R or d_k R, mod p) as an int8 GEMM per report:
  * mf_digits(v): s = v if v <= 127 J else v - p; u = s + 128 J; digits d_i = byte_i(u) XOR 0x80 as int8,
    so sum_i d_i 256^i = s == v (mod p) (J = 0x0101..01, 16 bytes);
  * B[16 h + j][slot] = byte_j(x_{call h, slot}) XOR 0x80 (the int8 digits of x - 128 J);
  * A[a][16 h + j] = d_{a-j}(v_{call h}), built per 32-bit word w by v_perm_b32(hi, lo, sel(a, w)) from
    the digit words floor(a/4) - w - 1 (lo) and floor(a/4) - w (hi), indices clamped to 0..3;
  * C[a][slot] = sum_{h,j} A[a][16 h + j] B[16 h + j][slot] over all K-steps (2 calls each);
  * fold: G_m = sum_t C[4 m + t][slot] 2^(8 t) at weight 2^(32 m), carry-propagated to a 288-bit two's
    complement value U (sign from the last carry), reduced mod p, minus 2^288 mod p when negative, plus
    the correction 128 J sum_k v_k.
These tests replay exactly those steps (including the v_perm byte semantics and the v16 accumulator lane
map) and compare with the direct modular sum.
"""
from __future__ import annotations

import random

P = 2**128 - 28 * 2**64 + 1
J = int.from_bytes(b"\x01" * 16, "little")
M128 = (1 << 128) - 1


def mf_digits(v: int) -> bytes:
    """Kernel mf_digits: the 16 stored bytes (byte_i(u) XOR 0x80)."""
    assert 0 <= v < P
    s = v if v <= 127 * J else v - P
    u = (s + 128 * J) & M128
    assert u - 128 * J == s
    return bytes(b ^ 0x80 for b in u.to_bytes(16, "little"))


def i8(b: int) -> int:
    return b - 256 if b >= 128 else b


def v_perm(hi: int, lo: int, sel: int) -> int:
    """v_perm_b32 D = perm(S0 = hi, S1 = lo, sel): bytes 0-3 of {S0:S1} are S1's, 4-7 S0's, 0x0c -> 0."""
    data = (hi << 32) | lo
    out = 0
    for t in range(4):
        sb = (sel >> (8 * t)) & 0xFF
        if sb <= 7:
            byte = (data >> (8 * sb)) & 0xFF
        elif sb == 0x0C:
            byte = 0
        else:
            raise AssertionError(f"selector {sb:#x} not used by the kernel")
        out |= byte << (8 * t)
    return out


def mf_sel(a: int, w: int) -> int:
    sel = 0
    base = 4 * ((a >> 2) - w - 1)
    for t in range(4):
        pos = a - 4 * w - t
        bsel = pos - base if 0 <= pos <= 15 else 0x0C
        assert bsel == 0x0C or 0 <= bsel <= 7
        sel |= bsel << (8 * t)
    return sel


def window(dig: bytes, a: int) -> list[int]:
    """A row a's 16 int8 values for one call: the kernel's 4 v_perm of clamped digit words."""
    words = [int.from_bytes(dig[4 * i:4 * i + 4], "little") for i in range(4)]
    src = [words[min(max((a >> 2) - 4 + i, 0), 3)] for i in range(5)]
    out = []
    for w in range(4):
        dw = v_perm(src[4 - w], src[3 - w], mf_sel(a, w))
        out += [i8((dw >> (8 * t)) & 0xFF) for t in range(4)]
    return out


def c_row(reg: int, lane: int) -> int:
    """v_mfma_i32_32x32x32_i8 accumulator map: register reg of lane holds C[row][lane & 31]."""
    return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)


def mfma_wire_sums(vs: list[int], xs: list[list[int]]):
    """vs[k]: coefficients of calls k (v_k R as field elements); xs[k][s]: elements for 32 slots.
    Returns the kernel's x_s for every slot, replaying digits, windows, the GEMM and the fold."""
    calls = len(vs)
    ks_n = (calls + 1) // 2
    C = [[0] * 32 for _ in range(32)]  # C[a][slot]
    for ks in range(ks_n):
        for h in range(2):
            k = 2 * ks + h
            dig = mf_digits(vs[k]) if k < calls else bytes(16)  # padded call: zero entry
            for a in range(32):
                A = window(dig, a)
                for s in range(32):
                    xb = (xs[k][s] if k < calls else 0).to_bytes(16, "little")
                    C[a][s] += sum(A[j] * i8(xb[j] ^ 0x80) for j in range(16))
    assert all(-(2**31) <= C[a][s] < 2**31 for a in range(32) for s in range(32))
    corr = 128 * J * sum(vs) % P
    c288 = pow(2, 288, P)
    out = []
    for s in range(32):
        # lane (slot s, h) holds rows c_row(reg, lane); G_m = sum_t C[4m + t] 2^(8t), m = 2 (reg >> 2) + h
        G = [0] * 8
        for h in range(2):
            lane = s + 32 * h
            for j in range(4):
                g = sum(C[c_row(4 * j + t, lane)][s] << (8 * t) for t in range(4))
                assert -(2**63) <= g < 2**63
                G[2 * j + h] = g
        L, carry = [], 0
        for m in range(8):
            t = G[m] + carry
            L.append(t & 0xFFFFFFFF)
            carry = t >> 32
        L.append(carry & 0xFFFFFFFF)
        U = sum(limb << (32 * i) for i, limb in enumerate(L))
        v = U % P
        if carry < 0:
            v = (v - c288) % P
        out.append((v + corr) % P)
    return out


def test_digits_exact():
    rng = random.Random(1)
    edge = [0, 1, 127 * J, 127 * J + 1, P - 1, P // 2, (P - 1) // 2, 2**127, 2**127 - 1, 128 * J, P - 128 * J]
    for v in edge + [rng.randrange(P) for _ in range(3000)]:
        if v >= P:
            continue
        d = [i8(b) for b in mf_digits(v)]
        assert sum(x * 256**j for j, x in enumerate(d)) % P == v
    # a zero staging entry (padded call) is the digits of 0
    assert mf_digits(0) == bytes(16)


def test_window_is_toeplitz():
    rng = random.Random(3)
    for _ in range(50):
        dig = mf_digits(rng.randrange(P))
        d = [i8(b) for b in dig]
        for a in range(32):
            want = [d[a - j] if 0 <= a - j <= 15 else 0 for j in range(16)]
            assert window(dig, a) == want


def test_wire_sums_match_direct():
    rng = random.Random(7)
    for calls in (1, 2, 5):
        vs = [rng.randrange(P) for _ in range(calls)]
        vs[0] = P - 1
        xs = [[rng.randrange(P) for _ in range(32)] for _ in range(calls)]
        xs[0][0] = 0
        xs[-1][31] = P - 1
        got = mfma_wire_sums(vs, xs)
        for s in range(32):
            assert got[s] == sum(v * row[s] for v, row in zip(vs, xs)) % P


def test_missing_elements_are_zero_entries():
    """Elements past the share (ragged last call) and padded slots are loaded from a zero constant: with
    the x - 128 J digit bias and the full correction they contribute exactly 0."""
    rng = random.Random(11)
    vs = [rng.randrange(P) for _ in range(3)]
    xs = [[rng.randrange(P) for _ in range(32)] for _ in range(3)]
    for s in range(20, 32):
        xs[2][s] = 0
    got = mfma_wire_sums(vs, xs)
    for s in range(32):
        assert got[s] == sum(v * row[s] for v, row in zip(vs, xs)) % P


def test_accumulator_headroom():
    """|C| <= calls * 16 * 128^2 < 2^31 for the supported 4096 calls; the 64-bit columns stay far below
    2^63 (G_m < 2^31 * 2^25)."""
    calls = 4096
    assert calls * 16 * 128 * 128 <= 2**31
    assert (2**31) * (1 + 2**8 + 2**16 + 2**24) < 2**63
