"""Host check of the arithmetic behind the matrix-core K3 (flp_psum_mfma_kernel).

The kernel computes the FLP wire sums  E_i = sum_k d_k x_{k,i},  O_i = sum_k c_k x_{k,i}  (mod p)
as an int8 GEMM per report:
  * coefficient c (canonical) -> v = c if c <= 127*J else c - p  (J = 0x0101..01, 16 bytes),
    u = v + 128*J mod 2^128, digits a_j = byte_j(u) XOR 0x80 as int8:  sum_j a_j 256^j = v == c;
  * measurement element x -> digits b_j = byte_j(x) XOR 0x80 as int8: sum_j b_j 256^j = x - 128*J;
  * v_mfma_i32_32x32x32_i8 tiles: rows = 16 c digits + 16 d digits, columns = (slot s, dword q),
    four instructions t = byte within the dword; lane (col, h) holds rows (r&3) + 8(r>>2) + 4h;
  * per lane the 32 int32 results of each half fold into 14 byte positions, biased by 2^30, as
    64-bit columns at 32-bit spacing; a shuffle tree adds the 8 lanes of a slot (column offset
    q + h); the sum is reduced mod p, the bias constant subtracted and 128*J*sum_k c_k added.
This test replays exactly those steps with Python integers and compares with the direct sum.
"""
from __future__ import annotations

import random

P = 2**128 - 28 * 2**64 + 1
J = int.from_bytes(b"\x01" * 16, "little")
B0 = 1 << 30


def digits_coef(c):
    v = c if c <= 127 * J else c - P
    u = (v + 128 * J) % 2**128
    return [((u >> (8 * j)) & 0xFF) - 128 for j in range(16)]


def digits_meas(x):
    return [((x >> (8 * j)) & 0xFF) - 128 for j in range(16)]


def fold(cols):
    """mf_fold: carry-normalise 64-bit columns at 32-bit spacing, then reduce mod p."""
    return sum(v << (32 * m) for m, v in enumerate(cols)) % P


def lane_columns(acc_half, q, h):
    """One lane's 8 relative columns (before the tree) for one half (c or d).

    acc_half[t][r8] = MFMA result of instruction t, register r8 (0..7) of this half."""
    Ppos = [0] * 15
    for t in range(4):
        for r8 in range(8):
            Ppos[(r8 & 3) + t + 8 * (r8 >> 2)] += acc_half[t][r8]
    cols = [0] * 8
    for pos in list(range(7)) + list(range(8, 15)):
        assert -B0 <= Ppos[pos] < B0
        cols[pos // 4] += (Ppos[pos] + B0) << (8 * (pos % 4))
    # the lane's columns sit at offset q + h of the slot's
    out = [0] * 8
    for m in range(8):
        if cols[m]:
            out[m + q + h] += cols[m]
    return out


def bias_constant():
    cols = [0] * 8
    for q in range(4):
        for h in range(2):
            for pos in list(range(7)) + list(range(8, 15)):
                cols[pos // 4 + q + h] += B0 << (8 * (pos % 4))
    return fold(cols)


def mfma_wire_sums(cs, ds, xs):
    """cs, ds: calls coefficients; xs[k][s] for 8 slots. Returns (E[s], O[s])."""
    calls = len(cs)
    A = [digits_coef(c) for c in cs]
    Ad = [digits_coef(d) for d in ds]
    X = [[digits_meas(x) for x in row] for row in xs]
    corr_c = 128 * J * sum(cs) % P
    corr_d = 128 * J * sum(ds) % P
    bias = bias_constant()
    E, O = [], []
    for s in range(8):
        tot = {"c": [0] * 8, "d": [0] * 8}
        for q in range(4):
            for h in range(2):
                # the MFMA tile entries this lane holds: rows (r&3)+8(r>>2)+4h, column (s, q), all t
                for half, D in (("c", A), ("d", Ad)):
                    acc = [[0] * 8 for _ in range(4)]
                    for t in range(4):
                        for r8 in range(8):
                            a = (r8 & 3) + 8 * (r8 >> 2) + 4 * h
                            acc[t][r8] = sum(D[k][a] * X[k][s][4 * q + t] for k in range(calls))
                    lc = lane_columns(acc, q, h)
                    tot[half] = [u + v for u, v in zip(tot[half], lc)]
        O.append((fold(tot["c"]) - bias + corr_c) % P)
        E.append((fold(tot["d"]) - bias + corr_d) % P)
    return E, O


def test_digits_exact():
    rng = random.Random(1)
    edge = [0, 1, 127 * J, 127 * J + 1, P - 1, P // 2, (P - 1) // 2, 2**127, 2**127 - 1, 128 * J, P - 128 * J]
    for c in edge + [rng.randrange(P) for _ in range(2000)]:
        if c >= P:
            continue
        d = digits_coef(c)
        assert all(-128 <= x <= 127 for x in d)
        assert sum(x * 256**j for j, x in enumerate(d)) % P == c
    for x in [0, P - 1, 2**128 - 1] + [rng.randrange(P) for _ in range(500)]:
        assert sum(b * 256**j for j, b in enumerate(digits_meas(x))) == x - 128 * J


def test_wire_sums_match_direct():
    rng = random.Random(7)
    for calls in (1, 3, 33):
        cs = [rng.randrange(P) for _ in range(calls)]
        ds = [rng.randrange(P) for _ in range(calls)]
        cs[0] = P - 1
        xs = [[rng.randrange(P) for _ in range(8)] for _ in range(calls)]
        xs[0][0] = 0
        xs[-1][7] = P - 1
        E, O = mfma_wire_sums(cs, ds, xs)
        for s in range(8):
            assert O[s] == sum(c * row[s] for c, row in zip(cs, xs)) % P
            assert E[s] == sum(d * row[s] for d, row in zip(ds, xs)) % P


def test_bias_column_headroom():
    """Columns stay below 2^64 at the largest supported call count (8192): |acc| <= calls * 2^14,
    a byte position sums <= 4 of them (< 2^29 < B0), and a final column sums <= 32 shifted terms."""
    calls = 8192
    assert 4 * calls * 2**14 < B0
    assert 32 * ((2 * B0) << 24) < 2**64
