"""Host model of the word-per-lane helper K1 (`xof_words_kernel`, jx_kernels.hip): the per-lane LDS
addresses, the rho operand trick and the message window, replayed instruction by instruction over the
64 lanes of a wave against a simulated LDS region, and checked against the pure-Python Keccak and
sponge of oracle/pyref.py. The GPU parity tests (test_gpu_parity.py::test_k1_split_variants[words],
test_gpu_fixedpoint.py::test_two_jobs_in_flight[words]) check the kernel itself against the oracle."""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import pyref  # noqa: E402

M32 = 0xFFFFFFFF
ROT = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]
KW_AS, KW_AJ, KW_BS, KW_BJ, KW_MSG, KW_INIT, KW_SINK, KW_WORDS = 0, 35, 70, 105, 140, 167, 188, 189


def alignbit(hi, lo, s):
    return (((hi << 32) | lo) >> (s & 31)) & M32


def lane_consts(lane):
    """KwLane of xof_words_kernel for one lane."""
    jg = lane >= 32
    i = lane & 31
    act = i < 25
    ia = i if act else 0
    x, y = ia % 5, ia // 5
    A0, B0 = (KW_AJ, KW_BJ) if jg else (KW_AS, KW_BS)
    xp, yp = y, (2 * x + 3 * y) % 5
    k = {}
    k["aw1"] = A0 + (x + 1) * 5 + y if act else KW_SINK
    k["aw2"] = KW_SINK if not act else (A0 + y if x == 4 else (A0 + 30 + y if x == 0 else k["aw1"]))
    k["ab"] = A0 + x * 5
    k["bw1"] = B0 + yp * 7 + xp if act else KW_SINK
    k["bw2"] = KW_SINK if not act else (k["bw1"] + 5 if xp < 2 else k["bw1"])
    k["bb"] = B0 + y * 7 + x
    R = ROT[ia]
    M = R & 31
    k["pm"] = M32 if ((R >= 32) != (M == 0)) else 0
    k["s"] = (32 - M) & 31
    k["m0"] = M32 if act and ia == 0 else 0
    return k


K = [lane_consts(lane) for lane in range(64)]


def kw_round(L, lo, hi, ir):
    """One kw_round over all 64 lanes; every LDS instruction completes for all lanes before the next."""
    rlo, rhi = pyref._RC[ir] & M32, pyref._RC[ir] >> 32
    for a in ("aw1", "aw2"):
        for ln in range(64):
            L[K[ln][a]] = (lo[ln], hi[ln])
    for ln in range(64):
        k = K[ln]
        cm = [L[k["ab"] + j] for j in range(5)]
        cp = [L[k["ab"] + j + 10] for j in range(5)]
        cml = cm[0][0] ^ cm[1][0] ^ cm[2][0] ^ cm[3][0] ^ cm[4][0]
        cmh = cm[0][1] ^ cm[1][1] ^ cm[2][1] ^ cm[3][1] ^ cm[4][1]
        cpl = cp[0][0] ^ cp[1][0] ^ cp[2][0] ^ cp[3][0] ^ cp[4][0]
        cph = cp[0][1] ^ cp[1][1] ^ cp[2][1] ^ cp[3][1] ^ cp[4][1]
        lo[ln] ^= cml ^ alignbit(cpl, cph, 31)
        hi[ln] ^= cmh ^ alignbit(cph, cpl, 31)
        P = (lo[ln] & k["pm"]) | (hi[ln] & ~k["pm"] & M32)
        Q = lo[ln] ^ hi[ln] ^ P
        lo[ln], hi[ln] = alignbit(Q, P, k["s"]), alignbit(P, Q, k["s"])
    for a in ("bw1", "bw2"):
        for ln in range(64):
            L[K[ln][a]] = (lo[ln], hi[ln])
    for ln in range(64):
        k = K[ln]
        b0, b1, b2 = L[k["bb"]], L[k["bb"] + 1], L[k["bb"] + 2]
        lo[ln] = (b0[0] ^ (~b1[0] & M32 & b2[0])) ^ (rlo & k["m0"])
        hi[ln] = (b0[1] ^ (~b1[1] & M32 & b2[1])) ^ (rhi & k["m0"])


def test_layout_addresses_are_a_partition():
    """Each sponge's words land in distinct theta slots and distinct chi slots (plus their wrap copies),
    the reads stay inside the sponge's own tables, and idle lanes write only the sink."""
    for grp, (A0, B0) in enumerate(((KW_AS, KW_BS), (KW_AJ, KW_BJ))):
        lanes = [32 * grp + i for i in range(25)]
        prim_a = {K[ln]["aw1"] for ln in lanes}
        prim_b = {K[ln]["bw1"] for ln in lanes}
        assert len(prim_a) == 25 and len(prim_b) == 25
        assert all(A0 <= a < A0 + 35 for a in prim_a | {K[ln]["aw2"] for ln in lanes})
        assert all(B0 <= a < B0 + 35 for a in prim_b | {K[ln]["bw2"] for ln in lanes})
        assert all(A0 <= K[ln]["ab"] and K[ln]["ab"] + 14 < A0 + 35 for ln in lanes)
        assert all(B0 <= K[ln]["bb"] and K[ln]["bb"] + 2 < B0 + 35 for ln in lanes)
    for ln in list(range(25, 32)) + list(range(57, 64)):
        assert {K[ln][a] for a in ("aw1", "aw2", "bw1", "bw2")} == {KW_SINK}


def test_rounds_match_keccak_p12():
    """12 kw_rounds (rounds 12..23) on both sponges of a wave == Keccak-p[1600,12] (oracle/pyref.py)."""
    rng = random.Random(5)
    for _ in range(3):
        S = [[rng.getrandbits(64) for _ in range(5)] for _ in range(5)]
        J = [[rng.getrandbits(64) for _ in range(5)] for _ in range(5)]
        lo, hi = [rng.getrandbits(32) for _ in range(64)], [rng.getrandbits(32) for _ in range(64)]
        for g, st in ((0, S), (32, J)):
            for i in range(25):
                w = st[i % 5][i // 5]
                lo[g + i], hi[g + i] = w & M32, w >> 32
        L = [(0, 0)] * KW_WORDS
        for ir in range(12, 24):
            kw_round(L, lo, hi, ir)
        for g, st in ((0, S), (32, J)):
            want = pyref.keccak_p(st, 12)
            got = [[lo[g + x + 5 * y] | (hi[g + x + 5 * y] << 32) for y in range(5)] for x in range(5)]
            assert got == want


def _header_window(h):
    """The message window's prefix (xof_words_kernel): words 0..5 = stream bytes [-48, 0), header at [-42, 0)."""
    w = [int.from_bytes(h[4 * q:4 * q + 4].ljust(4, b"\0"), "little") for q in range(11)]
    win = [(0, (w[0] << 16) & M32)]
    for t in range(1, 6):
        win.append((alignbit(w[2 * t - 1], w[2 * t - 2], 16), alignbit(w[2 * t], w[2 * t - 1], 16)))
    return win


def _j_words(win, last, nb):
    """J lane w's message word from window words (w, w + 1), with the last block's padding."""
    out = []
    for i in range(21):
        v0, v1 = win[i], win[i + 1]
        wd = [alignbit(v1[0], v0[1], 16), alignbit(v1[1], v1[0], 16)]
        if last:
            for h in range(2):
                d = 2 * i + h
                lb = 4 * d
                if lb >= nb:
                    wd[h] = 0
                elif lb + 4 > nb:
                    wd[h] &= (1 << (8 * (nb - lb))) - 1
                if d == nb >> 2:
                    wd[h] ^= 1 << (8 * (nb & 3))
                if d == 41:
                    wd[h] ^= 0x80000000
        out.append(wd[0] | (wd[1] << 32))
    return out


def test_message_window_absorbs_header_then_stream():
    """J absorbs header || S stream: the kernel's window (previous block's words 15..20, then the block)
    and 48-bit funnel give exactly the padded TurboSHAKE message blocks, for share lengths whose last
    block is partial, exactly full, or only padding."""
    rng = random.Random(9)
    for MB in (16 * 5, 16 * 21, 16 * 100, 168 * 3 - 42, 168 * 4 - 42 + 16, 168 * 2):
        hdr = bytes(rng.getrandbits(8) for _ in range(42))
        NM = (MB + 167) // 168
        stream = bytes(rng.getrandbits(8) for _ in range(168 * (NM + 1)))  # squeezed blocks (past the share too)
        ML = 42 + MB
        b_last = ML // 168
        msg = hdr + stream[:MB]
        padded = bytearray(msg) + b"\x01"
        while len(padded) % 168:
            padded.append(0)
        padded[-1] ^= 0x80
        assert len(padded) // 168 == b_last + 1
        win = _header_window(hdr)
        for m in range(b_last + 1):
            blk = stream[168 * m:168 * m + 168]
            cur = [(int.from_bytes(blk[8 * i:8 * i + 4], "little"), int.from_bytes(blk[8 * i + 4:8 * i + 8], "little"))
                   for i in range(21)]
            win = win[:6] + cur
            got = _j_words(win, m == b_last, ML - 168 * m)
            want = [int.from_bytes(padded[168 * m + 8 * i:168 * m + 8 * i + 8], "little") for i in range(21)]
            assert got == want, (MB, m)
            win = cur[15:21] + win[6:]
