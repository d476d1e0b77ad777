"""TEST INFRASTRUCTURE ONLY — an independent pure-Python restatement of Prio3 (VDAF-08).

Written in the style of the VDAF-08 reference pseudocode (draft-irtf-cfrg-vdaf-08
§6-§7) so it shares no code with the C oracle (prio3_oracle.c); the two are
cross-checked on small configurations in tests/test_oracle_crosscheck.py.
Pure-Python loops: use it for small cases only (Count, Sum with few bits,
small Histogram / SumVec). Parity vs prio 0.16.1 is UNPINNED.
"""
from __future__ import annotations

# --------------------------------------------------------------------------- Keccak / TurboSHAKE

_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_M64 = (1 << 64) - 1


def _rot(v, n):
    return ((v << n) | (v >> (64 - n))) & _M64 if n else v


def _rho_offsets():
    # derived from the (x, y) -> (y, 2x + 3y) walk of FIPS 202 §3.2.2
    r = [[0] * 5 for _ in range(5)]
    x, y = 1, 0
    for t in range(24):
        r[x][y] = ((t + 1) * (t + 2) // 2) % 64
        x, y = y, (2 * x + 3 * y) % 5
    return r


_R = _rho_offsets()


def keccak_p(lanes, rounds):
    """lanes[x][y] (5x5 of u64)."""
    A = [row[:] for row in lanes]
    for ir in range(24 - rounds, 24):
        C = [A[x][0] ^ A[x][1] ^ A[x][2] ^ A[x][3] ^ A[x][4] for x in range(5)]
        D = [C[(x - 1) % 5] ^ _rot(C[(x + 1) % 5], 1) for x in range(5)]
        A = [[A[x][y] ^ D[x] for y in range(5)] for x in range(5)]
        B = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                B[y][(2 * x + 3 * y) % 5] = _rot(A[x][y], _R[x][y])
        A = [[B[x][y] ^ ((~B[(x + 1) % 5][y]) & B[(x + 2) % 5][y]) for y in range(5)] for x in range(5)]
        A[0][0] ^= _RC[ir]
    return A


def _sponge(msg: bytes, D: int, outlen: int, rounds: int, rate: int = 168) -> bytes:
    padded = bytearray(msg)
    padded.append(D)
    while len(padded) % rate:
        padded.append(0)
    padded[-1] ^= 0x80
    A = [[0] * 5 for _ in range(5)]
    for off in range(0, len(padded), rate):
        blk = padded[off:off + rate]
        for i in range(rate // 8):
            A[i % 5][i // 5] ^= int.from_bytes(blk[8 * i:8 * i + 8], "little")
        A = keccak_p(A, rounds)
    out = bytearray()
    while True:
        for i in range(rate // 8):
            out += A[i % 5][i // 5].to_bytes(8, "little")
        if len(out) >= outlen:
            return bytes(out[:outlen])
        A = keccak_p(A, rounds)


def turboshake128(msg: bytes, D: int, outlen: int) -> bytes:
    return _sponge(msg, D, outlen, 12)


def shake128_24(msg: bytes, outlen: int) -> bytes:
    """SHAKE128 = 24 rounds, D = 0x1F: checked against hashlib in tests."""
    return _sponge(msg, 0x1F, outlen, 24)


# --------------------------------------------------------------------------- fields


class Field:
    def __init__(self, p, enc, gen_log2):
        self.p, self.ENCODED_SIZE, self.GEN_ORDER_LOG2 = p, enc, gen_log2
        self.GEN = pow(7, (p - 1) >> gen_log2, p)

    def root(self, n):  # n = power of two
        return pow(self.GEN, (1 << self.GEN_ORDER_LOG2) // n, self.p)

    def encode_vec(self, v):
        return b"".join(int(x).to_bytes(self.ENCODED_SIZE, "little") for x in v)

    def decode_vec(self, b):
        if len(b) % self.ENCODED_SIZE:
            raise ValueError("length")
        out = []
        for i in range(0, len(b), self.ENCODED_SIZE):
            x = int.from_bytes(b[i:i + self.ENCODED_SIZE], "little")
            if x >= self.p:
                raise ValueError("modulus overflow")
            out.append(x)
        return out


Field64 = Field(2**64 - 2**32 + 1, 8, 32)
Field128 = Field(2**128 - 28 * 2**64 + 1, 16, 66)


# --------------------------------------------------------------------------- XOF


class XofTurboShake128:
    SEED_SIZE = 16

    def __init__(self, seed: bytes, dst: bytes, binder: bytes):
        self.m = bytes([len(dst)]) + dst + seed + binder
        self.l = 0
        self.stream = b""

    def next(self, length):
        self.l += length
        if len(self.stream) < self.l:  # squeeze ahead (doubling) instead of re-squeezing per call
            self.stream = turboshake128(self.m, 1, max(self.l, 2 * len(self.stream), 168))
        return self.stream[self.l - length:self.l]

    def next_vec(self, field, length):
        m = (1 << (8 * field.ENCODED_SIZE)) - 1
        vec = []
        while len(vec) < length:
            x = int.from_bytes(self.next(field.ENCODED_SIZE), "little") & m
            if x < field.p:
                vec.append(x)
        return vec

    @classmethod
    def derive_seed(cls, seed, dst, binder):
        return cls(seed, dst, binder).next(cls.SEED_SIZE)

    @classmethod
    def expand_into_vec(cls, field, seed, dst, binder, length):
        return cls(seed, dst, binder).next_vec(field, length)


class XofHmacSha256Aes128(XofTurboShake128):
    """prio 0.16.1 XofHmacSha256Aes128 (used by Janus core/src/vdaf.rs:8,173-199): tag =
    HMAC-SHA256(seed, byte(len(dst)) || dst || binder); stream = AES-128-CTR keystream, key
    tag[:16], initial counter block tag[16:], low 64 bits a big-endian counter (Ctr64BE)."""
    SEED_SIZE = 32

    def __init__(self, seed: bytes, dst: bytes, binder: bytes):
        import hashlib
        import hmac

        from oracle.hpke_oracle import aes128_expand
        tag = hmac.new(seed, bytes([len(dst)]) + dst + binder, hashlib.sha256).digest()
        self.rk = aes128_expand(tag[:16])
        self.iv_hi, self.ctr = tag[16:24], int.from_bytes(tag[24:], "big")
        self.buf = b""

    def next(self, length):
        from oracle.hpke_oracle import aes128_encrypt_block
        while len(self.buf) < length:
            self.buf += aes128_encrypt_block(self.rk, self.iv_hi + self.ctr.to_bytes(8, "big"))
            self.ctr = (self.ctr + 1) % (1 << 64)
        out, self.buf = self.buf[:length], self.buf[length:]
        return out


# --------------------------------------------------------------------------- polynomials


def poly_eval(F, p, x):
    r = 0
    for c in reversed(p):
        r = (r * x + c) % F.p
    return r


def poly_mul(F, a, b):
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            out[i + j] = (out[i + j] + x * y) % F.p
    return out


def poly_interp(F, xs, ys):
    """Lagrange interpolation (quadratic; pure-Python oracle uses it for small P)."""
    n = len(xs)
    coef = [0] * n
    for i in range(n):
        num, den = [1], 1
        for j in range(n):
            if j != i:
                num = poly_mul(F, num, [(-xs[j]) % F.p, 1])
                den = den * (xs[i] - xs[j]) % F.p
        s = ys[i] * pow(den, F.p - 2, F.p) % F.p
        for k in range(n):
            coef[k] = (coef[k] + s * num[k]) % F.p
    return coef


# --------------------------------------------------------------------------- gadgets / circuits


class Mul:
    ARITY, DEGREE = 2, 2

    def eval(self, F, x):
        return x[0] * x[1] % F.p

    def eval_poly(self, F, polys):
        return poly_mul(F, polys[0], polys[1])


class Range2:  # PolyEval([0, -1, 1]) : x^2 - x
    ARITY, DEGREE = 1, 2

    def eval(self, F, x):
        return (x[0] * x[0] - x[0]) % F.p

    def eval_poly(self, F, polys):
        sq = poly_mul(F, polys[0], polys[0])
        return [(sq[i] - (polys[0][i] if i < len(polys[0]) else 0)) % F.p for i in range(len(sq))]


class ParallelSumMul:
    def __init__(self, count):
        self.count = count
        self.ARITY, self.DEGREE = 2 * count, 2

    def eval(self, F, x):
        return sum(x[2 * j] * x[2 * j + 1] for j in range(self.count)) % F.p

    def eval_poly(self, F, polys):
        out = None
        for j in range(self.count):
            t = poly_mul(F, polys[2 * j], polys[2 * j + 1])
            out = t if out is None else [(a + b) % F.p for a, b in zip(out, t)]
        return out


class ParallelSumPoly:
    """ParallelSum(PolyEval(poly), count): sum_j poly(x_j) (FixedPointBoundedL2VecSum's norm gadget)."""

    def __init__(self, poly, count):
        self.poly, self.count = poly, count
        self.ARITY, self.DEGREE = count, len(poly) - 1

    def eval(self, F, x):
        return sum(poly_eval(F, self.poly, x[j]) for j in range(self.count)) % F.p

    def eval_poly(self, F, polys):
        out = [0]
        for j in range(self.count):
            comp, pw = [0], [1]  # poly(f_j) by Horner-free expansion: sum_i c_i f_j^i
            for c in self.poly:
                term = [c * a % F.p for a in pw]
                comp = [((comp[i] if i < len(comp) else 0) + (term[i] if i < len(term) else 0)) % F.p
                        for i in range(max(len(comp), len(term)))]
                pw = poly_mul(F, pw, polys[j])
            out = [((out[i] if i < len(out) else 0) + (comp[i] if i < len(comp) else 0)) % F.p
                   for i in range(max(len(out), len(comp)))]
        return out


def next_pow2(n):
    p = 1
    while p < n:
        p <<= 1
    return p


def _isqrt(n):
    r = 0
    while (r + 1) * (r + 1) <= n:
        r += 1
    return r


class Valid:
    """Circuits as in VDAF-08 §7.4 (and prio 0.16.1 flp::types), plus prio's
    FixedPointBoundedL2VecSum (flp::types::fixedpoint_l2; restated from memory)."""

    def __init__(self, kind, bits=0, length=0, chunk=0, field=None):
        self.kind = kind
        if kind == "count":
            self.Field, self.GADGETS, self.GADGET_CALLS = Field64, [Mul()], [1]
            self.MEAS_LEN, self.OUTPUT_LEN, self.JOINT_RAND_LEN = 1, 1, 0
        elif kind == "sum":
            self.Field, self.GADGETS, self.GADGET_CALLS = Field128, [Range2()], [bits]
            self.MEAS_LEN, self.OUTPUT_LEN, self.JOINT_RAND_LEN = bits, 1, 1
        elif kind == "sumvec":
            self.Field, self.GADGETS = field or Field128, [ParallelSumMul(chunk)]
            self.MEAS_LEN, self.OUTPUT_LEN, self.JOINT_RAND_LEN = bits * length, length, 1
            self.GADGET_CALLS = [(self.MEAS_LEN + chunk - 1) // chunk]
        elif kind == "histogram":
            self.Field, self.GADGETS = Field128, [ParallelSumMul(chunk)]
            self.MEAS_LEN, self.OUTPUT_LEN, self.JOINT_RAND_LEN = length, length, 2
            self.GADGET_CALLS = [(length + chunk - 1) // chunk]
        elif kind == "fixedpoint":
            # entries of `bits`-bit fixed point numbers in [-1, 1) plus their claimed squared norm
            F = self.Field = Field128
            self.norm_bits = 2 * bits - 2
            self.MEAS_LEN, self.OUTPUT_LEN, self.JOINT_RAND_LEN = bits * length + self.norm_bits, length, 2
            c0, c1 = max(1, _isqrt(self.MEAS_LEN)), max(1, _isqrt(length))
            norm_poly = [1 << (2 * bits - 2), (-(1 << bits)) % F.p, 1]
            self.GADGETS = [ParallelSumMul(c0), ParallelSumPoly(norm_poly, c1)]
            self.GADGET_CALLS = [-(-self.MEAS_LEN // c0), -(-length // c1)]
            chunk = c0
        self.bits, self.length, self.chunk = bits, length, chunk
        self.Ps = [next_pow2(1 + c) for c in self.GADGET_CALLS]
        self.P = self.Ps[0]
        self.GADGET = self.GADGETS[0]
        self.PROOF_LEN = sum(g.ARITY + g.DEGREE * (P - 1) + 1 for g, P in zip(self.GADGETS, self.Ps))
        self.VERIFIER_LEN = 1 + sum(g.ARITY + 1 for g in self.GADGETS)
        self.PROVE_RAND_LEN = sum(g.ARITY for g in self.GADGETS)
        self.QUERY_RAND_LEN = len(self.GADGETS)

    def encode(self, m):
        if self.kind == "count":
            return [m]
        if self.kind == "sum":
            return [(m >> i) & 1 for i in range(self.bits)]
        if self.kind == "sumvec":
            return [(m[i] >> j) & 1 for i in range(self.length) for j in range(self.bits)]
        if self.kind == "fixedpoint":
            n = self.bits
            ys = [(x ^ (1 << (n - 1))) & ((1 << n) - 1) for x in m]  # to_field_integer
            norm = sum((y - (1 << (n - 1))) ** 2 for y in ys)
            out = [(y >> b) & 1 for y in ys for b in range(n)]
            return out + [(norm >> b) & 1 for b in range(self.norm_bits)]  # low bits if |x| >= 1 (dishonest)
        return [1 if i == m else 0 for i in range(self.length)]

    def truncate(self, meas):
        F = self.Field
        if self.kind in ("count", "histogram"):
            return list(meas)
        b = self.bits
        return [sum((1 << j) * meas[i * b + j] for j in range(b)) % F.p for i in range(self.OUTPUT_LEN)]

    def _range_checks(self, call, meas, r, num_shares):
        p = self.Field.p
        shares_inv = pow(num_shares, p - 2, p)
        chunk = self.GADGETS[0].ARITY // 2
        r_power, out = r, 0
        for i in range(self.GADGET_CALLS[0]):
            inputs = []
            for j in range(chunk):
                idx = i * chunk + j
                if idx < len(meas):
                    inputs += [r_power * meas[idx] % p, (meas[idx] - shares_inv) % p]
                    r_power = r_power * r % p
                else:
                    inputs += [0, (-shares_inv) % p]
            out = (out + call(inputs)) % p
        return out

    def eval(self, calls, meas, joint_rand, num_shares):
        F = self.Field
        p = F.p
        call = calls[0]
        if self.kind == "count":
            return (call([meas[0], meas[0]]) - meas[0]) % p
        if self.kind == "sum":
            out, r = 0, joint_rand[0]
            for b in meas:
                out = (out + r * call([b])) % p
                r = r * joint_rand[0] % p
            return out
        shares_inv = pow(num_shares, p - 2, p)
        range_check = self._range_checks(call, meas, joint_rand[0], num_shares)
        if self.kind == "sumvec":
            return range_check
        if self.kind == "fixedpoint":
            n, E, g1 = self.bits, self.length, self.GADGETS[1]
            ys = [sum(meas[i * n + b] << b for b in range(n)) % p for i in range(E)]
            pad = (1 << (n - 1)) * shares_inv % p
            computed = 0
            for k in range(self.GADGET_CALLS[1]):
                chunk = [ys[k * g1.count + j] if k * g1.count + j < E else pad for j in range(g1.count)]
                computed = (computed + calls[1](chunk)) % p
            claimed = sum(meas[E * n + b] << b for b in range(self.norm_bits)) % p
            return (joint_rand[1] * range_check + joint_rand[1] ** 2 * (computed - claimed)) % p
        sum_check = (sum(meas) - shares_inv) % p
        return (joint_rand[1] * range_check + joint_rand[1] ** 2 * sum_check) % p


class FlpGeneric:
    def __init__(self, valid: Valid):
        self.V = valid

    def _run(self, meas, wire_seeds, joint_rand, num_shares, out_fns):
        """wire_seeds[g] and out_fns[g] per gadget; returns (v, wires[g][j][k])."""
        V = self.V
        wires, ks, calls = [], [], []
        for g, (gadget, P) in enumerate(zip(V.GADGETS, V.Ps)):
            w = [[0] * P for _ in range(gadget.ARITY)]
            for j in range(gadget.ARITY):
                w[j][0] = wire_seeds[g][j]
            wires.append(w)
            ks.append([0])

            def call(inp, g=g, w=w, k=ks[-1]):
                k[0] += 1
                for j, x in enumerate(inp):
                    w[j][k[0]] = x
                return out_fns[g](inp, k[0])
            calls.append(call)
        v = V.eval(calls, meas, joint_rand, num_shares)
        return v, wires

    def _split(self, vec, sizes):
        out, o = [], 0
        for n in sizes:
            out.append(vec[o:o + n])
            o += n
        return out

    def prove(self, meas, prove_rand, joint_rand):
        V, F = self.V, self.V.Field
        seeds = self._split(list(prove_rand), [g.ARITY for g in V.GADGETS])
        _, wires = self._run(meas, seeds, joint_rand, 1,
                             [lambda inp, k, g=g: g.eval(F, inp) for g in V.GADGETS])
        proof = []
        for g, P, w, sd in zip(V.GADGETS, V.Ps, wires, seeds):
            alpha = F.root(P)
            xs = [pow(alpha, k, F.p) for k in range(P)]
            polys = [poly_interp(F, xs, wj) for wj in w]
            gp = g.eval_poly(F, polys)
            glen = g.DEGREE * (P - 1) + 1
            gp = (gp + [0] * glen)[:glen]
            proof += list(sd) + gp
        return proof

    def query(self, meas, proof, query_rand, joint_rand, num_shares):
        V, F = self.V, self.V.Field
        parts = self._split(proof, [g.ARITY + g.DEGREE * (P - 1) + 1 for g, P in zip(V.GADGETS, V.Ps)])
        seeds = [pt[:g.ARITY] for pt, g in zip(parts, V.GADGETS)]
        gps = [pt[g.ARITY:] for pt, g in zip(parts, V.GADGETS)]
        fns = [lambda inp, k, gp=gp, P=P: poly_eval(F, gp, pow(F.root(P), k, F.p)) for gp, P in zip(gps, V.Ps)]
        v, wires = self._run(meas, seeds, joint_rand, num_shares, fns)
        out = [v]
        for gi, (P, w, gp) in enumerate(zip(V.Ps, wires, gps)):
            t = query_rand[gi]
            if pow(t, P, F.p) == 1:
                raise ValueError("query rand is a root of unity")
            alpha = F.root(P)
            xs = [pow(alpha, k, F.p) for k in range(P)]
            for wj in w:
                out.append(poly_eval(F, poly_interp(F, xs, wj), t))
            out.append(poly_eval(F, gp, t))
        return out

    def decide(self, verifier):
        V, F = self.V, self.V.Field
        if verifier[0] != 0:
            return False
        o = 1
        for g in V.GADGETS:
            if g.eval(F, verifier[o:o + g.ARITY]) != verifier[o + g.ARITY]:
                return False
            o += g.ARITY + 1
        return True


# --------------------------------------------------------------------------- Prio3

ALGO_IDS = {"count": 0, "sum": 1, "sumvec": 2, "histogram": 3, "sumvec_f64_multiproof": 0xFFFF1003,
            "fixedpoint": 0xFFFF0000}
USAGE = dict(meas_share=1, proof_share=2, joint_randomness=3, prove_randomness=4, query_randomness=5,
             joint_rand_seed=6, joint_rand_part=7)


class Prio3:
    SHARES = 2

    def __init__(self, kind, proofs=1, **kw):
        self.ID = ALGO_IDS[kind]
        self.Xof = XofTurboShake128
        if kind == "sumvec_f64_multiproof":  # core/src/vdaf.rs:176-199
            assert proofs >= 2
            kind, kw["field"], self.Xof = "sumvec", Field64, XofHmacSha256Aes128
        self.PROOFS = proofs
        self.valid = Valid(kind, **kw)
        self.flp = FlpGeneric(self.valid)
        self.F = self.valid.Field
        self.S = self.Xof.SEED_SIZE

    def dst(self, usage):
        return bytes([8, 0]) + self.ID.to_bytes(4, "big") + USAGE[usage].to_bytes(2, "big")

    def helper_meas_share(self, agg_id, k):
        return self.Xof.expand_into_vec(self.F, k, self.dst("meas_share"), bytes([agg_id]),
                                                self.valid.MEAS_LEN)

    def helper_proofs_share(self, agg_id, k):
        return self.Xof.expand_into_vec(self.F, k, self.dst("proof_share"),
                                                bytes([self.PROOFS, agg_id]), self.valid.PROOF_LEN * self.PROOFS)

    def joint_rand_part(self, agg_id, blind, meas_share, nonce):
        return self.Xof.derive_seed(blind, self.dst("joint_rand_part"),
                                            bytes([agg_id]) + nonce + self.F.encode_vec(meas_share))

    def joint_rand_seed(self, parts):
        return self.Xof.derive_seed(bytes(self.S), self.dst("joint_rand_seed"), b"".join(parts))

    def joint_rands(self, seed):
        return self.Xof.expand_into_vec(self.F, seed, self.dst("joint_randomness"), bytes([self.PROOFS]),
                                                self.valid.JOINT_RAND_LEN * self.PROOFS)

    def query_rands(self, vk, nonce):
        return self.Xof.expand_into_vec(self.F, vk, self.dst("query_randomness"),
                                        bytes([self.PROOFS]) + nonce, self.valid.QUERY_RAND_LEN * self.PROOFS)

    def shard(self, measurement, nonce, rand):
        """rand = k_helper_meas || k_helper_proofs || k_prove || [blind_L || blind_H], SEED_SIZE each
        (same layout as the C oracle)."""
        p, S, V, NP = self.F.p, self.S, self.valid, self.PROOFS
        k_hm, k_hp, k_prove = rand[0:S], rand[S:2 * S], rand[2 * S:3 * S]
        meas = V.encode(measurement)
        hmeas = self.helper_meas_share(1, k_hm)
        lmeas = [(a - b) % p for a, b in zip(meas, hmeas)]
        jr, public = [], b""
        if V.JOINT_RAND_LEN:
            bl, bh = rand[3 * S:4 * S], rand[4 * S:5 * S]
            pl = self.joint_rand_part(0, bl, lmeas, nonce)
            ph = self.joint_rand_part(1, bh, hmeas, nonce)
            jr = self.joint_rands(self.joint_rand_seed([pl, ph]))
            public = pl + ph
        prove_rands = self.Xof.expand_into_vec(self.F, k_prove, self.dst("prove_randomness"), bytes([NP]),
                                               V.PROVE_RAND_LEN * NP)
        proofs = []
        for i in range(NP):
            proofs += self.flp.prove(meas, prove_rands[i * V.PROVE_RAND_LEN:(i + 1) * V.PROVE_RAND_LEN],
                                     jr[i * V.JOINT_RAND_LEN:(i + 1) * V.JOINT_RAND_LEN])
        hproof = self.helper_proofs_share(1, k_hp)
        lproof = [(a - b) % p for a, b in zip(proofs, hproof)]
        leader = self.F.encode_vec(lmeas) + self.F.encode_vec(lproof)
        helper = k_hm + k_hp
        if V.JOINT_RAND_LEN:
            leader += rand[3 * S:4 * S]
            helper += rand[4 * S:5 * S]
        return public, leader, helper

    def prep_init(self, vk, agg_id, nonce, public_share, input_share):
        V, F, S, NP = self.valid, self.F, self.S, self.PROOFS
        if agg_id == 0:
            n = V.MEAS_LEN * F.ENCODED_SIZE
            m = V.PROOF_LEN * NP * F.ENCODED_SIZE
            meas = F.decode_vec(input_share[:n])
            proof = F.decode_vec(input_share[n:n + m])
            blind = input_share[n + m:]
        else:
            meas = self.helper_meas_share(agg_id, input_share[:S])
            proof = self.helper_proofs_share(agg_id, input_share[S:2 * S])
            blind = input_share[2 * S:3 * S]
        out_share = V.truncate(meas)
        jr, corrected, part = [], None, b""
        if V.JOINT_RAND_LEN:
            part = self.joint_rand_part(agg_id, blind, meas, nonce)
            parts = [public_share[0:S], public_share[S:2 * S]]
            parts[agg_id] = part
            corrected = self.joint_rand_seed(parts)
            jr = self.joint_rands(corrected)
        qr = self.query_rands(vk, nonce)
        ver = []
        for i in range(NP):
            ver += self.flp.query(meas, proof[i * V.PROOF_LEN:(i + 1) * V.PROOF_LEN],
                                  qr[i * V.QUERY_RAND_LEN:(i + 1) * V.QUERY_RAND_LEN],
                                  jr[i * V.JOINT_RAND_LEN:(i + 1) * V.JOINT_RAND_LEN], self.SHARES)
        return (out_share, corrected), F.encode_vec(ver) + part

    def prep_shares_to_prep(self, shares):
        V, F, NP = self.valid, self.F, self.PROOFS
        n = V.VERIFIER_LEN * NP * F.ENCODED_SIZE
        ver = [0] * (V.VERIFIER_LEN * NP)
        parts = []
        for s in shares:
            if len(s) != n + (self.S if V.JOINT_RAND_LEN else 0):
                raise ValueError("decode")
            v = F.decode_vec(s[:n])
            ver = [(a + b) % F.p for a, b in zip(ver, v)]
            parts.append(s[n:])
        for i in range(NP):
            if not self.flp.decide(ver[i * V.VERIFIER_LEN:(i + 1) * V.VERIFIER_LEN]):
                raise AssertionError("decide")
        return self.joint_rand_seed(parts) if V.JOINT_RAND_LEN else b""

    def helper_prep(self, vk, nonce, public_share, helper_input_share, leader_prep_share):
        """Returns (verdict, prep_msg, out_share) mirroring the C oracle's jo_helper_prep."""
        try:
            state, hshare = self.prep_init(vk, 1, nonce, public_share, helper_input_share)
        except ValueError:
            return 1, b"", None
        try:
            msg = self.prep_shares_to_prep([leader_prep_share, hshare])
        except ValueError:
            return 2, b"", None
        except AssertionError:
            return 3, b"", None
        out_share, corrected = state
        if self.valid.JOINT_RAND_LEN and msg != corrected:
            return 4, b"", None
        return 0, msg, self.F.encode_vec(out_share)
