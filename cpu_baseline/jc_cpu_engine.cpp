// jc_cpu_engine.cpp — multithreaded CPU helper prep + aggregate for the Prio3 instances of the
// BASELINE configs: Prio3Count (Field64), Prio3Sum{bits}, Prio3SumVec, Prio3Histogram and
// Prio3FixedPointBoundedL2VecSum{16|32} (Field128, TurboSHAKE128).
//
// BENCHMARK BASELINE ONLY (bench.py's cpu_baseline leg): the product path is the HIP engine
// (janus_amd/lib/libjanus_prio3.so); nothing in janus_amd loads this library.
//
// It replaces the per-report loop Janus runs on its tokio workers (aggregator/src/aggregator.rs:
// 1763-2013 -> prio 0.16.1 helper_initialized + evaluate) and the accumulation
// (aggregation_job_writer.rs:608-708), written the way an optimised CPU implementation would be,
// with the GPU path's algorithmic choices so the comparison is about the hardware, not the algorithm:
//   * TurboSHAKE128 on 64-bit lanes, squeezed and absorbed a 168-byte block at a time (the
//     measurement-share squeeze feeds the joint_rand_part absorb directly, no second pass);
//   * Field128 products as 64x64->128 partial products with lazy 320-bit wire sums, one reduction
//     per wire;
//   * the FLP query by barycentric evaluation on the P-th roots of unity (one batch inversion per
//     report), no per-wire inverse DFT; the gadget-output part of v as sum_m g_m S_m with S_m =
//     sum_k (r alpha^m)^k computed for every m by one size-P DFT (Sum) or precomputed (r = 1);
//   * report-parallel over std::thread, per-thread partial aggregates merged at the end.
// Checked byte-for-byte against the committed golden fixtures (tests/test_cpu_baseline.py).
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace {

typedef unsigned __int128 u128;

// ------------------------------------------------------------------ Keccak-p[1600, 12]
const uint64_t RC[24] = {0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
                         0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
                         0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
                         0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
                         0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
                         0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

static inline uint64_t rol(uint64_t v, int n) { return (v << n) | (v >> ((64 - n) & 63)); }

static void keccak_p12(uint64_t* A) {
  for (int ir = 12; ir < 24; ir++) {
    uint64_t C0 = A[0] ^ A[5] ^ A[10] ^ A[15] ^ A[20], C1 = A[1] ^ A[6] ^ A[11] ^ A[16] ^ A[21],
             C2 = A[2] ^ A[7] ^ A[12] ^ A[17] ^ A[22], C3 = A[3] ^ A[8] ^ A[13] ^ A[18] ^ A[23],
             C4 = A[4] ^ A[9] ^ A[14] ^ A[19] ^ A[24];
    uint64_t D0 = C4 ^ rol(C1, 1), D1 = C0 ^ rol(C2, 1), D2 = C1 ^ rol(C3, 1), D3 = C2 ^ rol(C4, 1),
             D4 = C3 ^ rol(C0, 1);
    uint64_t B[25];
    // rho + pi: B[y + 5((2x+3y)%5)] = rol(A[x+5y] ^ D[x], r[x+5y])
    B[0] = A[0] ^ D0;
    B[10] = rol(A[1] ^ D1, 1);
    B[20] = rol(A[2] ^ D2, 62);
    B[5] = rol(A[3] ^ D3, 28);
    B[15] = rol(A[4] ^ D4, 27);
    B[16] = rol(A[5] ^ D0, 36);
    B[1] = rol(A[6] ^ D1, 44);
    B[11] = rol(A[7] ^ D2, 6);
    B[21] = rol(A[8] ^ D3, 55);
    B[6] = rol(A[9] ^ D4, 20);
    B[7] = rol(A[10] ^ D0, 3);
    B[17] = rol(A[11] ^ D1, 10);
    B[2] = rol(A[12] ^ D2, 43);
    B[12] = rol(A[13] ^ D3, 25);
    B[22] = rol(A[14] ^ D4, 39);
    B[23] = rol(A[15] ^ D0, 41);
    B[8] = rol(A[16] ^ D1, 45);
    B[18] = rol(A[17] ^ D2, 15);
    B[3] = rol(A[18] ^ D3, 21);
    B[13] = rol(A[19] ^ D4, 8);
    B[14] = rol(A[20] ^ D0, 18);
    B[24] = rol(A[21] ^ D1, 2);
    B[9] = rol(A[22] ^ D2, 61);
    B[19] = rol(A[23] ^ D3, 56);
    B[4] = rol(A[24] ^ D4, 14);
    for (int y = 0; y < 25; y += 5) {
      uint64_t b0 = B[y], b1 = B[y + 1], b2 = B[y + 2], b3 = B[y + 3], b4 = B[y + 4];
      A[y] = b0 ^ (~b1 & b2);
      A[y + 1] = b1 ^ (~b2 & b3);
      A[y + 2] = b2 ^ (~b3 & b4);
      A[y + 3] = b3 ^ (~b4 & b0);
      A[y + 4] = b4 ^ (~b0 & b1);
    }
    A[0] ^= RC[ir];
  }
}

// TurboSHAKE128 absorb of an arbitrary byte stream (D = 0x01), rate 168
struct Absorb {
  uint64_t s[25];
  uint8_t buf[168];
  unsigned pos;
  void init() {
    memset(s, 0, sizeof s);
    pos = 0;
  }
  void block() {
    uint64_t w[21];
    memcpy(w, buf, 168);
    for (int i = 0; i < 21; i++) s[i] ^= w[i];
    keccak_p12(s);
    pos = 0;
  }
  void put(const uint8_t* m, size_t n) {
    while (n) {
      size_t k = 168 - pos < n ? 168 - pos : n;
      memcpy(buf + pos, m, k);
      pos += (unsigned)k;
      m += k;
      n -= k;
      if (pos == 168) block();
    }
  }
  // pad and permute: the state then holds output block 0
  void finish() {
    memset(buf + pos, 0, 168 - pos);
    buf[pos] ^= 0x01;
    buf[167] ^= 0x80;
    block();
  }
};

// XofTurboShake128 stream (VDAF-08 §6.2.1): TurboSHAKE128(len(dst) || dst || seed || binder)
struct Squeeze {
  uint64_t s[25];
  uint8_t out[168];
  unsigned pos;
  void start(Absorb& a) {
    memcpy(s, a.s, sizeof s);
    memcpy(out, s, 168);
    pos = 0;
  }
  void read(uint8_t* dst, size_t n) {
    while (n) {
      if (pos == 168) {
        keccak_p12(s);
        memcpy(out, s, 168);
        pos = 0;
      }
      size_t k = 168 - pos < n ? 168 - pos : n;
      memcpy(dst, out + pos, k);
      pos += (unsigned)k;
      dst += k;
      n -= k;
    }
  }
};

// ------------------------------------------------------------------ Field128
const u128 P = ((u128)0xFFFFFFFFFFFFFFE4ULL << 64) | 1;
const u128 CFOLD = ((u128)27 << 64) | 0xFFFFFFFFFFFFFFFFULL;  // 2^128 mod p = 28*2^64 - 1

static inline u128 fadd(u128 a, u128 b) {
  u128 s = a + b;
  if (s < a || s >= P) s -= P;
  return s;
}
static inline u128 fsub(u128 a, u128 b) { return a >= b ? a - b : a + (P - b); }

struct W5 {  // 320-bit lazy sum
  uint64_t w[5];
};
static inline void w5_zero(W5& a) { memset(a.w, 0, sizeof a.w); }
// a += x * y (x, y < 2^128)
static inline void w5_mac(W5& a, u128 x, u128 y) {
  const uint64_t x0 = (uint64_t)x, x1 = (uint64_t)(x >> 64), y0 = (uint64_t)y, y1 = (uint64_t)(y >> 64);
  const u128 p00 = (u128)x0 * y0, p01 = (u128)x0 * y1, p10 = (u128)x1 * y0, p11 = (u128)x1 * y1;
  u128 t = (u128)a.w[0] + (uint64_t)p00;
  a.w[0] = (uint64_t)t;
  t = (t >> 64) + a.w[1] + (uint64_t)(p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
  a.w[1] = (uint64_t)t;
  t = (t >> 64) + a.w[2] + (uint64_t)(p01 >> 64) + (uint64_t)(p10 >> 64) + (uint64_t)p11;
  a.w[2] = (uint64_t)t;
  t = (t >> 64) + a.w[3] + (uint64_t)(p11 >> 64);
  a.w[3] = (uint64_t)t;
  a.w[4] += (uint64_t)(t >> 64);
}
u128 C256 = 0;  // 2^256 mod p (set by jc_helper_prep_aggregate before any thread starts)

// value mod p: 2^128 == CFOLD and 2^256 == C256 fold the high words until 128 bits remain
static u128 w5_reduce(W5 a) {
  for (;;) {
    const u128 lo = ((u128)a.w[1] << 64) | a.w[0];
    if ((a.w[2] | a.w[3] | a.w[4]) == 0) return lo >= P ? lo - P : lo;
    W5 r;
    r.w[0] = a.w[0];
    r.w[1] = a.w[1];
    r.w[2] = r.w[3] = r.w[4] = 0;
    w5_mac(r, ((u128)a.w[3] << 64) | a.w[2], CFOLD);  // < 2^197
    if (a.w[4]) w5_mac(r, (u128)a.w[4], C256);        // < 2^192
    a = r;
  }
}
static inline u128 fmul(u128 a, u128 b) {
  W5 t;
  w5_zero(t);
  w5_mac(t, a, b);
  return w5_reduce(t);
}
static u128 fpow(u128 a, u128 e) {
  u128 r = 1;
  while (e) {
    if (e & 1) r = fmul(r, a);
    a = fmul(a, a);
    e >>= 1;
  }
  return r;
}
static inline u128 finv(u128 a) { return fpow(a, P - 2); }
static inline u128 ld128(const uint8_t* p) {
  u128 v;
  memcpy(&v, p, 16);
  return v;
}
static inline void st128(uint8_t* p, u128 v) { memcpy(p, &v, 16); }

// ------------------------------------------------------------------ SHA-256 of a 16-byte report id
const uint32_t SK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
static inline uint32_t ror(uint32_t v, int n) { return (v >> n) | (v << (32 - n)); }
static void sha256_16(const uint8_t id[16], uint8_t out[32]) {
  uint32_t w[64] = {0};
  for (int i = 0; i < 4; i++) w[i] = (uint32_t)id[4 * i] << 24 | id[4 * i + 1] << 16 | id[4 * i + 2] << 8 | id[4 * i + 3];
  w[4] = 0x80000000u;
  w[15] = 128;
  for (int i = 16; i < 64; i++) {
    const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + SK[i] + w[i];
    const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  const uint32_t r[8] = {h[0] + a, h[1] + b, h[2] + c, h[3] + d, h[4] + e, h[5] + f, h[6] + g, h[7] + hh};
  for (int k = 0; k < 8; k++)
    for (int j = 0; j < 4; j++) out[4 * k + j] = (uint8_t)(r[k] >> (24 - 8 * j));
}

// ------------------------------------------------------------------ Field64 (Prio3Count)
const uint64_t P64 = 0xFFFFFFFF00000001ULL;
static inline uint64_t g_add(uint64_t a, uint64_t b) {
  u128 s = (u128)a + b;
  return (uint64_t)(s >= P64 ? s - P64 : s);
}
static inline uint64_t g_sub(uint64_t a, uint64_t b) { return a >= b ? a - b : (uint64_t)((u128)a + P64 - b); }
static inline uint64_t g_mul(uint64_t a, uint64_t b) { return (uint64_t)(((u128)a * b) % P64); }
static uint64_t g_pow(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = g_mul(r, a);
    a = g_mul(a, a);
    e >>= 1;
  }
  return r;
}

// ------------------------------------------------------------------ Prio3 instance
enum { A_COUNT = 0, A_SUM = 1, A_SUMVEC = 2, A_HIST = 3, A_FIXEDPOINT = 5 };

struct Gadget {  // one FLP gadget on the P-th roots of unity
  int arity, calls, chunk, P, logP, gpoly_len;
  std::vector<u128> omega, S;  // w^k (k < P), S_m = sum_{k=1..calls} w^{km} (m < gpoly_len)
  u128 invP;
};

struct Cfg {
  int algo, bits, length, chunk;
  uint32_t algo_id;
  int meas_len, out_len, jr_len, qr_len, proof_len, ver_len, norm_bits;
  int ng;
  Gadget g[2];
  u128 half;
  uint8_t vk[16];
  size_t ps_bytes, his_bytes, lps_bytes;
};

static int next_pow2(int v, int* lg) {
  int p = 1, l = 0;
  while (p < v) {
    p <<= 1;
    l++;
  }
  *lg = l;
  return p;
}
static int isqrt_floor(int v) {
  int r = 0;
  while ((long long)(r + 1) * (r + 1) <= v) r++;
  return r < 1 ? 1 : r;
}

static void gadget_make(Gadget& g, int arity, int calls, int chunk) {
  g.arity = arity;
  g.calls = calls;
  g.chunk = chunk;
  g.P = next_pow2(calls + 1, &g.logP);
  g.gpoly_len = 2 * (g.P - 1) + 1;
  // w = 7^((p-1)/2^66) ^ (2^(66 - logP))
  u128 w = fpow(7, (P - 1) >> 66);
  for (int i = 0; i < 66 - g.logP; i++) w = fmul(w, w);
  g.omega.resize(g.P);
  u128 wk = 1;
  for (int k = 0; k < g.P; k++) {
    g.omega[k] = wk;
    wk = fmul(wk, w);
  }
  g.S.resize(g.gpoly_len);
  for (int m = 0; m < g.gpoly_len; m++) {
    u128 s = 0;
    for (int k = 1; k <= calls; k++) s = fadd(s, g.omega[((uint64_t)k * m) % g.P]);
    g.S[m] = s;
  }
  g.invP = finv(g.P);
}

static void xof_start(Absorb& a, const Cfg& c, int usage, const uint8_t seed[16]) {
  // len(dst) || dst = VERSION 8 || class 0 || algorithm id (BE) || usage (BE) || seed
  const uint8_t pre[9] = {8,
                          8,
                          0,
                          (uint8_t)(c.algo_id >> 24),
                          (uint8_t)(c.algo_id >> 16),
                          (uint8_t)(c.algo_id >> 8),
                          (uint8_t)c.algo_id,
                          (uint8_t)(usage >> 8),
                          (uint8_t)usage};
  a.init();
  a.put(pre, 9);
  a.put(seed, 16);
}

// first `n` field elements of a finished XOF (rejection sampling)
static void sample(Squeeze& q, u128* out, int n) {
  for (int i = 0; i < n;) {
    uint8_t b[16];
    q.read(b, 16);
    const u128 v = ld128(b);
    if (v < P) out[i++] = v;
  }
}

struct Acc {
  std::vector<u128> agg;
  uint64_t count = 0;
  uint8_t checksum[32] = {0};
};

static void add_checksum(Acc& acc, const uint8_t* nonce) {
  uint8_t d[32];
  sha256_16(nonce, d);
  for (int k = 0; k < 32; k++) acc.checksum[k] ^= d[k];
}

// Barycentric weights of gadget g at t: c_k = w^k / (t - w^k) for k = 0..calls (the wire points
// beyond `calls` are 0), L = (t^P - 1)/P. Returns false if t is a P-th root of unity.
static bool bary(const Gadget& g, u128 t, std::vector<u128>& ck, u128& L) {
  u128 tP = t;
  for (int i = 0; i < g.logP; i++) tP = fmul(tP, tP);
  if (tP == 1) return false;
  L = fmul(fsub(tP, 1), g.invP);
  const int C = g.calls;
  u128 prod = 1;
  for (int k = 0; k <= C; k++) {  // prefix products
    ck[k] = prod;
    prod = fmul(prod, fsub(t, g.omega[k]));
  }
  u128 inv = finv(prod);
  for (int k = C; k >= 0; k--) {
    const u128 den_inv = fmul(inv, ck[k]);
    inv = fmul(inv, fsub(t, g.omega[k]));
    ck[k] = fmul(g.omega[k], den_inv);
  }
  return true;
}

static u128 horner(const u128* p, int len, u128 x) {
  u128 r = 0;
  for (int m = len - 1; m >= 0; m--) r = fadd(fmul(r, x), p[m]);
  return r;
}

// in-place size-n DFT: a_j <- sum_k a_k w^{jk}
static void dft(u128* a, int n, u128 w) {
  for (int i = 1, j = 0; i < n; i++) {
    int bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (int len = 2; len <= n; len <<= 1) {
    const u128 wl = fpow(w, (u128)(n / len));
    for (int i = 0; i < n; i += len) {
      u128 ww = 1;
      for (int k = 0; k < len / 2; k++) {
        const u128 u = a[i + k], v = fmul(a[i + k + len / 2], ww);
        a[i + k] = fadd(u, v);
        a[i + k + len / 2] = fsub(u, v);
        ww = fmul(ww, wl);
      }
    }
  }
}

struct Scratch {
  std::vector<u128> meas, proof, ck, dk, ck1, sdft, ver;
};

// FlpGeneric.query on this aggregator's shares (meas, proof), num_shares = 2: the verifier share
// [v, wires(t0) .., G0(t0), (FixedPoint) wires(t1) .., G1(t1)] into z.ver. Returns false if a query
// point is a root of unity of its gadget (prepare_init fails).
static bool flp_query(const Cfg& c, Scratch& z, const u128* jr, const u128* tq) {
  const std::vector<u128>& meas = z.meas;
  const std::vector<u128>& proof = z.proof;
  std::vector<u128>& ver = z.ver;
  const Gadget& G0 = c.g[0];
  const int C = G0.calls;
  const u128 t = tq[0];
  u128 L, L1 = 0;
  if (!bary(G0, t, z.ck, L)) return false;
  if (c.ng > 1 && !bary(c.g[1], tq[1], z.ck1, L1)) return false;
  const std::vector<u128>& ck = z.ck;
  // wire_j(t) = L (c_0 seed_j + sum_k c_k x_{k,j})
  if (c.algo == A_SUM) {
    // Range2 gadget, arity 1: wire_0 = (seed, x_0 .. x_{bits-1}); v = sum_k r^k G(w^k), k = 1..bits
    W5 e;
    w5_zero(e);
    for (int k = 1; k <= C; k++) w5_mac(e, meas[k - 1], ck[k]);
    ver[1] = fmul(L, fadd(fmul(ck[0], proof[0]), w5_reduce(e)));
    // S_j = sum_{k=1..C} r^k w^{jk}: one DFT of (0, r, r^2, ..., r^C, 0, ...); G folded mod x^P - 1
    std::vector<u128>& sd = z.sdft;
    std::fill(sd.begin(), sd.end(), 0);
    u128 rk = 1;
    for (int k = 1; k <= C; k++) {
      rk = fmul(rk, jr[0]);
      sd[k] = rk;
    }
    dft(sd.data(), G0.P, G0.omega[1]);
    const u128* g = proof.data() + 1;
    u128 v = 0;
    for (int m = 0; m < G0.gpoly_len; m++) v = fadd(v, fmul(g[m], sd[m % G0.P]));
    ver[0] = v;
    ver[2] = horner(g, G0.gpoly_len, t);
    return true;
  }
  // ParallelSum(Mul, chunk) range check (SumVec, Histogram, FixedPoint gadget 0)
  const int ch = G0.chunk, A = G0.arity;
  u128 sumc = 0;
  for (int k = 1; k <= C; k++) sumc = fadd(sumc, ck[k]);
  const u128 r = jr[0];
  const u128 rc = fpow(r, (u128)ch);
  u128 rp = 1;
  for (int k = 1; k <= C; k++) {
    z.dk[k] = fmul(ck[k], rp);
    rp = fmul(rp, rc);
  }
  const u128 halfsum = fmul(sumc, c.half);
  u128 rj = r;
  for (int jj = 0; jj < ch; jj++) {
    W5 e, o;
    w5_zero(e);
    w5_zero(o);
    for (int k = 1; k <= C; k++) {
      const int idx = (k - 1) * ch + jj;
      if (idx >= c.meas_len) break;
      w5_mac(e, meas[idx], z.dk[k]);
      w5_mac(o, meas[idx], ck[k]);
    }
    const u128 E = fmul(rj, w5_reduce(e)), O = w5_reduce(o);
    rj = fmul(rj, r);
    ver[1 + 2 * jj] = fmul(L, fadd(fmul(ck[0], proof[2 * jj]), E));
    ver[2 + 2 * jj] = fmul(L, fsub(fadd(fmul(ck[0], proof[2 * jj + 1]), O), halfsum));
  }
  // range check: sum_k G0(w^k) = sum_m g_m S_m; G0(t)
  const u128* g = proof.data() + A;
  u128 range = 0;
  for (int m = 0; m < G0.gpoly_len; m++) range = fadd(range, fmul(g[m], G0.S[m]));
  ver[1 + A] = horner(g, G0.gpoly_len, t);
  if (c.algo == A_SUMVEC) {
    ver[0] = range;
  } else if (c.algo == A_HIST) {  // jr1 * range + jr1^2 * (sum x - 1/2)
    u128 sx = 0;
    for (int i = 0; i < c.meas_len; i++) sx = fadd(sx, meas[i]);
    ver[0] = fadd(fmul(jr[1], range), fmul(fmul(jr[1], jr[1]), fsub(sx, c.half)));
  } else {  // FixedPointBoundedL2VecSum: gadget 1 = ParallelSum(PolyEval(2^(2n-2) - 2^n y + y^2)) over entries
    const Gadget& G1 = c.g[1];
    const int n = c.bits, E = c.length, ch1 = G1.chunk, C1 = G1.calls, vo = 2 + A;
    const std::vector<u128>& c1 = z.ck1;
    const u128 zero_share = (u128)1 << (n - 2);  // 2^(n-1) / num_shares (2)
    const u128* p1 = proof.data() + G0.arity + G0.gpoly_len;  // [seeds (chunk1) || gadget poly]
    for (int jj = 0; jj < ch1; jj++) {
      W5 e;
      w5_zero(e);
      u128 pad = 0;
      for (int k = 1; k <= C1; k++) {
        const int idx = (k - 1) * ch1 + jj;
        if (idx < E) {
          u128 y = 0;  // decode the entry's n bits
          for (int b = n - 1; b >= 0; b--) y = fadd(fadd(y, y), meas[(size_t)idx * n + b]);
          w5_mac(e, y, c1[k]);
        } else {
          pad = fadd(pad, c1[k]);
        }
      }
      ver[vo + jj] = fmul(L1, fadd(fadd(fmul(c1[0], p1[jj]), w5_reduce(e)), fmul(pad, zero_share)));
    }
    const u128* g1 = p1 + ch1;
    u128 computed = 0;
    for (int m = 0; m < G1.gpoly_len; m++) computed = fadd(computed, fmul(g1[m], G1.S[m]));
    ver[vo + ch1] = horner(g1, G1.gpoly_len, tq[1]);
    u128 claimed = 0;
    for (int b = c.norm_bits - 1; b >= 0; b--) claimed = fadd(fadd(claimed, claimed), meas[(size_t)E * n + b]);
    ver[0] = fadd(fmul(jr[1], range), fmul(fmul(jr[1], jr[1]), fsub(computed, claimed)));
  }
  return true;
}

// FlpGeneric.decide on the combined verifier V (both shares added)
static bool flp_decide(const Cfg& c, const std::vector<u128>& V) {
  if (V[0] != 0) return false;
  if (c.algo == A_SUM) return fsub(fmul(V[1], V[1]), V[1]) == V[2];
  const int A = c.g[0].arity;
  u128 gsum = 0;
  for (int jj = 0; jj < c.g[0].chunk; jj++) gsum = fadd(gsum, fmul(V[1 + 2 * jj], V[2 + 2 * jj]));
  if (gsum != V[1 + A]) return false;
  if (c.algo != A_FIXEDPOINT) return true;
  const int n = c.bits, vo = 2 + A, ch1 = c.g[1].chunk;
  const u128 p0c = (u128)1 << (2 * n - 2), p1c = fsub(0, (u128)1 << n);
  u128 gsum1 = 0;
  for (int jj = 0; jj < ch1; jj++) {
    const u128 y = V[vo + jj];
    gsum1 = fadd(gsum1, fadd(fadd(p0c, fmul(p1c, y)), fmul(y, y)));
  }
  return gsum1 == V[vo + ch1];
}

// out_i = truncate(meas share): Histogram the share itself, else sum_b 2^b x_{i*bits+b}
static void accumulate_share(const Cfg& c, const std::vector<u128>& meas, const uint8_t* nonce, Acc& acc) {
  if (c.algo == A_HIST) {
    for (int i = 0; i < c.out_len; i++) acc.agg[i] = fadd(acc.agg[i], meas[i]);
  } else {
    for (int i = 0; i < c.out_len; i++) {
      u128 o = 0;
      for (int b = c.bits - 1; b >= 0; b--) o = fadd(fadd(o, o), meas[(size_t)i * c.bits + b]);
      acc.agg[i] = fadd(acc.agg[i], o);
    }
  }
  acc.count++;
  add_checksum(acc, nonce);
}

// XOF tail shared by both roles: corrected joint-rand seed XOF(0, DST(6), part_L || part_H), the
// joint rands from it, and the query rands XOF(vk, DST(5), [1] || nonce).
static void xof_tail(const Cfg& c, const uint8_t* part_l, const uint8_t* part_h, const uint8_t* nonce, uint8_t corr[16],
                     u128* jr, u128* tq) {
  const uint8_t zero[16] = {0}, one = 1;
  Absorb a;
  xof_start(a, c, 6, zero);
  a.put(part_l, 16);
  a.put(part_h, 16);
  a.finish();
  memcpy(corr, a.s, 16);
  Squeeze q;
  xof_start(a, c, 3, corr);
  a.put(&one, 1);
  a.finish();
  q.start(a);
  sample(q, jr, c.jr_len);
  xof_start(a, c, 5, c.vk);
  a.put(&one, 1);
  a.put(nonce, 16);
  a.finish();
  q.start(a);
  sample(q, tq, c.qr_len);
}

// Ping-pong helper step + accumulate for one Field128 report; returns the verdict (0 finished).
static int helper_report(const Cfg& c, const uint8_t* nonce, const uint8_t* ps, const uint8_t* his, const uint8_t* lps,
                         uint8_t* msg_out, Scratch& z, Acc& acc) {
  std::vector<u128>& meas = z.meas;
  // ---- measurement share fused with the joint_rand_part absorb
  Absorb a, j;
  xof_start(a, c, 1, his);
  const uint8_t one = 1;
  a.put(&one, 1);
  a.finish();
  Squeeze q;
  q.start(a);
  xof_start(j, c, 7, his + 32);
  j.put(&one, 1);
  j.put(nonce, 16);
  for (int e = 0; e < c.meas_len;) {
    uint8_t b[16];
    q.read(b, 16);
    const u128 v = ld128(b);
    if (v >= P) continue;
    meas[e++] = v;
    j.put(b, 16);
  }
  j.finish();
  uint8_t part_h[16];
  memcpy(part_h, j.s, 16);
  // ---- proof share
  xof_start(a, c, 2, his + 16);
  const uint8_t pb[2] = {1, 1};
  a.put(pb, 2);
  a.finish();
  q.start(a);
  sample(q, z.proof.data(), c.proof_len);
  // ---- corrected seed, joint rands, query rands; the prep message from the leader's part
  uint8_t corr[16], msg[16];
  u128 jr[2], tq[2];
  xof_tail(c, ps, part_h, nonce, corr, jr, tq);
  const uint8_t* lead_part = lps + (size_t)c.ver_len * 16;
  {
    const uint8_t zero[16] = {0};
    xof_start(a, c, 6, zero);
    a.put(lead_part, 16);
    a.put(part_h, 16);
    a.finish();
    memcpy(msg, a.s, 16);
  }
  if (!flp_query(c, z, jr, tq)) return 1;
  // the leader's verifier share (decode: elements >= p fail), then decide on the sum
  for (int i = 0; i < c.ver_len; i++) {
    const u128 l = ld128(lps + 16 * (size_t)i);
    if (l >= P) return 2;
    z.ver[i] = fadd(z.ver[i], l);
  }
  if (!flp_decide(c, z.ver)) return 3;
  if (memcmp(msg, corr, 16)) return 4;
  memcpy(msg_out, msg, 16);
  accumulate_share(c, meas, nonce, acc);  // BatchAggregation::merged_with
  return 0;
}

// Leader prepare_init (agg_id 0) on the explicit leader input share (meas || proof || k_blind): the
// prep share (verifier share || own joint_rand_part) and the corrected seed (the prepare state).
// Returns 0, or 1 (prepare_init failure: an element >= p, or a query point a root of unity).
static int leader_report(const Cfg& c, const uint8_t* nonce, const uint8_t* ps, const uint8_t* lis, uint8_t* prep_share,
                         uint8_t* seed_out, Scratch& z) {
  Absorb j;
  xof_start(j, c, 7, lis + (size_t)(c.meas_len + c.proof_len) * 16);
  const uint8_t zero_id = 0;
  j.put(&zero_id, 1);
  j.put(nonce, 16);
  j.put(lis, (size_t)c.meas_len * 16);
  j.finish();
  uint8_t part_l[16];
  memcpy(part_l, j.s, 16);
  bool bad = false;
  for (int i = 0; i < c.meas_len; i++) {
    z.meas[i] = ld128(lis + 16 * (size_t)i);
    bad |= z.meas[i] >= P;
  }
  for (int i = 0; i < c.proof_len; i++) {
    z.proof[i] = ld128(lis + 16 * (size_t)(c.meas_len + i));
    bad |= z.proof[i] >= P;
  }
  if (bad) return 1;
  u128 jr[2], tq[2];
  xof_tail(c, part_l, ps + 16, nonce, seed_out, jr, tq);
  if (!flp_query(c, z, jr, tq)) return 1;
  for (int i = 0; i < c.ver_len; i++) st128(prep_share + 16 * (size_t)i, z.ver[i]);
  memcpy(prep_share + 16 * (size_t)c.ver_len, part_l, 16);
  return 0;
}

// Prio3Count (Field64, no joint randomness): meas share x, proof share (s0, s1, g0, g1, g2), Mul gadget
// with one call on the square roots of unity {1, -1}: v = G(-1) - x, wire_j(t) = L (c_0 s_j + c_1 x).
static int count_report(const Cfg& c, const uint8_t* nonce, const uint8_t* his, const uint8_t* lps, Acc& acc) {
  auto stream = [&](int usage, const uint8_t* seed, const uint8_t* binder, int blen, uint64_t* out, int n) {
    Absorb a;
    xof_start(a, c, usage, seed);
    a.put(binder, blen);
    a.finish();
    Squeeze q;
    q.start(a);
    for (int i = 0; i < n;) {
      uint8_t b[8];
      q.read(b, 8);
      uint64_t v;
      memcpy(&v, b, 8);
      if (v < P64) out[i++] = v;
    }
  };
  const uint8_t one = 1, pb[2] = {1, 1};
  uint64_t x, pr[5], t;
  stream(1, his, &one, 1, &x, 1);
  stream(2, his + 16, pb, 2, pr, 5);
  uint8_t qb[17];
  qb[0] = 1;
  memcpy(qb + 1, nonce, 16);
  stream(5, c.vk, qb, 17, &t, 1);
  const uint64_t t2 = g_mul(t, t);
  if (t2 == 1) return 1;
  uint64_t ld[4];
  for (int i = 0; i < 4; i++) {
    memcpy(&ld[i], lps + 8 * i, 8);
    if (ld[i] >= P64) return 2;
  }
  const uint64_t m1 = P64 - 1;  // w = -1
  const uint64_t L = g_mul(g_sub(t2, 1), g_pow(2, P64 - 2));
  const uint64_t inv0 = g_pow(g_sub(t, 1), P64 - 2), inv1 = g_pow(g_add(t, 1), P64 - 2);  // c_0 = 1/(t-1), c_1 = -1/(t+1)
  const uint64_t c0 = inv0, c1 = g_mul(m1, inv1);
  const uint64_t w0 = g_mul(L, g_add(g_mul(c0, pr[0]), g_mul(c1, x)));
  const uint64_t w1 = g_mul(L, g_add(g_mul(c0, pr[1]), g_mul(c1, x)));
  const uint64_t v = g_sub(g_add(g_sub(pr[2], pr[3]), pr[4]), x);              // G(-1) - x
  const uint64_t Gt = g_add(g_add(pr[2], g_mul(pr[3], t)), g_mul(pr[4], t2));  // G(t)
  const uint64_t V0 = g_add(v, ld[0]), A0 = g_add(w0, ld[1]), A1 = g_add(w1, ld[2]), VG = g_add(Gt, ld[3]);
  if (V0 != 0 || g_mul(A0, A1) != VG) return 3;
  acc.agg[0] = (u128)g_add((uint64_t)acc.agg[0], x);
  acc.count++;
  add_checksum(acc, nonce);
  return 0;
}

static int cfg_make(Cfg& c, int algo, int bits, int length, int chunk, const uint8_t* vk) {
  c = Cfg();
  c.algo = algo;
  c.bits = bits;
  c.length = length;
  c.chunk = chunk;
  c.algo_id = (uint32_t)algo;
  c.ng = 1;
  c.qr_len = 1;
  c.norm_bits = 0;
  memcpy(c.vk, vk, 16);
  switch (algo) {
    case A_COUNT:
      c.meas_len = c.out_len = 1;
      c.jr_len = 0;
      c.proof_len = 5;
      c.ver_len = 4;
      c.ps_bytes = 0;
      c.his_bytes = 32;
      c.lps_bytes = 32;
      return 0;
    case A_SUM:
      if (bits < 1 || bits > 64) return -1;
      c.meas_len = bits;
      c.out_len = 1;
      c.jr_len = 1;
      gadget_make(c.g[0], 1, bits, 1);
      break;
    case A_SUMVEC:
      if (bits < 1 || bits > 64 || length < 1 || chunk < 1) return -1;
      c.meas_len = bits * length;
      c.out_len = length;
      c.jr_len = 1;
      gadget_make(c.g[0], 2 * chunk, (c.meas_len + chunk - 1) / chunk, chunk);
      break;
    case A_HIST:
      if (length < 1 || chunk < 1) return -1;
      c.bits = 1;
      c.meas_len = c.out_len = length;
      c.jr_len = 2;
      gadget_make(c.g[0], 2 * chunk, (length + chunk - 1) / chunk, chunk);
      break;
    case A_FIXEDPOINT: {  // prio 0.16.1 FixedPointBoundedL2VecSum::new, as oracle/prio3_oracle.c cfg_make
      if ((bits != 16 && bits != 32) || length < 1) return -1;
      c.algo_id = 0xFFFF0000u;
      c.norm_bits = 2 * bits - 2;
      c.meas_len = bits * length + c.norm_bits;
      c.out_len = length;
      c.jr_len = 2;
      c.qr_len = 2;
      c.ng = 2;
      const int ch0 = isqrt_floor(c.meas_len), ch1 = isqrt_floor(length);
      gadget_make(c.g[0], 2 * ch0, (c.meas_len + ch0 - 1) / ch0, ch0);
      gadget_make(c.g[1], ch1, (length + ch1 - 1) / ch1, ch1);
      break;
    }
    default:
      return -1;
  }
  c.proof_len = 0;
  c.ver_len = 1;
  for (int i = 0; i < c.ng; i++) {
    c.proof_len += c.g[i].arity + c.g[i].gpoly_len;
    c.ver_len += c.g[i].arity + 1;
  }
  c.half = finv(2);
  c.ps_bytes = 32;
  c.his_bytes = 48;
  c.lps_bytes = (size_t)c.ver_len * 16 + 16;
  return 0;
}

static void init_c256() {  // 2^256 mod p = CFOLD^2 mod p (its 256-bit product folds with CFOLD alone)
  static std::once_flag once;
  std::call_once(once, [] {
    W5 t;
    memset(t.w, 0, sizeof t.w);
    w5_mac(t, CFOLD, CFOLD);
    C256 = 0;
    C256 = w5_reduce(t);
  });
}

}  // namespace

extern "C" {

// Helper prep + aggregate of n reports (fixed-stride DAP encodings, as jx_helper_prep_aggregate).
// algo 0 = Prio3Count, 1 = Prio3Sum{bits}, 2 = Prio3SumVec{bits, length, chunk_length},
// 3 = Prio3Histogram{length, chunk_length}, 5 = Prio3FixedPointBoundedL2VecSum{bits = 16 | 32, length}.
// agg_out: out_len x field bytes LE (8 for Count, else 16); verdicts / prep_msgs nullable.
// Returns 0, or -1 on bad parameters.
int jc_helper_prep_aggregate(int algo, int bits, int length, int chunk, const uint8_t* verify_key, uint64_t n,
                             const uint8_t* nonces, const uint8_t* public_shares, const uint8_t* helper_input_shares,
                             const uint8_t* leader_prep_shares, uint8_t* verdicts, uint8_t* prep_msgs,
                             uint8_t* agg_out, uint64_t* count_out, uint8_t* checksum_out, int nthreads) {
  init_c256();
  Cfg c;
  if (cfg_make(c, algo, bits, length, chunk, verify_key)) return -1;
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n && n) nthreads = (int)n;
  std::vector<Acc> accs(nthreads);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      Acc& acc = accs[t];
      acc.agg.assign(c.out_len, 0);
      Scratch z;
      z.meas.resize(c.meas_len);
      z.proof.resize(c.proof_len);
      if (algo != A_COUNT) {
        z.ck.resize(c.g[0].calls + 1);
        z.dk.resize(c.g[0].calls + 1);
        z.sdft.resize(c.g[0].P);
        z.ver.resize(c.ver_len);
        if (c.ng > 1) z.ck1.resize(c.g[1].calls + 1);
      }
      const uint64_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
      for (uint64_t i = lo; i < hi; i++) {
        uint8_t msg[16] = {0};
        const int v = algo == A_COUNT
                          ? count_report(c, nonces + 16 * i, helper_input_shares + c.his_bytes * i,
                                         leader_prep_shares + c.lps_bytes * i, acc)
                          : helper_report(c, nonces + 16 * i, public_shares + c.ps_bytes * i,
                                          helper_input_shares + c.his_bytes * i, leader_prep_shares + c.lps_bytes * i,
                                          msg, z, acc);
        if (verdicts) verdicts[i] = (uint8_t)v;
        if (prep_msgs && algo != A_COUNT) memcpy(prep_msgs + 16 * i, msg, 16);
      }
    });
  }
  for (auto& x : th) x.join();
  std::vector<u128> agg(c.out_len, 0);
  uint64_t count = 0;
  uint8_t cs[32] = {0};
  for (auto& a : accs) {
    for (int i = 0; i < c.out_len; i++)
      agg[i] = algo == A_COUNT ? (u128)g_add((uint64_t)agg[i], (uint64_t)a.agg[i]) : fadd(agg[i], a.agg[i]);
    count += a.count;
    for (int k = 0; k < 32; k++) cs[k] ^= a.checksum[k];
  }
  if (agg_out) {
    for (int i = 0; i < c.out_len; i++) {
      if (algo == A_COUNT) {
        const uint64_t v = (uint64_t)agg[i];
        memcpy(agg_out + 8 * (size_t)i, &v, 8);
      } else {
        st128(agg_out + 16 * (size_t)i, agg[i]);
      }
    }
  }
  if (count_out) *count_out = count;
  if (checksum_out) memcpy(checksum_out, cs, 32);
  return 0;
}

// Leader prepare_init of n reports (Field128 TurboSHAKE instances: algo 1, 2, 3, 5): out_prep_shares
// (n x LPS, the payloads of PingPongMessage::Initialize), out_seeds (n x 16, the corrected joint-rand
// seeds = the prepare state), out_verdicts (0 initialized, 1 prepare_init failure).
int jc_leader_prep_init(int algo, int bits, int length, int chunk, const uint8_t* verify_key, uint64_t n,
                        const uint8_t* nonces, const uint8_t* public_shares, const uint8_t* leader_input_shares,
                        uint8_t* out_prep_shares, uint8_t* out_seeds, uint8_t* out_verdicts, int nthreads) {
  init_c256();
  Cfg c;
  if (algo == A_COUNT || cfg_make(c, algo, bits, length, chunk, verify_key)) return -1;
  const size_t lis_bytes = (size_t)(c.meas_len + c.proof_len) * 16 + 16;
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n && n) nthreads = (int)n;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      Scratch z;
      z.meas.resize(c.meas_len);
      z.proof.resize(c.proof_len);
      z.ck.resize(c.g[0].calls + 1);
      z.dk.resize(c.g[0].calls + 1);
      z.sdft.resize(c.g[0].P);
      z.ver.resize(c.ver_len);
      if (c.ng > 1) z.ck1.resize(c.g[1].calls + 1);
      const uint64_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
      for (uint64_t i = lo; i < hi; i++)
        out_verdicts[i] = (uint8_t)leader_report(c, nonces + 16 * i, public_shares + c.ps_bytes * i,
                                                 leader_input_shares + lis_bytes * i, out_prep_shares + c.lps_bytes * i,
                                                 out_seeds + 16 * i, z);
    });
  }
  for (auto& x : th) x.join();
  return 0;
}

// Leader prepare_next on the helper's prep messages + accumulate: report i finishes iff it
// initialized (init_verdicts[i] == 0), the helper did not reject it (peer_verdicts[i] == 0,
// nullable) and prep_msgs[i] equals its corrected seed; its output share is truncated from the
// explicit measurement share. out_verdicts: 0, 4 (prepare_next failure) or 5 (helper rejected).
int jc_leader_finish_aggregate(int algo, int bits, int length, int chunk, uint64_t n, const uint8_t* nonces,
                               const uint8_t* leader_input_shares, const uint8_t* seeds, const uint8_t* init_verdicts,
                               const uint8_t* prep_msgs, const uint8_t* peer_verdicts, uint8_t* out_verdicts,
                               uint8_t* agg_out, uint64_t* count_out, uint8_t* checksum_out, int nthreads) {
  init_c256();
  Cfg c;
  const uint8_t vk[16] = {0};
  if (algo == A_COUNT || cfg_make(c, algo, bits, length, chunk, vk)) return -1;
  const size_t lis_bytes = (size_t)(c.meas_len + c.proof_len) * 16 + 16;
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n && n) nthreads = (int)n;
  std::vector<Acc> accs(nthreads);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      Acc& acc = accs[t];
      acc.agg.assign(c.out_len, 0);
      std::vector<u128> meas(c.meas_len);
      const uint64_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
      for (uint64_t i = lo; i < hi; i++) {
        uint8_t v = init_verdicts[i];
        if (v == 0 && peer_verdicts && peer_verdicts[i]) v = 5;
        if (v == 0 && memcmp(prep_msgs + 16 * i, seeds + 16 * i, 16)) v = 4;
        out_verdicts[i] = v;
        if (v) continue;
        const uint8_t* ls = leader_input_shares + lis_bytes * i;
        for (int e = 0; e < c.meas_len; e++) meas[e] = ld128(ls + 16 * (size_t)e);
        accumulate_share(c, meas, nonces + 16 * i, acc);
      }
    });
  }
  for (auto& x : th) x.join();
  std::vector<u128> agg(c.out_len, 0);
  uint64_t count = 0;
  uint8_t cs[32] = {0};
  for (auto& a : accs) {
    for (int i = 0; i < c.out_len; i++) agg[i] = fadd(agg[i], a.agg[i]);
    count += a.count;
    for (int k = 0; k < 32; k++) cs[k] ^= a.checksum[k];
  }
  if (agg_out)
    for (int i = 0; i < c.out_len; i++) st128(agg_out + 16 * (size_t)i, agg[i]);
  if (count_out) *count_out = count;
  if (checksum_out) memcpy(checksum_out, cs, 32);
  return 0;
}

}  // extern "C"
