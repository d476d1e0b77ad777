// jc_cpu_engine.cpp — multithreaded CPU helper prep + aggregate for Prio3SumVec / Prio3Histogram.
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
//     report), no per-wire inverse DFT;
//   * report-parallel over std::thread, per-thread partial aggregates merged at the end.
// Checked byte-for-byte against the committed golden fixtures (tests/test_cpu_baseline.py).
#include <cstdint>
#include <cstring>
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

// ------------------------------------------------------------------ Prio3 instance
struct Cfg {
  int algo, bits, length, chunk;  // algo: 2 SumVec, 3 Histogram
  int meas_len, out_len, jr_len, calls, P, logP, arity, gpoly_len, proof_len, ver_len;
  std::vector<u128> omega, S;  // w^k (k < P), S_m = sum_{k=1..calls} w^{km}
  u128 invP, half;
  uint8_t vk[16];
};

static void xof_start(Absorb& a, const Cfg& c, int usage, const uint8_t seed[16]) {
  const uint8_t pre[9] = {8, 8, 0, 0, 0, 0, (uint8_t)c.algo, (uint8_t)(usage >> 8), (uint8_t)usage};
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

// Ping-pong helper step + accumulate for one report; returns the verdict (0 finished).
static int helper_report(const Cfg& c, const uint8_t* nonce, const uint8_t* ps, const uint8_t* his, const uint8_t* lps,
                         uint8_t* msg_out, std::vector<u128>& meas, std::vector<u128>& proof, std::vector<u128>& ck,
                         std::vector<u128>& dk, Acc& acc) {
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
  sample(q, proof.data(), c.proof_len);
  // ---- corrected joint-rand seed, joint rands, prep message, query rand
  const uint8_t zero[16] = {0};
  uint8_t corr[16], msg[16];
  xof_start(a, c, 6, zero);
  a.put(ps, 16);
  a.put(part_h, 16);
  a.finish();
  memcpy(corr, a.s, 16);
  const uint8_t* lead_part = lps + (size_t)c.ver_len * 16;
  xof_start(a, c, 6, zero);
  a.put(lead_part, 16);
  a.put(part_h, 16);
  a.finish();
  memcpy(msg, a.s, 16);
  u128 jr[2];
  xof_start(a, c, 3, corr);
  a.put(&one, 1);
  a.finish();
  q.start(a);
  sample(q, jr, c.jr_len);
  u128 t;
  xof_start(a, c, 5, c.vk);
  a.put(&one, 1);
  a.put(nonce, 16);
  a.finish();
  q.start(a);
  sample(q, &t, 1);
  // ---- FLP query by barycentric evaluation: c_k = w^k/(t - w^k), L = (t^P - 1)/P
  const int C = c.calls;
  const u128 tP = fpow(t, (u128)c.P);
  if (tP == 1) return 1;
  const u128 L = fmul(fsub(tP, 1), c.invP);
  u128 prod = 1;
  for (int k = 0; k <= C; k++) {  // prefix products
    ck[k] = prod;
    prod = fmul(prod, fsub(t, c.omega[k]));
  }
  u128 inv = finv(prod);
  u128 sumc = 0;
  for (int k = C; k >= 0; k--) {
    const u128 den_inv = fmul(inv, ck[k]);
    inv = fmul(inv, fsub(t, c.omega[k]));
    ck[k] = fmul(c.omega[k], den_inv);
    if (k) sumc = fadd(sumc, ck[k]);
  }
  const u128 r = jr[0];
  const u128 rc = fpow(r, (u128)c.chunk);
  u128 rp = 1;
  for (int k = 1; k <= C; k++) {
    dk[k] = fmul(ck[k], rp);
    rp = fmul(rp, rc);
  }
  const u128 halfsum = fmul(sumc, c.half);
  // leader verifier share (decode: elements >= p fail)
  auto lead = [&](int i, bool& bad) {
    const u128 v = ld128(lps + 16 * (size_t)i);
    if (v >= P) bad = true;
    return v;
  };
  bool bad = false;
  for (int i = 0; i < c.ver_len; i++) (void)lead(i, bad);
  if (bad) return 2;
  // wires and the gadget check sum_j Ve_j Vo_j
  const int A = c.arity, ch = c.chunk;
  u128 gsum = 0, rj = r;
  for (int jj = 0; jj < ch; jj++) {
    W5 e, o;
    w5_zero(e);
    w5_zero(o);
    for (int k = 1; k <= C; k++) {
      const int idx = (k - 1) * ch + jj;
      if (idx >= c.meas_len) break;
      w5_mac(e, meas[idx], dk[k]);
      w5_mac(o, meas[idx], ck[k]);
    }
    const u128 E = fmul(rj, w5_reduce(e)), O = w5_reduce(o);
    rj = fmul(rj, r);
    const u128 we = fmul(L, fadd(fmul(ck[0], proof[2 * jj]), E));
    const u128 wo = fmul(L, fsub(fadd(fmul(ck[0], proof[2 * jj + 1]), O), halfsum));
    const u128 ve = fadd(we, ld128(lps + 16 * (size_t)(1 + 2 * jj)));
    const u128 vo = fadd(wo, ld128(lps + 16 * (size_t)(2 + 2 * jj)));
    gsum = fadd(gsum, fmul(ve, vo));
  }
  // v (the range check's share: sum_m g_m S_m) and G(t)
  const u128* g = proof.data() + A;
  u128 v = 0, G = 0;
  for (int m = c.gpoly_len - 1; m >= 0; m--) {
    v = fadd(v, fmul(g[m], c.S[m]));
    G = fadd(fmul(G, t), g[m]);
  }
  if (c.algo == 3) {  // Histogram: jr1 * range + jr1^2 * (sum x - 1/2)
    u128 sx = 0;
    for (int i = 0; i < c.meas_len; i++) sx = fadd(sx, meas[i]);
    v = fadd(fmul(jr[1], v), fmul(fmul(jr[1], jr[1]), fsub(sx, c.half)));
  }
  const u128 V0 = fadd(v, ld128(lps)), VG = fadd(G, ld128(lps + 16 * (size_t)(A + 1)));
  if (V0 != 0 || gsum != VG) return 3;
  if (memcmp(msg, corr, 16)) return 4;
  memcpy(msg_out, msg, 16);
  // ---- accumulate (BatchAggregation::merged_with): truncate, add, count, checksum
  if (c.algo == 2) {
    for (int i = 0; i < c.out_len; i++) {
      u128 o = 0;
      for (int b = c.bits - 1; b >= 0; b--) o = fadd(fadd(o, o), meas[(size_t)i * c.bits + b]);
      acc.agg[i] = fadd(acc.agg[i], o);
    }
  } else {
    for (int i = 0; i < c.out_len; i++) acc.agg[i] = fadd(acc.agg[i], meas[i]);
  }
  acc.count++;
  uint8_t d[32];
  sha256_16(nonce, d);
  for (int k = 0; k < 32; k++) acc.checksum[k] ^= d[k];
  return 0;
}

}  // namespace

extern "C" {

// Helper prep + aggregate of n reports (fixed-stride DAP encodings, as jx_helper_prep_aggregate).
// algo 2 = Prio3SumVec{bits, length, chunk_length}, 3 = Prio3Histogram{length, chunk_length}.
// agg_out: out_len x 16 LE; verdicts / prep_msgs nullable. Returns 0, or -1 on bad parameters.
int jc_helper_prep_aggregate(int algo, int bits, int length, int chunk, const uint8_t* verify_key, uint64_t n,
                             const uint8_t* nonces, const uint8_t* public_shares, const uint8_t* helper_input_shares,
                             const uint8_t* leader_prep_shares, uint8_t* verdicts, uint8_t* prep_msgs,
                             uint8_t* agg_out, uint64_t* count_out, uint8_t* checksum_out, int nthreads) {
  if ((algo != 2 && algo != 3) || length < 1 || chunk < 1 || (algo == 2 && (bits < 1 || bits > 64))) return -1;
  Cfg c;
  c.algo = algo;
  c.bits = algo == 2 ? bits : 1;
  c.length = length;
  c.chunk = chunk;
  c.meas_len = algo == 2 ? bits * length : length;
  c.out_len = length;
  c.jr_len = algo == 2 ? 1 : 2;
  c.calls = (c.meas_len + chunk - 1) / chunk;
  c.P = 1;
  c.logP = 0;
  while (c.P < c.calls + 1) {
    c.P <<= 1;
    c.logP++;
  }
  c.arity = 2 * chunk;
  c.gpoly_len = 2 * (c.P - 1) + 1;
  c.proof_len = c.arity + c.gpoly_len;
  c.ver_len = c.arity + 2;
  memcpy(c.vk, verify_key, 16);
  {  // 2^256 mod p = CFOLD^2 mod p (its 256-bit product folds with CFOLD alone)
    W5 t;
    memset(t.w, 0, sizeof t.w);
    w5_mac(t, CFOLD, CFOLD);
    C256 = 0;
    C256 = w5_reduce(t);
  }
  // w = 7^((p-1)/2^66) ^ (2^(66 - logP))
  u128 w = fpow(7, (P - 1) >> 66);
  for (int i = 0; i < 66 - c.logP; i++) w = fmul(w, w);
  c.omega.resize(c.P);
  u128 wk = 1;
  for (int k = 0; k < c.P; k++) {
    c.omega[k] = wk;
    wk = fmul(wk, w);
  }
  c.S.resize(c.gpoly_len);
  for (int m = 0; m < c.gpoly_len; m++) {
    u128 s = 0;
    for (int k = 1; k <= c.calls; k++) s = fadd(s, c.omega[((uint64_t)k * m) % c.P]);
    c.S[m] = s;
  }
  c.invP = finv(c.P);
  c.half = finv(2);
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n && n) nthreads = (int)n;
  const size_t LPS = (size_t)c.ver_len * 16 + 16;
  std::vector<Acc> accs(nthreads);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      Acc& acc = accs[t];
      acc.agg.assign(c.out_len, 0);
      std::vector<u128> meas(c.meas_len), proof(c.proof_len), ck(c.calls + 1), dk(c.calls + 1);
      const uint64_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
      for (uint64_t i = lo; i < hi; i++) {
        uint8_t msg[16] = {0};
        const int v = helper_report(c, nonces + 16 * i, public_shares + 32 * i, helper_input_shares + 48 * i,
                                    leader_prep_shares + LPS * i, msg, meas, proof, ck, dk, acc);
        if (verdicts) verdicts[i] = (uint8_t)v;
        if (prep_msgs) memcpy(prep_msgs + 16 * i, msg, 16);
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
