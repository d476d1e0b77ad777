/*
 * prio3_oracle.c — TEST INFRASTRUCTURE ONLY (see prio3_oracle.h for who may use it).
 *
 * A deliberately literal CPU restatement of Prio3 as specified in
 * draft-irtf-cfrg-vdaf-08 and implemented by the external `prio` crate v0.16.1
 * (Cargo.lock:3435-3438; not vendored in /root/reference). Section numbers
 * refer to the VDAF-08 text; Janus call sites are cited as file:line under
 * /root/reference. The FLP is computed the way the spec writes it (record wire
 * values, interpolate by inverse DFT, evaluate by Horner) — NOT the way the GPU
 * kernels do it — so that agreement between the two is meaningful.
 *
 * Parity: UNPINNED against prio 0.16.1 (no Prio3 vectors exist in the
 * reference tree). TurboSHAKE128 is pinned by published KATs.
 */
#include "prio3_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef u128 fe; /* a field element (Field64 values live in the low 64 bits) */

/* ------------------------------------------------------------------------- */
/* Keccak-p[1600, n_r] and TurboSHAKE128 (RFC 9861; VDAF-08 §6.2.1 XofTurboShake128,
 * implemented in prio via sha3 0.10.8 / keccak 0.1.4, Cargo.lock:4252,2537).   */

static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

/* rotation offsets r[x + 5y] */
static const int KECCAK_ROT[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                   25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

static inline uint64_t rotl64(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }

void jo_keccak_p1600(uint64_t A[25], int rounds) {
  for (int ir = 24 - rounds; ir < 24; ir++) {
    uint64_t C[5], D[5], B[25];
    for (int x = 0; x < 5; x++) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
    for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; i++) A[i] ^= D[i % 5];
    /* rho + pi: B[y, 2x+3y] = rot(A[x,y], r[x,y]) */
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(A[x + 5 * y], KECCAK_ROT[x + 5 * y]);
    /* chi */
    for (int y = 0; y < 5; y++)
      for (int x = 0; x < 5; x++)
        A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
    A[0] ^= KECCAK_RC[ir];
  }
}

#define TS_RATE 168
typedef struct {
  uint64_t s[25];
  unsigned pos;
  int squeezing;
  uint8_t D;
} ts_t;

static void ts_init(ts_t *t, uint8_t D) {
  memset(t, 0, sizeof *t);
  t->D = D;
}
static inline void ts_xor_byte(ts_t *t, unsigned i, uint8_t b) { t->s[i / 8] ^= (uint64_t)b << (8 * (i % 8)); }
static inline uint8_t ts_get_byte(const ts_t *t, unsigned i) { return (uint8_t)(t->s[i / 8] >> (8 * (i % 8))); }

static void ts_absorb(ts_t *t, const uint8_t *m, size_t len) {
  for (size_t i = 0; i < len; i++) {
    ts_xor_byte(t, t->pos++, m[i]);
    if (t->pos == TS_RATE) {
      jo_keccak_p1600(t->s, 12);
      t->pos = 0;
    }
  }
}
static void ts_squeeze(ts_t *t, uint8_t *out, size_t len) {
  if (!t->squeezing) {
    ts_xor_byte(t, t->pos, t->D);
    ts_xor_byte(t, TS_RATE - 1, 0x80);
    jo_keccak_p1600(t->s, 12);
    t->pos = 0;
    t->squeezing = 1;
  }
  for (size_t i = 0; i < len; i++) {
    if (t->pos == TS_RATE) {
      jo_keccak_p1600(t->s, 12);
      t->pos = 0;
    }
    out[i] = ts_get_byte(t, t->pos++);
  }
}

void jo_turboshake128(const uint8_t *msg, size_t len, uint8_t D, uint8_t *out, size_t outlen) {
  ts_t t;
  ts_init(&t, D);
  ts_absorb(&t, msg, len);
  ts_squeeze(&t, out, outlen);
}

/* XofTurboShake128 (VDAF-08 §6.2.1): M = byte(len(dst)) || dst || seed || binder, D = 1. */
static void xof_init(ts_t *x, const uint8_t seed[16], const uint8_t *dst, size_t dst_len) {
  uint8_t l = (uint8_t)dst_len;
  ts_init(x, 1);
  ts_absorb(x, &l, 1);
  ts_absorb(x, dst, dst_len);
  ts_absorb(x, seed, 16);
}

void jo_xof_expand(const uint8_t seed[16], const uint8_t *dst, size_t dst_len, const uint8_t *binder,
                   size_t binder_len, uint8_t *out, size_t outlen) {
  ts_t x;
  xof_init(&x, seed, dst, dst_len);
  ts_absorb(&x, binder, binder_len);
  ts_squeeze(&x, out, outlen);
}

/* ------------------------------------------------------------------------- */
/* SHA-256 (FIPS 180-4): ReportIdChecksum (core/src/report_id.rs:19-42) and the HMAC of
 * XofHmacSha256Aes128.                                                        */

static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static inline uint32_t ror32(uint32_t v, int n) { return (v >> n) | (v << (32 - n)); }

static void sha256_block(uint32_t h[8], const uint8_t *blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 | (uint32_t)blk[4 * i + 2] << 8 | blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t S1 = ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + SHA_K[i] + w[i];
    uint32_t S0 = ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

typedef struct {
  uint32_t h[8];
  uint8_t buf[64];
  size_t blen;
  uint64_t total;
} sha_t;

static void sha_init(sha_t *s) {
  static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(s->h, H0, sizeof H0);
  s->blen = 0;
  s->total = 0;
}
static void sha_update(sha_t *s, const uint8_t *m, size_t len) {
  s->total += len;
  for (size_t i = 0; i < len; i++) {
    s->buf[s->blen++] = m[i];
    if (s->blen == 64) {
      sha256_block(s->h, s->buf);
      s->blen = 0;
    }
  }
}
static void sha_final(sha_t *s, uint8_t out[32]) {
  uint64_t bits = s->total * 8;
  uint8_t pad = 0x80, z = 0;
  sha_update(s, &pad, 1);
  while (s->blen != 56) sha_update(s, &z, 1);
  uint8_t L[8];
  for (int k = 0; k < 8; k++) L[k] = (uint8_t)(bits >> (56 - 8 * k));
  sha_update(s, L, 8);
  for (int k = 0; k < 8; k++) {
    out[4 * k] = (uint8_t)(s->h[k] >> 24);
    out[4 * k + 1] = (uint8_t)(s->h[k] >> 16);
    out[4 * k + 2] = (uint8_t)(s->h[k] >> 8);
    out[4 * k + 3] = (uint8_t)s->h[k];
  }
}

void jo_sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
  sha_t s;
  sha_init(&s);
  sha_update(&s, msg, len);
  sha_final(&s, out);
}

/* HMAC-SHA256 (RFC 2104) with a key of at most 64 bytes (the XOF's 32-byte seeds). */
typedef struct {
  sha_t inner;
  uint8_t okey[64];
} hmac_t;

static void hmac_init(hmac_t *m, const uint8_t *key, size_t klen) {
  uint8_t ik[64];
  memset(ik, 0, 64);
  memcpy(ik, key, klen);
  for (int i = 0; i < 64; i++) {
    m->okey[i] = ik[i] ^ 0x5c;
    ik[i] ^= 0x36;
  }
  sha_init(&m->inner);
  sha_update(&m->inner, ik, 64);
}
static void hmac_final(hmac_t *m, uint8_t tag[32]) {
  uint8_t ih[32];
  sha_final(&m->inner, ih);
  sha_t o;
  sha_init(&o);
  sha_update(&o, m->okey, 64);
  sha_update(&o, ih, 32);
  sha_final(&o, tag);
}

/* ------------------------------------------------------------------------- */
/* AES-128 (FIPS 197), byte-oriented, S-box derived from the GF(2^8) inverse.  */

static uint8_t AES_SBOX[256];
static pthread_once_t aes_once = PTHREAD_ONCE_INIT;

static uint8_t gf_mul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return r;
}
static void aes_init_sbox(void) {
  for (int x = 0; x < 256; x++) {
    uint8_t inv = 0;
    for (int y = 1; y < 256 && x; y++)
      if (gf_mul((uint8_t)x, (uint8_t)y) == 1) {
        inv = (uint8_t)y;
        break;
      }
    uint8_t s = inv;
    for (int i = 1; i <= 4; i++) s ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
    AES_SBOX[x] = s ^ 0x63;
  }
}
static void aes128_expand(const uint8_t key[16], uint8_t rk[176]) {
  pthread_once(&aes_once, aes_init_sbox);
  memcpy(rk, key, 16);
  uint8_t rcon = 1;
  for (int i = 4; i < 44; i++) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % 4 == 0) {
      uint8_t t0 = t[0];
      t[0] = AES_SBOX[t[1]] ^ rcon;
      t[1] = AES_SBOX[t[2]];
      t[2] = AES_SBOX[t[3]];
      t[3] = AES_SBOX[t0];
      rcon = gf_mul(rcon, 2);
    }
    for (int j = 0; j < 4; j++) rk[4 * i + j] = rk[4 * (i - 4) + j] ^ t[j];
  }
}
static void aes128_block(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16], t[16];
  for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
  for (int r = 1; r <= 10; r++) {
    for (int i = 0; i < 16; i++) s[i] = AES_SBOX[s[i]];
    for (int i = 0; i < 16; i++) t[i] = s[(i + 4 * (i % 4)) % 16]; /* ShiftRows, column-major s[4c+r] */
    if (r < 10) {
      for (int c = 0; c < 4; c++) {
        const uint8_t *a = t + 4 * c;
        uint8_t m0 = gf_mul(a[0], 2) ^ gf_mul(a[1], 3) ^ a[2] ^ a[3];
        uint8_t m1 = a[0] ^ gf_mul(a[1], 2) ^ gf_mul(a[2], 3) ^ a[3];
        uint8_t m2 = a[0] ^ a[1] ^ gf_mul(a[2], 2) ^ gf_mul(a[3], 3);
        uint8_t m3 = gf_mul(a[0], 3) ^ a[1] ^ a[2] ^ gf_mul(a[3], 2);
        s[4 * c] = m0;
        s[4 * c + 1] = m1;
        s[4 * c + 2] = m2;
        s[4 * c + 3] = m3;
      }
    } else {
      memcpy(s, t, 16);
    }
    for (int i = 0; i < 16; i++) s[i] ^= rk[16 * r + i];
  }
  memcpy(out, s, 16);
}

void jo_aes128_encrypt(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
  uint8_t rk[176];
  aes128_expand(key, rk);
  aes128_block(rk, in, out);
}

/* ------------------------------------------------------------------------- */
/* The Prio3 XOF, two instantiations:
 *  - XofTurboShake128 (VDAF-08 §6.2.1), SEED_SIZE 16: TurboSHAKE128(byte(len(dst)) || dst ||
 *    seed || binder, D = 1);
 *  - XofHmacSha256Aes128 (prio 0.16.1 vdaf::xof, "experimental"; Janus
 *    core/src/vdaf.rs:8,173-199), SEED_SIZE 32: tag = HMAC-SHA256(key = seed,
 *    byte(len(dst)) || dst || binder); the stream is AES-128-CTR keystream with key tag[0:16]
 *    and initial counter block tag[16:32], the low 64 bits a big-endian counter
 *    (ctr 0.9.2 Ctr64BE; aes 0.8.4 / hmac 0.12.1 per Cargo.lock:41,979,1781).      */

enum { XOF_TURBOSHAKE = 0, XOF_HMAC_AES = 1 };

typedef struct {
  int kind;
  int squeezing;
  ts_t ts;
  hmac_t mac;
  uint8_t rk[176];
  uint8_t ctr[16];
  uint8_t ks[16];
  unsigned kpos;
} xof_t;

static void xof_start(xof_t *x, int kind, const uint8_t *seed, const uint8_t *dst, size_t dst_len) {
  uint8_t l = (uint8_t)dst_len;
  x->kind = kind;
  x->squeezing = 0;
  if (kind == XOF_TURBOSHAKE) {
    xof_init(&x->ts, seed, dst, dst_len);
  } else {
    hmac_init(&x->mac, seed, 32);
    sha_update(&x->mac.inner, &l, 1);
    sha_update(&x->mac.inner, dst, dst_len);
  }
}
static void xof_update(xof_t *x, const uint8_t *m, size_t len) {
  if (x->kind == XOF_TURBOSHAKE)
    ts_absorb(&x->ts, m, len);
  else
    sha_update(&x->mac.inner, m, len);
}
static void xof_read(xof_t *x, uint8_t *out, size_t len) {
  if (x->kind == XOF_TURBOSHAKE) {
    ts_squeeze(&x->ts, out, len);
    return;
  }
  if (!x->squeezing) {
    uint8_t tag[32];
    hmac_final(&x->mac, tag);
    aes128_expand(tag, x->rk);
    memcpy(x->ctr, tag + 16, 16);
    x->kpos = 16;
    x->squeezing = 1;
  }
  for (size_t i = 0; i < len; i++) {
    if (x->kpos == 16) {
      aes128_block(x->rk, x->ctr, x->ks);
      for (int k = 15; k >= 8; k--) /* Ctr64BE: increment the low 64 bits, wrapping */
        if (++x->ctr[k] != 0) break;
      x->kpos = 0;
    }
    out[i] = x->ks[x->kpos++];
  }
}

void jo_xof_hmac_aes(const uint8_t seed[32], const uint8_t *dst, size_t dst_len, const uint8_t *binder,
                     size_t binder_len, uint8_t *out, size_t outlen) {
  xof_t x;
  xof_start(&x, XOF_HMAC_AES, seed, dst, dst_len);
  xof_update(&x, binder, binder_len);
  xof_read(&x, out, outlen);
}

/* ------------------------------------------------------------------------- */
/* Fields (VDAF-08 §6.1.2): Field64 p = 2^64-2^32+1, Field128 p = 2^128-28*2^64+1.
 * GEN = 7^((p-1)/2^GEN_LOG2). LE encoding; decode rejects values >= p.       */

typedef struct {
  int is64;
  int enc;
  fe p;
  fe gen;
  int gen_log2;
} field_t;

static const u128 P128 = (((u128)0xFFFFFFFFFFFFFFE4ULL) << 64) | 1u;
static const u128 P64 = 0xFFFFFFFF00000001ULL;

static field_t F64, F128;
static pthread_once_t fields_once = PTHREAD_ONCE_INIT;

static inline fe f_add(const field_t *F, fe a, fe b) {
  if (F->is64) {
    u128 s = a + b;
    return s >= F->p ? s - F->p : s;
  }
  u128 s = a + b;
  int carry = s < a;
  if (carry || s >= F->p) s -= F->p; /* wraps mod 2^128 correctly when carry */
  return s;
}
static inline fe f_sub(const field_t *F, fe a, fe b) { return a >= b ? a - b : a + (F->p - b); }
static inline fe f_neg(const field_t *F, fe a) { return a ? F->p - a : 0; }

static void mul_128x128(u128 a, u128 b, uint64_t z[4]) {
  uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64), b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  u128 p00 = (u128)a0 * b0, p01 = (u128)a0 * b1, p10 = (u128)a1 * b0, p11 = (u128)a1 * b1;
  u128 mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
  u128 hi = p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
  z[0] = (uint64_t)p00;
  z[1] = (uint64_t)mid;
  z[2] = (uint64_t)hi;
  z[3] = (uint64_t)(hi >> 64);
}

/* reduce a 256-bit value mod p128 by folding 2^128 == 28*2^64 - 1 (mod p) */
static fe reduce256_p128(uint64_t z[4]) {
  const u128 c = (((u128)28) << 64) - 1;
  while (z[2] | z[3]) {
    u128 H = ((u128)z[3] << 64) | z[2];
    u128 L = ((u128)z[1] << 64) | z[0];
    uint64_t t[4];
    mul_128x128(H, c, t);
    u128 lo = ((u128)t[1] << 64) | t[0];
    u128 s = lo + L;
    u128 carry = s < lo;
    u128 hi = (((u128)t[3] << 64) | t[2]) + carry;
    z[0] = (uint64_t)s;
    z[1] = (uint64_t)(s >> 64);
    z[2] = (uint64_t)hi;
    z[3] = (uint64_t)(hi >> 64);
  }
  u128 v = ((u128)z[1] << 64) | z[0];
  while (v >= P128) v -= P128;
  return v;
}

static inline fe f_mul(const field_t *F, fe a, fe b) {
  if (F->is64) return (a * b) % F->p;
  uint64_t z[4];
  mul_128x128(a, b, z);
  return reduce256_p128(z);
}

static fe f_pow(const field_t *F, fe a, u128 e) {
  fe r = 1;
  while (e) {
    if (e & 1) r = f_mul(F, r, a);
    a = f_mul(F, a, a);
    e >>= 1;
  }
  return r;
}
static fe f_inv(const field_t *F, fe a) { return f_pow(F, a, F->p - 2); }
static fe f_from_u64(const field_t *F, uint64_t v) { return (fe)v % F->p; }

/* root of unity of order 2^l */
static fe f_root(const field_t *F, int l) {
  fe r = F->gen;
  for (int i = l; i < F->gen_log2; i++) r = f_mul(F, r, r);
  return r;
}

static void init_fields(void) {
  F64.is64 = 1;
  F64.enc = 8;
  F64.p = P64;
  F64.gen_log2 = 32;
  F64.gen = f_pow(&F64, 7, (P64 - 1) >> 32);
  F128.is64 = 0;
  F128.enc = 16;
  F128.p = P128;
  F128.gen_log2 = 66;
  F128.gen = f_pow(&F128, 7, (P128 - 1) >> 66);
}

static void f_encode(const field_t *F, fe v, uint8_t *out) {
  for (int i = 0; i < F->enc; i++) out[i] = (uint8_t)(v >> (8 * i));
}
/* returns 0 on success, -1 if the encoding is >= p */
static int f_decode(const field_t *F, const uint8_t *in, fe *v) {
  fe x = 0;
  for (int i = F->enc - 1; i >= 0; i--) x = (x << 8) | in[i];
  if (x >= F->p) return -1;
  *v = x;
  return 0;
}

/* XOF.next_vec (VDAF-08 §6.2): read ENC bytes LE, mask to next_pow2(p)-1 (a no-op
 * for both fields), reject if >= p, continue the stream. */
static void xof_next_vec(const field_t *F, xof_t *x, fe *out, size_t n) {
  uint8_t buf[16];
  size_t i = 0;
  while (i < n) {
    xof_read(x, buf, (size_t)F->enc);
    fe v;
    if (f_decode(F, buf, &v) == 0) out[i++] = v;
  }
}

/* ------------------------------------------------------------------------- */
/* Prio3 configuration (VDAF-08 §7; Janus VdafInstance core/src/vdaf.rs:65-108,
 * constructors core/src/vdaf.rs:203-262).                                     */

enum { G_MUL = 0, G_RANGE2 = 1, G_PSUM_MUL = 2, G_PSUM_POLY = 3 };
#define SEED_MAX 32
#define MAX_GADGETS 2
/* Private-use algorithm id of Prio3SumVecField64MultiproofHmacSha256Aes128 (core/src/vdaf.rs:18-20). */
#define ALGO_ID_SUMVEC_F64_MULTIPROOF 0xFFFF1003u
/* Algorithm id prio 0.16.1 gives Prio3FixedPointBoundedL2VecSum (Prio3::new(.., 0xFFFF0000, ..) in
 * new_fixedpoint_boundedl2_vec_sum[_multithreaded]; the constructor Janus calls at
 * core/src/vdaf.rs:315-333 and aggregator/src/aggregator.rs:916-932). [M] */
#define ALGO_ID_FIXEDPOINT_L2 0xFFFF0000u
enum {
  USAGE_MEAS_SHARE = 1,
  USAGE_PROOF_SHARE = 2,
  USAGE_JOINT_RANDOMNESS = 3,
  USAGE_PROVE_RANDOMNESS = 4,
  USAGE_QUERY_RANDOMNESS = 5,
  USAGE_JOINT_RAND_SEED = 6,
  USAGE_JOINT_RAND_PART = 7,
};

/* One FLP gadget (VDAF-08 §7.3.2): Mul, PolyEval(x^2 - x) ("Range2"), ParallelSum(Mul, chunk) or
 * ParallelSum(PolyEval(poly), chunk). Every gadget here has degree 2. */
typedef struct {
  int kind;       /* G_* */
  int arity, degree, calls, chunk, P;
  int gpoly_len;  /* degree * (P - 1) + 1 */
  int proof_off;  /* offset of [wire seeds || gadget poly] in one proof */
  fe poly[3];     /* G_PSUM_POLY: the inner PolyEval polynomial, low degree first */
} gadget_t;

typedef struct {
  int algo, bits, length, chunk, proofs;
  uint32_t algo_id; /* the DST's algorithm id */
  int xof;          /* XOF_TURBOSHAKE or XOF_HMAC_AES */
  int seed;         /* SEED_SIZE (= verify key length): 16 or 32 */
  const field_t *F;
  int meas_len, out_len, jr_len, qr_len;
  int ng;           /* gadgets */
  gadget_t gd[MAX_GADGETS];
  int proof_len, verifier_len, prove_rand_len;
  int norm_bits;    /* FixedPointBoundedL2VecSum: bits of the claimed squared norm (2n - 2) */
} cfg_t;

static int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

static int isqrt_floor(int v) {
  int r = 0;
  while ((long long)(r + 1) * (r + 1) <= v) r++;
  return r;
}

static void gadget_init(gadget_t *g, int kind, int arity, int calls, int chunk) {
  memset(g, 0, sizeof *g);
  g->kind = kind;
  g->arity = arity;
  g->degree = 2;
  g->calls = calls;
  g->chunk = chunk;
  g->P = next_pow2(1 + calls);
  g->gpoly_len = g->degree * (g->P - 1) + 1;
}

static int cfg_make(cfg_t *c, int algo, int bits, int length, int chunk, int proofs) {
  pthread_once(&fields_once, init_fields);
  memset(c, 0, sizeof *c);
  c->algo = algo;
  c->bits = bits;
  c->length = length;
  c->chunk = chunk;
  c->proofs = proofs;
  c->algo_id = (uint32_t)algo;
  c->xof = XOF_TURBOSHAKE;
  c->seed = 16;
  c->ng = 1;
  if (proofs < 1 || proofs > 255) return -1;
  switch (algo) {
    case JO_COUNT:
      c->F = &F64;
      c->meas_len = 1;
      c->out_len = 1;
      c->jr_len = 0;
      gadget_init(&c->gd[0], G_MUL, 2, 1, 1);
      break;
    case JO_SUM:
      if (bits < 1 || bits > 64) return -1;
      c->F = &F128;
      c->meas_len = bits;
      c->out_len = 1;
      c->jr_len = 1;
      gadget_init(&c->gd[0], G_RANGE2, 1, bits, 1);
      break;
    case JO_SUMVEC_F64_MULTIPROOF: /* new_prio3_sum_vec_field64_multiproof_hmacsha256_aes128, core/src/vdaf.rs:176-199 */
      if (proofs < 2) return -1;
      c->algo_id = ALGO_ID_SUMVEC_F64_MULTIPROOF;
      c->xof = XOF_HMAC_AES;
      c->seed = 32;
      /* SumVec<Field64, ParallelSum<Field64, Mul<Field64>>> */
      __attribute__((fallthrough));
    case JO_SUMVEC:
      if (bits < 1 || bits > 64 || length < 1 || chunk < 1) return -1;
      c->F = algo == JO_SUMVEC ? &F128 : &F64;
      c->meas_len = bits * length;
      c->out_len = length;
      c->jr_len = 1;
      gadget_init(&c->gd[0], G_PSUM_MUL, 2 * chunk, (c->meas_len + chunk - 1) / chunk, chunk);
      break;
    case JO_HISTOGRAM:
      if (length < 1 || chunk < 1) return -1;
      c->F = &F128;
      c->meas_len = length;
      c->out_len = length;
      c->jr_len = 2;
      gadget_init(&c->gd[0], G_PSUM_MUL, 2 * chunk, (length + chunk - 1) / chunk, chunk);
      break;
    case JO_FIXEDPOINT_L2: {
      /* FixedPointBoundedL2VecSum<FixedI{n}<U{n-1}>, ParallelSum<PolyEval>, ParallelSum<Mul>>
       * (prio 0.16.1 flp::types::fixedpoint_l2::FixedPointBoundedL2VecSum::new(entries); Janus builds it
       * for BitSize16 / BitSize32 at aggregator/src/aggregator.rs:916-932, gadget bounds core/src/dp.rs:
       * 127-143). [M] items, restated from memory of prio 0.16.1:
       *  - input = n bits per entry (entry + 2^(n-1), LE) || 2n-2 bits of the claimed squared norm;
       *  - gadget 0 = ParallelSum(Mul, chunk0) range check of every input bit (parallel_sum_range_checks),
       *    chunk0 = max(1, floor(sqrt(n*entries + 2n-2)));
       *  - gadget 1 = ParallelSum(PolyEval(2^(2n-2) - 2^n y + y^2), chunk1) over the decoded entries y,
       *    chunk1 = max(1, floor(sqrt(entries))), short chunks padded with 2^(n-1)/num_shares;
       *  - v = jr[1] * range_check + jr[1]^2 * (computed_norm - claimed_norm); JOINT_RAND_LEN 2;
       *  - output = the decoded entries (OUTPUT_LEN = entries).
       * bits == chunk unused; entries * 2^(2n+2) must stay below p (FixedPointBoundedL2VecSum::new). */
      if ((bits != 16 && bits != 32) || length < 1) return -1;
      c->F = &F128;
      c->algo_id = ALGO_ID_FIXEDPOINT_L2;
      c->norm_bits = 2 * bits - 2;
      if ((u128)length >= (P128 >> (c->norm_bits + 4))) return -1;
      c->meas_len = bits * length + c->norm_bits;
      c->out_len = length;
      c->jr_len = 2;
      c->ng = 2;
      int ch0 = isqrt_floor(c->meas_len), ch1 = isqrt_floor(length);
      if (ch0 < 1) ch0 = 1;
      if (ch1 < 1) ch1 = 1;
      c->chunk = ch0;
      gadget_init(&c->gd[0], G_PSUM_MUL, 2 * ch0, (c->meas_len + ch0 - 1) / ch0, ch0);
      gadget_init(&c->gd[1], G_PSUM_POLY, ch1, (length + ch1 - 1) / ch1, ch1);
      /* norm_summand_poly = [2^(2n-2), -2^n, 1] */
      c->gd[1].poly[0] = ((fe)1) << (2 * bits - 2);
      c->gd[1].poly[1] = f_neg(c->F, ((fe)1) << bits);
      c->gd[1].poly[2] = 1;
      break;
    }
    default:
      return -1;
  }
  c->qr_len = c->ng; /* FlpGeneric::query_rand_len = number of gadgets */
  int off = 0;
  c->verifier_len = 1;
  for (int g = 0; g < c->ng; g++) {
    c->gd[g].proof_off = off;
    off += c->gd[g].arity + c->gd[g].gpoly_len;
    c->verifier_len += c->gd[g].arity + 1;
    c->prove_rand_len += c->gd[g].arity;
  }
  c->proof_len = off;
  return 0;
}

int jo_sizes(int algo, int bits, int length, int chunk, int proofs, uint32_t out[JO_NSIZES]) {
  cfg_t c;
  if (cfg_make(&c, algo, bits, length, chunk, proofs)) return -1;
  int E = c.F->enc, jr = c.jr_len > 0, S = c.seed;
  out[0] = c.meas_len;
  out[1] = c.out_len;
  out[2] = c.jr_len;
  out[3] = c.proof_len;
  out[4] = c.verifier_len;
  out[5] = jr ? 2 * S : 0;
  out[6] = (c.meas_len + c.proof_len * proofs) * E + (jr ? S : 0);
  out[7] = 2 * S + (jr ? S : 0);
  out[8] = c.verifier_len * proofs * E + (jr ? S : 0);
  out[9] = jr ? S : 0;
  out[10] = E;
  out[11] = S * (3 + (jr ? 2 : 0));
  out[12] = c.gd[0].arity;
  out[13] = c.gd[0].calls;
  out[14] = c.gd[0].P;
  out[15] = S;
  out[16] = S;
  out[17] = c.gd[0].chunk;
  out[18] = c.ng > 1 ? c.gd[1].arity : 0;
  out[19] = c.ng > 1 ? c.gd[1].calls : 0;
  out[20] = c.ng > 1 ? c.gd[1].P : 0;
  return 0;
}

static void dst_make(const cfg_t *c, int usage, uint8_t dst[8]) {
  /* VDAF-08 §7.2.x domain_separation_tag = format_dst(0, ID, usage): VERSION=8 */
  uint32_t id = c->algo_id;
  dst[0] = 8;
  dst[1] = 0;
  dst[2] = (uint8_t)(id >> 24);
  dst[3] = (uint8_t)(id >> 16);
  dst[4] = (uint8_t)(id >> 8);
  dst[5] = (uint8_t)id;
  dst[6] = (uint8_t)(usage >> 8);
  dst[7] = (uint8_t)usage;
}

static void expand_into_vec(const cfg_t *c, const uint8_t *seed, int usage, const uint8_t *binder, size_t blen,
                            fe *out, size_t n) {
  uint8_t dst[8];
  xof_t x;
  dst_make(c, usage, dst);
  xof_start(&x, c->xof, seed, dst, 8);
  xof_update(&x, binder, blen);
  xof_next_vec(c->F, &x, out, n);
}

/* ------------------------------------------------------------------------- */
/* Polynomials (VDAF-08 §6.1.3 poly_eval / poly_interp via the DFT over alpha). */

static fe poly_eval(const field_t *F, const fe *p, int len, fe x) {
  fe r = 0;
  for (int i = len - 1; i >= 0; i--) r = f_add(F, f_mul(F, r, x), p[i]);
  return r;
}

/* in-place DFT: X_i = sum_j x_j w^{ij}, n a power of two */
static void dft(const field_t *F, fe *a, int n, fe w) {
  for (int i = 1, j = 0; i < n; i++) {
    int bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) {
      fe t = a[i];
      a[i] = a[j];
      a[j] = t;
    }
  }
  for (int len = 2; len <= n; len <<= 1) {
    fe wl = f_pow(F, w, (u128)(n / len));
    for (int i = 0; i < n; i += len) {
      fe ww = 1;
      for (int k = 0; k < len / 2; k++) {
        fe u = a[i + k], v = f_mul(F, a[i + k + len / 2], ww);
        a[i + k] = f_add(F, u, v);
        a[i + k + len / 2] = f_sub(F, u, v);
        ww = f_mul(F, ww, wl);
      }
    }
  }
}

/* coefficients of the unique poly of degree < n with p(w^i) = vals[i] */
static void poly_interp_roots(const field_t *F, const fe *vals, fe *coef, int n, fe w) {
  memcpy(coef, vals, sizeof(fe) * n);
  dft(F, coef, n, f_inv(F, w));
  fe ninv = f_inv(F, f_from_u64(F, (uint64_t)n));
  for (int i = 0; i < n; i++) coef[i] = f_mul(F, coef[i], ninv);
}

/* ------------------------------------------------------------------------- */
/* FLP (VDAF-08 §7.3 FlpGeneric) with gadgets Mul, PolyEval(x^2-x), ParallelSum(Mul),
 * ParallelSum(PolyEval(p)). */

static fe gadget_eval(const cfg_t *c, const gadget_t *gd, const fe *x) {
  const field_t *F = c->F;
  switch (gd->kind) {
    case G_MUL:
      return f_mul(F, x[0], x[1]);
    case G_RANGE2: /* PolyEval([0,-1,1]) : x^2 - x */
      return f_sub(F, f_mul(F, x[0], x[0]), x[0]);
    case G_PSUM_MUL: {
      fe s = 0;
      for (int j = 0; j < gd->chunk; j++) s = f_add(F, s, f_mul(F, x[2 * j], x[2 * j + 1]));
      return s;
    }
    default: { /* G_PSUM_POLY: sum_j p(x_j) */
      fe s = 0;
      for (int j = 0; j < gd->chunk; j++) s = f_add(F, s, poly_eval(F, gd->poly, 3, x[j]));
      return s;
    }
  }
}

typedef struct {
  const gadget_t *gd;
  fe *wire; /* arity x P, row-major */
  int k;
  int query;
  const fe *gpoly;
  fe alpha;
} grec_t;

static fe gadget_call(const cfg_t *c, grec_t *g, const fe *inp) {
  const gadget_t *gd = g->gd;
  g->k++;
  for (int j = 0; j < gd->arity; j++) g->wire[j * gd->P + g->k] = inp[j];
  if (!g->query) return gadget_eval(c, gd, inp); /* ProveGadget */
  /* QueryGadget: gadget_poly(alpha^k) */
  return poly_eval(c->F, g->gpoly, gd->gpoly_len, f_pow(c->F, g->alpha, (u128)g->k));
}

/* ParallelSum range checks as in prio's parallel_sum_range_checks (padding with
 * (0, -1/num_shares) and no r_power update for padded slots) over input[0..len). */
static fe psum_range_checks(const cfg_t *c, grec_t *g, const fe *meas, int len, fe r, int num_shares, fe *buf) {
  const field_t *F = c->F;
  const int chunk = g->gd->chunk;
  fe shares_inv = f_inv(F, f_from_u64(F, (uint64_t)num_shares));
  fe out = 0, r_power = r;
  for (int call = 0; call < g->gd->calls; call++) {
    for (int j = 0; j < chunk; j++) {
      int idx = call * chunk + j;
      if (idx < len) {
        buf[2 * j] = f_mul(F, r_power, meas[idx]);
        buf[2 * j + 1] = f_sub(F, meas[idx], shares_inv);
        r_power = f_mul(F, r_power, r);
      } else {
        buf[2 * j] = 0;
        buf[2 * j + 1] = f_neg(F, shares_inv);
      }
    }
    out = f_add(F, out, gadget_call(c, g, buf));
  }
  return out;
}

/* Field::decode_bitvector: sum_b 2^b x_b */
static fe decode_bits(const field_t *F, const fe *x, int nbits) {
  fe acc = 0, pw = 1;
  for (int b = 0; b < nbits; b++) {
    acc = f_add(F, acc, f_mul(F, pw, x[b]));
    pw = f_add(F, pw, pw);
  }
  return acc;
}

static fe valid_eval(const cfg_t *c, grec_t *g, const fe *meas, const fe *jr, int num_shares) {
  const field_t *F = c->F;
  switch (c->algo) {
    case JO_COUNT: { /* Mul(x, x) - x */
      fe in[2] = {meas[0], meas[0]};
      return f_sub(F, gadget_call(c, &g[0], in), meas[0]);
    }
    case JO_SUM: { /* sum_i r^(i+1) * Range2(bit_i) */
      fe out = 0, r = jr[0];
      for (int i = 0; i < c->meas_len; i++) {
        out = f_add(F, out, f_mul(F, r, gadget_call(c, &g[0], &meas[i])));
        r = f_mul(F, r, jr[0]);
      }
      return out;
    }
    case JO_SUMVEC:
    case JO_SUMVEC_F64_MULTIPROOF: {
      fe *buf = calloc((size_t)c->gd[0].arity, sizeof(fe));
      fe out = psum_range_checks(c, &g[0], meas, c->meas_len, jr[0], num_shares, buf);
      free(buf);
      return out;
    }
    case JO_HISTOGRAM: {
      fe *buf = calloc((size_t)c->gd[0].arity, sizeof(fe));
      fe rc = psum_range_checks(c, &g[0], meas, c->meas_len, jr[0], num_shares, buf);
      free(buf);
      fe sc = f_neg(F, f_inv(F, f_from_u64(F, (uint64_t)num_shares)));
      for (int i = 0; i < c->meas_len; i++) sc = f_add(F, sc, meas[i]);
      return f_add(F, f_mul(F, jr[1], rc), f_mul(F, f_mul(F, jr[1], jr[1]), sc));
    }
    default: { /* FixedPointBoundedL2VecSum::valid */
      const int n = c->bits, E = c->length;
      fe *buf = calloc((size_t)c->gd[0].arity, sizeof(fe));
      /* (I) every input bit (entries and claimed norm) is 0 or 1 */
      fe range = psum_range_checks(c, &g[0], meas, c->meas_len, jr[0], num_shares, buf);
      free(buf);
      /* (II) computed squared norm: sum over the decoded entries y of 2^(2n-2) - 2^n y + y^2,
       * chunks of chunk1 entries through ParallelSum(PolyEval); a short chunk is padded with a share
       * of the encoding of 0.0, 2^(n-1) / num_shares */
      const gadget_t *g1 = &c->gd[1];
      fe zero_share = f_mul(F, ((fe)1) << (n - 1), f_inv(F, f_from_u64(F, (uint64_t)num_shares)));
      fe *in = calloc((size_t)g1->chunk, sizeof(fe));
      fe computed = 0;
      for (int k = 0; k < g1->calls; k++) {
        for (int j = 0; j < g1->chunk; j++) {
          int idx = k * g1->chunk + j;
          in[j] = idx < E ? decode_bits(F, meas + (size_t)idx * n, n) : zero_share;
        }
        computed = f_add(F, computed, gadget_call(c, &g[1], in));
      }
      free(in);
      fe claimed = decode_bits(F, meas + (size_t)E * n, c->norm_bits);
      fe norm_check = f_sub(F, computed, claimed);
      return f_add(F, f_mul(F, jr[1], range), f_mul(F, f_mul(F, jr[1], jr[1]), norm_check));
    }
  }
}

static void flp_encode(const cfg_t *c, uint64_t m, const uint64_t *vec, fe *meas) {
  const field_t *F = c->F;
  switch (c->algo) {
    case JO_COUNT:
      meas[0] = f_from_u64(F, m);
      break;
    case JO_SUM:
      for (int i = 0; i < c->bits; i++) meas[i] = (m >> i) & 1;
      break;
    case JO_SUMVEC:
    case JO_SUMVEC_F64_MULTIPROOF:
      for (int i = 0; i < c->length; i++)
        for (int j = 0; j < c->bits; j++) meas[i * c->bits + j] = (vec[i] >> j) & 1;
      break;
    case JO_HISTOGRAM:
      for (int i = 0; i < c->length; i++) meas[i] = (i == (int)m);
      break;
    default: { /* FixedPointBoundedL2VecSum::encode_measurement */
      const int n = c->bits;
      const uint64_t mask = n == 64 ? ~0ull : ((1ull << n) - 1);
      u128 norm = 0;
      for (int i = 0; i < c->length; i++) {
        /* CompatibleFloat::to_field_integer: the two's-complement bits with the sign bit flipped */
        uint64_t y = (vec[i] ^ (1ull << (n - 1))) & mask;
        for (int b = 0; b < n; b++) meas[(size_t)i * n + b] = (y >> b) & 1;
        int64_t d = (int64_t)y - (int64_t)(1ull << (n - 1)); /* compute_norm_of_entries: sum (y - 2^(n-1))^2 */
        norm += (u128)((__int128)d * d);
      }
      /* prio refuses to encode a vector whose squared norm needs more than 2n-2 bits
       * (fill_with_bitvector_representation); the oracle encodes its low bits instead, i.e. a
       * client that lies about the norm, which the FLP must reject. */
      for (int b = 0; b < c->norm_bits; b++) meas[(size_t)c->length * n + b] = (fe)((norm >> b) & 1);
    }
  }
}

static void flp_truncate(const cfg_t *c, const fe *meas, fe *out) {
  const field_t *F = c->F;
  switch (c->algo) {
    case JO_COUNT:
    case JO_HISTOGRAM:
      memcpy(out, meas, sizeof(fe) * c->out_len);
      break;
    default: /* SumVec / Sum: out_i = sum_j 2^j meas[i*bits + j]; FixedPoint: the decoded entries */
      for (int i = 0; i < c->out_len; i++) out[i] = decode_bits(F, meas + (size_t)i * c->bits, c->bits);
  }
}

/* FlpGeneric.prove (VDAF-08 §7.3.3): run the circuit with num_shares = 1, then per gadget
 * gadget_poly = G(wire polys), computed through a size-2P DFT. */
static void flp_prove(const cfg_t *c, const fe *meas, const fe *prove_rand, const fe *jr, fe *proof) {
  const field_t *F = c->F;
  grec_t g[MAX_GADGETS];
  int pr = 0;
  for (int gi = 0; gi < c->ng; gi++) {
    const gadget_t *gd = &c->gd[gi];
    g[gi] = (grec_t){gd, calloc((size_t)gd->arity * gd->P, sizeof(fe)), 0, 0, NULL, 0};
    for (int j = 0; j < gd->arity; j++) g[gi].wire[j * gd->P] = prove_rand[pr + j];
    pr += gd->arity;
  }
  (void)valid_eval(c, g, meas, jr, 1);
  pr = 0;
  for (int gi = 0; gi < c->ng; gi++) {
    const gadget_t *gd = &c->gd[gi];
    const int P = gd->P, A = gd->arity, N = 2 * P;
    const fe *wire = g[gi].wire;
    fe aP = f_root(F, __builtin_ctz((unsigned)P));
    fe aN = f_root(F, __builtin_ctz((unsigned)N));
    fe *acc = calloc((size_t)N, sizeof(fe));
    fe *e0 = calloc((size_t)N, sizeof(fe)), *e1 = calloc((size_t)N, sizeof(fe));
    fe *coef = calloc((size_t)P, sizeof(fe));
    /* wire polys evaluated at the N-th roots of unity */
#define WIRE_EVALS(dst, idx)                                   \
  do {                                                         \
    poly_interp_roots(F, &wire[(idx) * P], coef, P, aP);       \
    memset((dst), 0, sizeof(fe) * N);                          \
    memcpy((dst), coef, sizeof(fe) * P);                       \
    dft(F, (dst), N, aN);                                      \
  } while (0)
    if (gd->kind == G_RANGE2) {
      WIRE_EVALS(e0, 0);
      for (int i = 0; i < N; i++) acc[i] = f_sub(F, f_mul(F, e0[i], e0[i]), e0[i]);
    } else if (gd->kind == G_PSUM_POLY) {
      for (int j = 0; j < A; j++) {
        WIRE_EVALS(e0, j);
        for (int i = 0; i < N; i++) acc[i] = f_add(F, acc[i], poly_eval(F, gd->poly, 3, e0[i]));
      }
    } else { /* Mul / ParallelSum(Mul): pairs of wires */
      for (int j = 0; j < A / 2; j++) {
        WIRE_EVALS(e0, 2 * j);
        WIRE_EVALS(e1, 2 * j + 1);
        for (int i = 0; i < N; i++) acc[i] = f_add(F, acc[i], f_mul(F, e0[i], e1[i]));
      }
    }
#undef WIRE_EVALS
    dft(F, acc, N, f_inv(F, aN));
    fe ninv = f_inv(F, f_from_u64(F, (uint64_t)N));
    fe *pp = proof + gd->proof_off;
    for (int j = 0; j < A; j++) pp[j] = prove_rand[pr + j];
    pr += A;
    for (int i = 0; i < gd->gpoly_len; i++) pp[A + i] = f_mul(F, acc[i], ninv);
    /* degree check: coefficient 2P-1 must vanish */
    if (f_mul(F, acc[N - 1], ninv) != 0) abort();
    free(acc);
    free(e0);
    free(e1);
    free(coef);
    free(g[gi].wire);
  }
}

/* FlpGeneric.query (VDAF-08 §7.3.3). Returns 0, or -1 if some t_g is a P_g-th root of unity.
 * verifier = [v] || per gadget g: [wire_j(t_g) for j < arity_g] || gadget_poly_g(t_g). */
static int flp_query(const cfg_t *c, const fe *meas, const fe *proof, const fe *qr, const fe *jr, int num_shares,
                     fe *verifier) {
  const field_t *F = c->F;
  grec_t g[MAX_GADGETS];
  for (int gi = 0; gi < c->ng; gi++) {
    const gadget_t *gd = &c->gd[gi];
    const fe *pp = proof + gd->proof_off;
    g[gi] = (grec_t){gd, calloc((size_t)gd->arity * gd->P, sizeof(fe)), 0, 1, pp + gd->arity,
                     f_root(F, __builtin_ctz((unsigned)gd->P))};
    for (int j = 0; j < gd->arity; j++) g[gi].wire[j * gd->P] = pp[j];
  }
  verifier[0] = valid_eval(c, g, meas, jr, num_shares);
  int rc = 0, vo = 1;
  for (int gi = 0; gi < c->ng && !rc; gi++) {
    const gadget_t *gd = &c->gd[gi];
    const int P = gd->P, A = gd->arity;
    fe t = qr[gi];
    if (f_pow(F, t, (u128)P) == 1) {
      rc = -1;
      break;
    }
    fe *coef = calloc((size_t)P, sizeof(fe));
    for (int j = 0; j < A; j++) {
      poly_interp_roots(F, &g[gi].wire[j * P], coef, P, g[gi].alpha);
      verifier[vo + j] = poly_eval(F, coef, P, t);
    }
    verifier[vo + A] = poly_eval(F, g[gi].gpoly, gd->gpoly_len, t);
    vo += A + 1;
    free(coef);
  }
  for (int gi = 0; gi < c->ng; gi++) free(g[gi].wire);
  return rc;
}

static int flp_decide(const cfg_t *c, const fe *verifier) {
  if (verifier[0] != 0) return 0;
  int vo = 1;
  for (int gi = 0; gi < c->ng; gi++) {
    const gadget_t *gd = &c->gd[gi];
    if (gadget_eval(c, gd, verifier + vo) != verifier[vo + gd->arity]) return 0;
    vo += gd->arity + 1;
  }
  return 1;
}

/* ------------------------------------------------------------------------- */
/* Prio3 (VDAF-08 §7.2).                                                       */

/* Xof::derive_seed: the first SEED_SIZE bytes of the stream */
static void derive_seed(const cfg_t *c, const uint8_t *seed, int usage, const uint8_t *binder, size_t blen,
                        uint8_t *out) {
  uint8_t dst[8];
  xof_t x;
  dst_make(c, usage, dst);
  xof_start(&x, c->xof, seed, dst, 8);
  xof_update(&x, binder, blen);
  xof_read(&x, out, (size_t)c->seed);
}

static void joint_rand_part(const cfg_t *c, int agg_id, const uint8_t *blind, const fe *meas_share,
                            const uint8_t nonce[16], uint8_t *out) {
  uint8_t dst[8], b = (uint8_t)agg_id, enc[16];
  xof_t x;
  dst_make(c, USAGE_JOINT_RAND_PART, dst);
  xof_start(&x, c->xof, blind, dst, 8);
  xof_update(&x, &b, 1);
  xof_update(&x, nonce, 16);
  for (int i = 0; i < c->meas_len; i++) {
    f_encode(c->F, meas_share[i], enc);
    xof_update(&x, enc, (size_t)c->F->enc);
  }
  xof_read(&x, out, (size_t)c->seed);
}

static void joint_rand_seed(const cfg_t *c, const uint8_t *part0, const uint8_t *part1, uint8_t *out) {
  uint8_t zero[SEED_MAX] = {0}, parts[2 * SEED_MAX];
  memcpy(parts, part0, (size_t)c->seed);
  memcpy(parts + c->seed, part1, (size_t)c->seed);
  derive_seed(c, zero, USAGE_JOINT_RAND_SEED, parts, 2 * (size_t)c->seed, out);
}

static void joint_rands(const cfg_t *c, const uint8_t *seed, fe *out) {
  uint8_t binder = (uint8_t)c->proofs;
  expand_into_vec(c, seed, USAGE_JOINT_RANDOMNESS, &binder, 1, out, (size_t)c->jr_len * c->proofs);
}

static void query_rands(const cfg_t *c, const uint8_t *vk, const uint8_t nonce[16], fe *out) {
  uint8_t binder[17];
  binder[0] = (uint8_t)c->proofs;
  memcpy(binder + 1, nonce, 16);
  expand_into_vec(c, vk, USAGE_QUERY_RANDOMNESS, binder, 17, out, (size_t)c->qr_len * c->proofs);
}

static void helper_meas_share(const cfg_t *c, int agg_id, const uint8_t *seed, fe *out) {
  uint8_t binder = (uint8_t)agg_id;
  expand_into_vec(c, seed, USAGE_MEAS_SHARE, &binder, 1, out, (size_t)c->meas_len);
}

static void helper_proofs_share(const cfg_t *c, int agg_id, const uint8_t *seed, fe *out) {
  uint8_t binder[2] = {(uint8_t)c->proofs, (uint8_t)agg_id};
  expand_into_vec(c, seed, USAGE_PROOF_SHARE, binder, 2, out, (size_t)c->proof_len * c->proofs);
}

#define CFG_OR_FAIL(c)                                               \
  cfg_t c;                                                           \
  if (cfg_make(&c, algo, bits, length, chunk, proofs)) return -1;

int jo_shard(int algo, int bits, int length, int chunk, int proofs, const uint64_t *measurement,
             const uint8_t nonce[16], const uint8_t *rand, uint8_t *public_share, uint8_t *leader_input_share,
             uint8_t *helper_input_share) {
  CFG_OR_FAIL(c);
  const field_t *F = c.F;
  int E = F->enc, JR = c.jr_len > 0, S = c.seed;
  /* rand = k_helper_meas || k_helper_proofs || k_prove || [blind_L || blind_H], SEED_SIZE each */
  const uint8_t *k_hmeas = rand, *k_hproofs = rand + S, *k_prove = rand + 2 * S;
  const uint8_t *blind_l = rand + 3 * S, *blind_h = rand + 4 * S;
  fe *meas = calloc((size_t)c.meas_len, sizeof(fe)), *hmeas = calloc((size_t)c.meas_len, sizeof(fe));
  fe *proofs_v = calloc((size_t)c.proof_len * proofs, sizeof(fe));
  fe *hproofs = calloc((size_t)c.proof_len * proofs, sizeof(fe));
  fe *prove_rands = calloc((size_t)c.prove_rand_len * proofs, sizeof(fe));
  fe jr[2 * 256];
  flp_encode(&c, measurement[0], measurement, meas);
  helper_meas_share(&c, 1, k_hmeas, hmeas);
  for (int i = 0; i < c.meas_len; i++) meas[i] = f_sub(F, meas[i], hmeas[i]); /* leader share */
  uint8_t part_l[SEED_MAX], part_h[SEED_MAX];
  if (JR) {
    joint_rand_part(&c, 0, blind_l, meas, nonce, part_l);
    joint_rand_part(&c, 1, blind_h, hmeas, nonce, part_h);
    uint8_t seed[SEED_MAX];
    joint_rand_seed(&c, part_l, part_h, seed);
    joint_rands(&c, seed, jr);
  }
  {
    uint8_t binder = (uint8_t)proofs;
    expand_into_vec(&c, k_prove, USAGE_PROVE_RANDOMNESS, &binder, 1, prove_rands,
                    (size_t)c.prove_rand_len * proofs);
  }
  /* full measurement for prove */
  fe *full = calloc((size_t)c.meas_len, sizeof(fe));
  flp_encode(&c, measurement[0], measurement, full);
  for (int p = 0; p < proofs; p++)
    flp_prove(&c, full, prove_rands + p * c.prove_rand_len, jr + p * c.jr_len, proofs_v + p * c.proof_len);
  helper_proofs_share(&c, 1, k_hproofs, hproofs);
  for (int i = 0; i < c.proof_len * proofs; i++) proofs_v[i] = f_sub(F, proofs_v[i], hproofs[i]);
  /* encodings */
  if (JR) {
    memcpy(public_share, part_l, (size_t)S);
    memcpy(public_share + S, part_h, (size_t)S);
  }
  uint8_t *o = leader_input_share;
  for (int i = 0; i < c.meas_len; i++, o += E) f_encode(F, meas[i], o);
  for (int i = 0; i < c.proof_len * proofs; i++, o += E) f_encode(F, proofs_v[i], o);
  if (JR) memcpy(o, blind_l, (size_t)S);
  memcpy(helper_input_share, k_hmeas, (size_t)S);
  memcpy(helper_input_share + S, k_hproofs, (size_t)S);
  if (JR) memcpy(helper_input_share + 2 * S, blind_h, (size_t)S);
  free(meas);
  free(hmeas);
  free(proofs_v);
  free(hproofs);
  free(prove_rands);
  free(full);
  return 0;
}

static int prep_init_cfg(const cfg_t *c, const uint8_t *vk, int agg_id, const uint8_t nonce[16],
                         const uint8_t *public_share, const uint8_t *input_share, uint8_t *prep_share,
                         fe *out_share, uint8_t *corrected) {
  const field_t *F = c->F;
  int E = F->enc, JR = c->jr_len > 0, np = c->proofs, S = c->seed;
  fe *meas = calloc((size_t)c->meas_len, sizeof(fe));
  fe *proofs_v = calloc((size_t)c->proof_len * np, sizeof(fe));
  const uint8_t *blind = NULL;
  int rc = 0;
  if (agg_id == 0) {
    const uint8_t *p = input_share;
    for (int i = 0; i < c->meas_len; i++, p += E)
      if (f_decode(F, p, &meas[i])) rc = JO_PREPARE_INIT_FAILURE;
    for (int i = 0; i < c->proof_len * np; i++, p += E)
      if (f_decode(F, p, &proofs_v[i])) rc = JO_PREPARE_INIT_FAILURE;
    blind = p;
  } else {
    helper_meas_share(c, agg_id, input_share, meas);
    helper_proofs_share(c, agg_id, input_share + S, proofs_v);
    blind = input_share + 2 * S;
  }
  if (!rc) {
    flp_truncate(c, meas, out_share);
    fe jr[2 * 256] = {0}, qr[256];
    uint8_t own_part[SEED_MAX];
    if (JR) {
      uint8_t parts[2][SEED_MAX];
      joint_rand_part(c, agg_id, blind, meas, nonce, own_part);
      memcpy(parts[0], public_share, (size_t)S);
      memcpy(parts[1], public_share + S, (size_t)S);
      memcpy(parts[agg_id], own_part, (size_t)S);
      joint_rand_seed(c, parts[0], parts[1], corrected);
      joint_rands(c, corrected, jr);
    }
    query_rands(c, vk, nonce, qr);
    fe *ver = calloc((size_t)c->verifier_len * np, sizeof(fe));
    for (int p = 0; p < np && !rc; p++)
      if (flp_query(c, meas, proofs_v + p * c->proof_len, qr + p * c->qr_len, jr + p * c->jr_len, 2,
                    ver + p * c->verifier_len))
        rc = JO_PREPARE_INIT_FAILURE;
    if (!rc) {
      uint8_t *o = prep_share;
      for (int i = 0; i < c->verifier_len * np; i++, o += E) f_encode(F, ver[i], o);
      if (JR) memcpy(o, own_part, (size_t)S);
    }
    free(ver);
  }
  free(meas);
  free(proofs_v);
  return rc;
}

int jo_prep_init(int algo, int bits, int length, int chunk, int proofs, const uint8_t *verify_key, int agg_id,
                 const uint8_t nonce[16], const uint8_t *public_share, const uint8_t *input_share,
                 uint8_t *prep_share, uint8_t *out_share, uint8_t *corrected_seed) {
  CFG_OR_FAIL(c);
  fe *out = calloc((size_t)c.out_len, sizeof(fe));
  uint8_t corr[SEED_MAX] = {0};
  int rc = prep_init_cfg(&c, verify_key, agg_id, nonce, public_share, input_share, prep_share, out, corr);
  if (!rc) {
    for (int i = 0; i < c.out_len; i++) f_encode(c.F, out[i], out_share + (size_t)i * c.F->enc);
    if (corrected_seed) memcpy(corrected_seed, corr, (size_t)c.seed);
  }
  free(out);
  return rc;
}

/* decode a prep share (Prio3PrepareShare): verifiers || [joint_rand_part] */
static int decode_prep_share(const cfg_t *c, const uint8_t *b, size_t len, fe *ver, uint8_t *part) {
  int E = c->F->enc, n = c->verifier_len * c->proofs;
  size_t want = (size_t)n * E + (c->jr_len ? (size_t)c->seed : 0);
  if (len != want) return -1;
  for (int i = 0; i < n; i++)
    if (f_decode(c->F, b + (size_t)i * E, &ver[i])) return -1;
  if (c->jr_len) memcpy(part, b + (size_t)n * E, (size_t)c->seed);
  return 0;
}

static int prep_shares_to_prep_cfg(const cfg_t *c, const uint8_t *ls, size_t llen, const uint8_t *hs, size_t hlen,
                                   uint8_t *msg) {
  int n = c->verifier_len * c->proofs;
  fe *lv = calloc((size_t)n, sizeof(fe)), *hv = calloc((size_t)n, sizeof(fe));
  uint8_t lp[SEED_MAX], hp[SEED_MAX];
  int rc = 0;
  if (decode_prep_share(c, ls, llen, lv, lp) || decode_prep_share(c, hs, hlen, hv, hp)) {
    rc = JO_PREP_SHARE_DECODE_FAILURE;
  } else {
    for (int i = 0; i < n; i++) lv[i] = f_add(c->F, lv[i], hv[i]);
    for (int p = 0; p < c->proofs && !rc; p++)
      if (!flp_decide(c, lv + p * c->verifier_len)) rc = JO_PREPARE_MESSAGE_FAILURE;
    if (!rc && c->jr_len) joint_rand_seed(c, lp, hp, msg);
  }
  free(lv);
  free(hv);
  return rc;
}

int jo_prep_shares_to_prep(int algo, int bits, int length, int chunk, int proofs, const uint8_t *leader_prep_share,
                           size_t leader_len, const uint8_t *helper_prep_share, size_t helper_len,
                           uint8_t *prep_msg) {
  CFG_OR_FAIL(c);
  return prep_shares_to_prep_cfg(&c, leader_prep_share, leader_len, helper_prep_share, helper_len, prep_msg);
}

/* prio ping-pong helper_initialized + evaluate (topology::ping_pong), as called at
 * aggregator/src/aggregator.rs:1947-1956; error mapping error.rs:379-424. */
static int helper_prep_cfg(const cfg_t *c, const uint8_t *vk, const uint8_t nonce[16], const uint8_t *ps,
                           const uint8_t *his, const uint8_t *lps, size_t llen, uint8_t *msg, fe *out) {
  uint32_t sz[JO_NSIZES];
  jo_sizes(c->algo, c->bits, c->length, c->chunk, c->proofs, sz);
  uint8_t *hshare = malloc(sz[8]);
  uint8_t corrected[SEED_MAX] = {0}, m[SEED_MAX] = {0};
  int rc = prep_init_cfg(c, vk, 1, nonce, ps, his, hshare, out, corrected);
  if (!rc) {
    rc = prep_shares_to_prep_cfg(c, lps, llen, hshare, sz[8], m);
    /* prepare_next: prep_msg must equal the corrected joint-rand seed */
    if (!rc && c->jr_len && memcmp(m, corrected, (size_t)c->seed) != 0) rc = JO_PREPARE_NEXT_FAILURE;
    if (!rc && msg && c->jr_len) memcpy(msg, m, (size_t)c->seed);
  }
  free(hshare);
  return rc;
}

int jo_helper_prep(int algo, int bits, int length, int chunk, int proofs, const uint8_t *verify_key,
                   const uint8_t nonce[16], const uint8_t *public_share, const uint8_t *helper_input_share,
                   const uint8_t *leader_prep_share, size_t leader_len, uint8_t *prep_msg, uint8_t *out_share) {
  CFG_OR_FAIL(c);
  fe *out = calloc((size_t)c.out_len, sizeof(fe));
  int rc = helper_prep_cfg(&c, verify_key, nonce, public_share, helper_input_share, leader_prep_share, leader_len,
                           prep_msg, out);
  if (!rc && out_share)
    for (int i = 0; i < c.out_len; i++) f_encode(c.F, out[i], out_share + (size_t)i * c.F->enc);
  free(out);
  return rc;
}

/* ------------------------------------------------------------------------- */
/* Batched drivers (pthreads, report-parallel).                               */

typedef struct {
  const cfg_t *c;
  const uint8_t *vk;
  uint64_t lo, hi;
  const uint8_t *nonces, *ps, *his, *lps;
  uint8_t *msgs, *verdicts, *outs;
  fe *agg;
  uint64_t count;
  uint8_t checksum[32];
  /* client/leader batch */
  const uint64_t *meas;
  const uint8_t *rands;
  uint8_t *ps_out, *his_out, *lps_out, *lout;
} job_t;

static void *helper_worker(void *arg) {
  job_t *j = arg;
  const cfg_t *c = j->c;
  uint32_t sz[JO_NSIZES];
  jo_sizes(c->algo, c->bits, c->length, c->chunk, c->proofs, sz);
  fe *out = calloc((size_t)c->out_len, sizeof(fe));
  for (uint64_t r = j->lo; r < j->hi; r++) {
    uint8_t msg[SEED_MAX] = {0};
    int v = helper_prep_cfg(c, j->vk, j->nonces + 16 * r, j->ps + sz[5] * r, j->his + sz[7] * r,
                            j->lps + sz[8] * r, sz[8], msg, out);
    if (j->verdicts) j->verdicts[r] = (uint8_t)v;
    if (j->msgs && sz[9]) memcpy(j->msgs + sz[9] * r, msg, sz[9]);
    if (v == 0) {
      if (j->outs)
        for (int i = 0; i < c->out_len; i++) f_encode(c->F, out[i], j->outs + (sz[1] * r + i) * sz[10]);
      if (j->agg)
        for (int i = 0; i < c->out_len; i++) j->agg[i] = f_add(c->F, j->agg[i], out[i]);
      j->count++;
      uint8_t d[32];
      jo_sha256(j->nonces + 16 * r, 16, d);
      for (int k = 0; k < 32; k++) j->checksum[k] ^= d[k];
    }
  }
  free(out);
  return NULL;
}

int jo_helper_prep_batch(int algo, int bits, int length, int chunk, int proofs, const uint8_t *verify_key,
                         uint64_t n, const uint8_t *nonces, const uint8_t *public_shares,
                         const uint8_t *helper_input_shares, const uint8_t *leader_prep_shares, uint8_t *prep_msgs,
                         uint8_t *verdicts, uint8_t *out_shares, uint8_t *agg_out, uint64_t *count_out,
                         uint8_t *checksum_out, int nthreads) {
  CFG_OR_FAIL(c);
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n && n > 0) nthreads = (int)n;
  job_t *jobs = calloc((size_t)nthreads, sizeof(job_t));
  pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    job_t *j = &jobs[t];
    j->c = &c;
    j->vk = verify_key;
    j->lo = n * t / nthreads;
    j->hi = n * (t + 1) / nthreads;
    j->nonces = nonces;
    j->ps = public_shares;
    j->his = helper_input_shares;
    j->lps = leader_prep_shares;
    j->msgs = prep_msgs;
    j->verdicts = verdicts;
    j->outs = out_shares;
    j->agg = agg_out ? calloc((size_t)c.out_len, sizeof(fe)) : NULL;
    pthread_create(&th[t], NULL, helper_worker, j);
  }
  fe *agg = calloc((size_t)c.out_len, sizeof(fe));
  uint64_t count = 0;
  uint8_t cs[32] = {0};
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].agg) {
      for (int i = 0; i < c.out_len; i++) agg[i] = f_add(c.F, agg[i], jobs[t].agg[i]);
      free(jobs[t].agg);
    }
    count += jobs[t].count;
    for (int k = 0; k < 32; k++) cs[k] ^= jobs[t].checksum[k];
  }
  if (agg_out)
    for (int i = 0; i < c.out_len; i++) f_encode(c.F, agg[i], agg_out + (size_t)i * c.F->enc);
  if (count_out) *count_out = count;
  if (checksum_out) memcpy(checksum_out, cs, 32);
  free(agg);
  free(jobs);
  free(th);
  return 0;
}

static void *client_worker(void *arg) {
  job_t *j = arg;
  const cfg_t *c = j->c;
  uint32_t sz[JO_NSIZES];
  jo_sizes(c->algo, c->bits, c->length, c->chunk, c->proofs, sz);
  int mstride = (c->algo == JO_SUMVEC || c->algo == JO_SUMVEC_F64_MULTIPROOF || c->algo == JO_FIXEDPOINT_L2)
                    ? c->length
                    : 1;
  uint8_t *lin = malloc(sz[6]);
  uint8_t corr[SEED_MAX];
  for (uint64_t r = j->lo; r < j->hi; r++) {
    jo_shard(c->algo, c->bits, c->length, c->chunk, c->proofs, j->meas + (size_t)mstride * r, j->nonces + 16 * r,
             j->rands + (size_t)sz[11] * r, j->ps_out + (size_t)sz[5] * r, lin, j->his_out + (size_t)sz[7] * r);
    fe *out = calloc((size_t)c->out_len, sizeof(fe));
    int rc = prep_init_cfg(c, j->vk, 0, j->nonces + 16 * r, j->ps_out + (size_t)sz[5] * r, lin,
                           j->lps_out + (size_t)sz[8] * r, out, corr);
    if (rc) memset(j->lps_out + (size_t)sz[8] * r, 0xff, sz[8]);
    if (j->lout)
      for (int i = 0; i < c->out_len; i++) f_encode(c->F, out[i], j->lout + ((size_t)sz[1] * r + i) * sz[10]);
    free(out);
  }
  free(lin);
  return NULL;
}

int jo_client_leader_batch(int algo, int bits, int length, int chunk, int proofs, const uint8_t *verify_key,
                           uint64_t n, const uint64_t *measurements, const uint8_t *nonces, const uint8_t *rands,
                           uint8_t *public_shares, uint8_t *helper_input_shares, uint8_t *leader_prep_shares,
                           uint8_t *leader_out_shares, int nthreads) {
  CFG_OR_FAIL(c);
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n && n > 0) nthreads = (int)n;
  job_t *jobs = calloc((size_t)nthreads, sizeof(job_t));
  pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    job_t *j = &jobs[t];
    j->c = &c;
    j->vk = verify_key;
    j->lo = n * t / nthreads;
    j->hi = n * (t + 1) / nthreads;
    j->meas = measurements;
    j->nonces = nonces;
    j->rands = rands;
    j->ps_out = public_shares;
    j->his_out = helper_input_shares;
    j->lps_out = leader_prep_shares;
    j->lout = leader_out_shares;
    pthread_create(&th[t], NULL, client_worker, j);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
  return 0;
}

int jo_aggregate(int algo, int bits, int length, int chunk, int proofs, uint64_t n, const uint8_t *out_shares,
                 uint8_t *agg_out) {
  CFG_OR_FAIL(c);
  fe *agg = calloc((size_t)c.out_len, sizeof(fe));
  for (uint64_t r = 0; r < n; r++)
    for (int i = 0; i < c.out_len; i++) {
      fe v;
      if (f_decode(c.F, out_shares + ((size_t)r * c.out_len + i) * c.F->enc, &v)) {
        free(agg);
        return -1;
      }
      agg[i] = f_add(c.F, agg[i], v);
    }
  for (int i = 0; i < c.out_len; i++) f_encode(c.F, agg[i], agg_out + (size_t)i * c.F->enc);
  free(agg);
  return 0;
}

/* op: 0 add, 1 sub, 2 mul, 3 inv, 4 root(order 2^a[0]), 5 gen */
int jo_field_op(int field64, int op, const uint8_t *a, const uint8_t *b, uint8_t *out) {
  pthread_once(&fields_once, init_fields);
  const field_t *F = field64 ? &F64 : &F128;
  fe x = 0, y = 0, r = 0;
  if (a && op != 4 && f_decode(F, a, &x)) return -1;
  if (b && f_decode(F, b, &y)) return -1;
  switch (op) {
    case 0: r = f_add(F, x, y); break;
    case 1: r = f_sub(F, x, y); break;
    case 2: r = f_mul(F, x, y); break;
    case 3: r = f_inv(F, x); break;
    case 4: r = f_root(F, a[0]); break;
    case 5: r = F->gen; break;
    default: return -1;
  }
  f_encode(F, r, out);
  return 0;
}
