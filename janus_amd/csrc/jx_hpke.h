// jx_hpke.h — RFC 9180 base-mode HPKE open for the suite Janus uses to protect report shares:
// DHKEM(X25519, HKDF-SHA256) / HKDF-SHA256 / AES-128-GCM (core/src/hpke.rs:200-230,
// docs/samples/tasks.yaml:54-58). One report per lane; __host__ __device__ so the same code
// is unit-tested on the CPU (tests/csrc/hosttest.cpp) against oracle/hpke_oracle.py.
//
//  * X25519 (RFC 7748): field 2^255 - 19 in ten 26-bit limbs (loosely reduced, < 2^28),
//    products accumulated in 64-bit columns by v_mad_u64_u32 with no carries, reduced once per
//    multiplication (2^260 == 608 mod p). The recipient scalar is the same for every lane, so
//    the ladder's conditional swaps are wave-uniform branches.
//  * SHA-256 / HMAC / HKDF over messages whose layout is fixed at compile time (every byte
//    position is a constant after unrolling, so message buffers live in registers).
//  * AES-128 with the S-box in LDS (device) and packed-byte MixColumns; GHASH bit-serial.
#pragma once
#include "jx_sha256.h"

namespace jx {

// ============================================================================ X25519

struct fe {
  uint32_t v[10];  // value = sum v[i] 2^(26 i)
};
constexpr uint32_t M26 = (1u << 26) - 1;

JX_HD void fe_from_bytes(fe& h, const uint32_t w[8]) {  // 32 bytes LE (8 LE words); bit 255 masked
  uint64_t acc = 0;
  int nb = 0, wi = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    while (nb < 26 && wi < 8) {
      acc |= (uint64_t)(wi == 7 ? (w[7] & 0x7FFFFFFFu) : w[wi]) << nb;
      nb += 32;
      wi++;
    }
    h.v[i] = (uint32_t)(acc & M26);
    acc >>= 26;
    nb -= 26;
  }
}

// reduce 20 64-bit columns (sum c[k] 2^(26k)) to a loosely reduced element
JX_HD void fe_reduce_cols(fe& h, uint64_t c[20]) {
#pragma unroll
  for (int k = 0; k < 19; k++) {
    c[k + 1] += c[k] >> 26;
    c[k] &= M26;
  }
#pragma unroll
  for (int k = 10; k < 20; k++) c[k - 10] += 608ull * c[k];  // 2^260 == 2^5 * 19
#pragma unroll
  for (int k = 0; k < 9; k++) {
    c[k + 1] += c[k] >> 26;
    c[k] &= M26;
  }
  const uint64_t t = c[9] >> 21;  // bits >= 255
  c[9] &= (1u << 21) - 1;
  c[0] += 19 * t;
  c[1] += c[0] >> 26;
  c[0] &= M26;
#pragma unroll
  for (int k = 0; k < 10; k++) h.v[k] = (uint32_t)c[k];
}

JX_HD void fe_mul(fe& h, const fe& a, const fe& b) {
  uint64_t c[20];
#pragma unroll
  for (int k = 0; k < 20; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++)
#pragma unroll
    for (int j = 0; j < 10; j++) c[i + j] += (uint64_t)a.v[i] * b.v[j];
  fe_reduce_cols(h, c);
}
JX_HD void fe_sq(fe& h, const fe& a) {
  uint64_t c[20];
#pragma unroll
  for (int k = 0; k < 20; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    c[2 * i] += (uint64_t)a.v[i] * a.v[i];
#pragma unroll
    for (int j = i + 1; j < 10; j++) c[i + j] += (uint64_t)(2 * a.v[i]) * a.v[j];
  }
  fe_reduce_cols(h, c);
}
JX_HD void fe_mul_small(fe& h, const fe& a, uint32_t s) {
  uint64_t c[20];
#pragma unroll
  for (int k = 0; k < 10; k++) c[k] = (uint64_t)a.v[k] * s;
#pragma unroll
  for (int k = 10; k < 20; k++) c[k] = 0;
  fe_reduce_cols(h, c);
}
JX_HD void fe_add(fe& h, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = a.v[i] + b.v[i];
}
// a + 2p - b (b loosely reduced by fe_reduce_cols: limbs <= 2^26, top limb < 2^21 + small)
JX_HD void fe_sub(fe& h, const fe& a, const fe& b) {
  h.v[0] = a.v[0] + ((1u << 27) - 38) - b.v[0];
#pragma unroll
  for (int i = 1; i < 9; i++) h.v[i] = a.v[i] + ((1u << 27) - 2) - b.v[i];
  h.v[9] = a.v[9] + ((1u << 22) - 2) - b.v[9];
}

// z^(p-2) (ref10 addition chain: 254 squarings, 11 multiplications)
JX_HD void fe_sqn(fe& h, const fe& a, int n) {
  fe_sq(h, a);
  for (int i = 1; i < n; i++) fe_sq(h, h);
}
JX_HD void fe_invert(fe& out, const fe& z) {
  fe z2, z9, z11, t, z5, z10, z20, z50, z100;
  fe_sq(z2, z);
  fe_sqn(t, z2, 2);
  fe_mul(z9, t, z);
  fe_mul(z11, z9, z2);
  fe_sq(t, z11);
  fe_mul(z5, t, z9);  // z^(2^5 - 1)
  fe_sqn(t, z5, 5);
  fe_mul(z10, t, z5);  // 2^10 - 1
  fe_sqn(t, z10, 10);
  fe_mul(z20, t, z10);  // 2^20 - 1
  fe_sqn(t, z20, 20);
  fe_mul(t, t, z20);  // 2^40 - 1
  fe_sqn(t, t, 10);
  fe_mul(z50, t, z10);  // 2^50 - 1
  fe_sqn(t, z50, 50);
  fe_mul(z100, t, z50);  // 2^100 - 1
  fe_sqn(t, z100, 100);
  fe_mul(t, t, z100);  // 2^200 - 1
  fe_sqn(t, t, 50);
  fe_mul(t, t, z50);  // 2^250 - 1
  fe_sqn(t, t, 5);
  fe_mul(out, t, z11);  // 2^255 - 21
}

// canonical little-endian encoding (8 LE words)
JX_HD void fe_to_bytes(uint32_t w[8], const fe& a) {
  uint64_t c[10];
#pragma unroll
  for (int k = 0; k < 10; k++) c[k] = a.v[k];
#pragma unroll
  for (int r = 0; r < 2; r++) {  // carry, fold bits >= 255 twice: value < 2^255 + small
#pragma unroll
    for (int k = 0; k < 9; k++) {
      c[k + 1] += c[k] >> 26;
      c[k] &= M26;
    }
    const uint64_t t = c[9] >> 21;
    c[9] &= (1u << 21) - 1;
    c[0] += 19 * t;
  }
#pragma unroll
  for (int k = 0; k < 9; k++) {
    c[k + 1] += c[k] >> 26;
    c[k] &= M26;
  }
  // now 0 <= value < 2^255; subtract p if value >= p  (value + 19 >= 2^255)
  uint64_t q = c[0] + 19;
#pragma unroll
  for (int k = 1; k < 10; k++) q = c[k] + (q >> 26);
  q >>= 21;  // 1 iff value >= p
  c[0] += 19 * q;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    c[k + 1] += c[k] >> 26;
    c[k] &= M26;
  }
  c[9] &= (1u << 21) - 1;
  // pack 26-bit limbs
  uint64_t acc = 0;
  int nb = 0, wi = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    acc |= c[k] << nb;
    nb += 26;
    while (nb >= 32 && wi < 8) {
      w[wi++] = (uint32_t)acc;
      acc >>= 32;
      nb -= 32;
    }
  }
  if (wi < 8) w[wi] = (uint32_t)acc;
}

// X25519(k, u) with a wave-uniform clamped scalar k (8 LE words, bit 254 set, bits 0..2 clear)
JX_HD void x25519_ladder(uint32_t out[8], const uint32_t k[8], const uint32_t u[8]) {
  fe x1, x2, z2, x3, z3, A, AA, B, BB, E, C, D, DA, CB, t;
  fe_from_bytes(x1, u);
#pragma unroll
  for (int i = 0; i < 10; i++) {
    x2.v[i] = i == 0;
    z2.v[i] = 0;
    x3.v[i] = x1.v[i];
    z3.v[i] = i == 0;
  }
  uint32_t swap = 0;
  for (int pos = 254; pos >= 0; pos--) {
    const uint32_t kt = (k[pos >> 5] >> (pos & 31)) & 1u;
    if (swap ^ kt) {  // uniform: the scalar is the same in every lane
      fe s = x2;
      x2 = x3;
      x3 = s;
      s = z2;
      z2 = z3;
      z3 = s;
    }
    swap = kt;
    fe_add(A, x2, z2);
    fe_sq(AA, A);
    fe_sub(B, x2, z2);
    fe_sq(BB, B);
    fe_sub(E, AA, BB);
    fe_add(C, x3, z3);
    fe_sub(D, x3, z3);
    fe_mul(DA, D, A);
    fe_mul(CB, C, B);
    fe_add(t, DA, CB);
    fe_sq(x3, t);
    fe_sub(t, DA, CB);
    fe_sq(t, t);
    fe_mul(z3, x1, t);
    fe_mul(x2, AA, BB);
    fe_mul_small(t, E, 121665);
    fe_add(t, AA, t);
    fe_mul(z2, E, t);
  }
  if (swap) {
    x2 = x3;
    z2 = z3;
  }
  fe_invert(t, z2);
  fe_mul(x2, x2, t);
  fe_to_bytes(out, x2);
}

// ============================================================================ SHA-256 / HMAC

// a message of up to 128 bytes following a 64-byte prefix already absorbed into the state
// (HMAC's key block); bytes are written big-endian into 32 words at compile-time positions
struct Msg128 {
  uint32_t w[32];
};
JX_HD void m_zero(Msg128& m) {
#pragma unroll
  for (int i = 0; i < 32; i++) m.w[i] = 0;
}
JX_HD void m_byte(Msg128& m, int pos, uint32_t v) { m.w[pos >> 2] |= (v & 0xffu) << (24 - 8 * (pos & 3)); }
JX_HD int m_str(Msg128& m, int pos, const char* s) {  // string literal (compile-time)
  for (int i = 0; s[i]; i++) m_byte(m, pos++, (uint8_t)s[i]);
  return pos;
}
// 32 bytes held as 8 little-endian memory words
JX_HD int m_le32(Msg128& m, int pos, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 32; i++) m_byte(m, pos + i, w[i >> 2] >> (8 * (i & 3)));
  return pos + 32;
}
// 32 bytes held as 8 big-endian words (a SHA-256 digest)
JX_HD int m_be32(Msg128& m, int pos, const uint32_t h[8]) {
#pragma unroll
  for (int i = 0; i < 32; i++) m_byte(m, pos + i, h[i >> 2] >> (24 - 8 * (i & 3)));
  return pos + 32;
}

constexpr uint32_t SHA256_IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

JX_HD void sha256_compress(uint32_t st[8], const uint32_t* blk) {  // 16 big-endian words
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = ror32(w15, 7) ^ ror32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = ror32(w2, 17) ^ ror32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA256_K[i] + wi;
    uint32_t S0 = ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// finish a hash whose state st already absorbed one 64-byte block: message m of len bytes
JX_HD void sha256_finish64(uint32_t out[8], const uint32_t st0[8], Msg128& m, int len) {
  m_byte(m, len, 0x80);
  const int nblk = (len + 9 + 63) / 64;  // 1 or 2
  const uint64_t bits = 8ull * (64 + len);
  m.w[nblk * 16 - 2] = (uint32_t)(bits >> 32);
  m.w[nblk * 16 - 1] = (uint32_t)bits;
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = st0[i];
  sha256_compress(out, m.w);
  if (nblk == 2) sha256_compress(out, m.w + 16);
}

// HMAC-SHA256 key pads for a 32-byte key given as 8 big-endian words (RFC 2104)
JX_HD void hmac_pads(const uint32_t key[8], uint32_t ist[8], uint32_t ost[8]) {
  uint32_t bi[16], bo[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t k = i < 8 ? key[i] : 0u;
    bi[i] = k ^ 0x36363636u;
    bo[i] = k ^ 0x5c5c5c5cu;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    ist[i] = SHA256_IV[i];
    ost[i] = SHA256_IV[i];
  }
  sha256_compress(ist, bi);
  sha256_compress(ost, bo);
}
// HMAC outer hash over an inner digest
JX_HD void hmac_outer(uint32_t out[8], const uint32_t ost[8], const uint32_t inner[8]) {
  Msg128 m;
  m_zero(m);
  m_be32(m, 0, inner);
  sha256_finish64(out, ost, m, 32);
}

// ============================================================================ AES-128 / GCM

// round keys: 44 words, word = 4 bytes little-endian (byte 0 in bits 0..7)
JX_HD uint32_t sub_word(const uint8_t* sbox, uint32_t w) {
  return (uint32_t)sbox[w & 0xff] | ((uint32_t)sbox[(w >> 8) & 0xff] << 8) | ((uint32_t)sbox[(w >> 16) & 0xff] << 16) |
         ((uint32_t)sbox[w >> 24] << 24);
}
JX_HD void aes128_expand_key(const uint8_t* sbox, const uint32_t key[4], uint32_t rk[44]) {
#pragma unroll
  for (int i = 0; i < 4; i++) rk[i] = key[i];
  uint32_t rcon = 1;
#pragma unroll
  for (int i = 4; i < 44; i++) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = sub_word(sbox, (t >> 8) | (t << 24)) ^ rcon;
      rcon = (rcon << 1) ^ ((rcon >> 7) * 0x11bu);
    }
    rk[i] = rk[i - 4] ^ t;
  }
}
JX_HD uint32_t xtime4(uint32_t x) { return ((x & 0x7f7f7f7fu) << 1) ^ (((x >> 7) & 0x01010101u) * 0x1bu); }
// one 16-byte block as 4 little-endian column words
JX_HD void aes128_encrypt(const uint8_t* sbox, const uint32_t rk[44], const uint32_t in[4], uint32_t out[4]) {
  uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
  for (int r = 1; r <= 10; r++) {
    // SubBytes + ShiftRows: row i of column c comes from column (c + i) mod 4
    uint32_t t0 = (uint32_t)sbox[s0 & 0xff] | ((uint32_t)sbox[(s1 >> 8) & 0xff] << 8) |
                  ((uint32_t)sbox[(s2 >> 16) & 0xff] << 16) | ((uint32_t)sbox[s3 >> 24] << 24);
    uint32_t t1 = (uint32_t)sbox[s1 & 0xff] | ((uint32_t)sbox[(s2 >> 8) & 0xff] << 8) |
                  ((uint32_t)sbox[(s3 >> 16) & 0xff] << 16) | ((uint32_t)sbox[s0 >> 24] << 24);
    uint32_t t2 = (uint32_t)sbox[s2 & 0xff] | ((uint32_t)sbox[(s3 >> 8) & 0xff] << 8) |
                  ((uint32_t)sbox[(s0 >> 16) & 0xff] << 16) | ((uint32_t)sbox[s1 >> 24] << 24);
    uint32_t t3 = (uint32_t)sbox[s3 & 0xff] | ((uint32_t)sbox[(s0 >> 8) & 0xff] << 8) |
                  ((uint32_t)sbox[(s1 >> 16) & 0xff] << 16) | ((uint32_t)sbox[s2 >> 24] << 24);
    if (r != 10) {  // MixColumns: b_i = 2(a_i ^ a_{i+1}) ^ a_{i+1} ^ a_{i+2} ^ a_{i+3}
      uint32_t c[4] = {t0, t1, t2, t3};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t w = c[q];
        const uint32_t r1 = (w >> 8) | (w << 24), r2 = (w >> 16) | (w << 16), r3 = (w >> 24) | (w << 8);
        c[q] = xtime4(w ^ r1) ^ r1 ^ r2 ^ r3;
      }
      t0 = c[0];
      t1 = c[1];
      t2 = c[2];
      t3 = c[3];
    }
    s0 = t0 ^ rk[4 * r];
    s1 = t1 ^ rk[4 * r + 1];
    s2 = t2 ^ rk[4 * r + 2];
    s3 = t3 ^ rk[4 * r + 3];
  }
  out[0] = s0;
  out[1] = s1;
  out[2] = s2;
  out[3] = s3;
}

// GF(2^128) multiply in GCM's bit order; operands as 4 big-endian words (x[0] = bytes 0..3)
JX_HD void ghash_mul(uint32_t x[4], const uint32_t h[4]) {
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0, v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3];
#pragma unroll 1
  for (int i = 0; i < 128; i++) {
    const uint32_t bit = (x[i >> 5] >> (31 - (i & 31))) & 1u;
    const uint32_t m = 0u - bit;
    z0 ^= v0 & m;
    z1 ^= v1 & m;
    z2 ^= v2 & m;
    z3 ^= v3 & m;
    const uint32_t lsb = v3 & 1u;
    v3 = (v3 >> 1) | (v2 << 31);
    v2 = (v2 >> 1) | (v1 << 31);
    v1 = (v1 >> 1) | (v0 << 31);
    v0 = (v0 >> 1) ^ ((0u - lsb) & 0xE1000000u);
  }
  x[0] = z0;
  x[1] = z1;
  x[2] = z2;
  x[3] = z3;
}

}  // namespace jx
