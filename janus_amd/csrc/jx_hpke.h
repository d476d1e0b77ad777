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
//  * SHA-256 / HMAC and AES-128 come from jx_sha_aes.h; GHASH is bit-serial.
#pragma once
#include "jx_sha_aes.h"

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

// Reduce the 64-bit columns of a product (sum c[k] 2^(26k), k < 19; the inputs' limbs < 2^28, so every column
// < 10 * 2^56 < 2^59.4) to a loosely reduced element. One open is ~2,800 of these in a chain, and the wave issues
// them alone on its SIMD, so the count of instructions is the time: the high columns fold down first, split at
// bit 26 (2^260 == 608: the low part to k - 10, the high part to k - 9; no column can overflow), then ONE carry
// chain over the ten limbs and the carry out of bit 255 back x19 (instead of a 19-limb chain before the fold and a
// second chain after it). Out: limb 0 < 2^26, limb 1 < 2^26 + 2^17, limbs 2..8 < 2^26, limb 9 < 2^21 (fe_sub's 2p
// needs <= 2^27 - 38, 2^27 - 2, 2^22 - 2).
JX_HD void fe_reduce_cols(fe& h, uint64_t c[20]) {
#pragma unroll
  for (int k = 10; k < 19; k++) {
    c[k - 10] += 608ull * (c[k] & M26);
    c[k - 9] += 608ull * (c[k] >> 26);
  }
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
