// jx_field.h — Field64 / Field128 arithmetic for the gfx950 Prio3 engine.
//
// Fields are those of VDAF-08 §6.1.2 as used by prio 0.16.1 (Janus pins prio at
// /root/reference/Cargo.toml:50): Field64 p = 2^64 - 2^32 + 1 (Prio3Count),
// Field128 p = 2^128 - 28*2^64 + 1 (Prio3Sum/SumVec/Histogram, core/src/vdaf.rs:203-262).
//
// Field128 representation: four 32-bit limbs (the native VALU width) in a
// struct of two uint64 halves. Products use Montgomery multiplication with
// R = 2^128: since p == 1 (mod 2^64), -p^-1 mod 2^64 = -1 and m*p needs only a
// multiply by 28, so each of the two 64-bit REDC steps is a handful of adds.
// Values that stream through HBM (measurement shares, output shares, verifier
// shares) stay canonical; per-report coefficients are stored in Montgomery form
// so that mont(x_canonical, c*R) = x*c comes out canonical with ONE reduction.
//
// Everything here is __host__ __device__ so the exact same code is unit-tested
// on the CPU (tests/csrc/hosttest.cpp) before it runs on the GPU.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define JX_HD __host__ __device__ __forceinline__
#else
#define JX_HD static inline
#endif

namespace jx {

// ----------------------------------------------------------------------------
// 128-bit helpers

struct f128 {
  uint64_t lo, hi;
};

// 3-input XOR and majority: one v_bitop3_b32 each on gfx950 (the compiler does not always fuse them)
#if defined(__HIP_DEVICE_COMPILE__)
JX_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
JX_HD uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8); }
#else
JX_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }
JX_HD uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) { return (a & b) ^ (a & c) ^ (b & c); }
#endif
JX_HD uint32_t lo32(uint64_t v) { return (uint32_t)v; }
JX_HD uint32_t hi32(uint64_t v) { return (uint32_t)(v >> 32); }

// add with carry-out
JX_HD uint64_t addc64(uint64_t a, uint64_t b, uint32_t& carry) {
  uint64_t s = a + b;
  uint32_t c1 = s < a;
  uint64_t s2 = s + carry;
  uint32_t c2 = s2 < s;
  carry = c1 | c2;
  return s2;
}
JX_HD uint64_t subb64(uint64_t a, uint64_t b, uint32_t& borrow) {
  uint64_t d = a - b;
  uint32_t b1 = a < b;
  uint64_t d2 = d - borrow;
  uint32_t b2 = d < (uint64_t)borrow;
  borrow = b1 | b2;
  return d2;
}

// Field128 modulus p = 2^128 - 28*2^64 + 1
constexpr uint64_t P128_LO = 1ull;
constexpr uint64_t P128_HI = 0xFFFFFFFFFFFFFFE4ull;

JX_HD f128 make128(uint64_t lo, uint64_t hi) {
  f128 r;
  r.lo = lo;
  r.hi = hi;
  return r;
}
JX_HD bool eq128(f128 a, f128 b) { return a.lo == b.lo && a.hi == b.hi; }
JX_HD bool is_zero128(f128 a) { return (a.lo | a.hi) == 0; }
JX_HD bool ge_p128(f128 a) { return a.hi > P128_HI || (a.hi == P128_HI && a.lo >= P128_LO); }

// canonical modular add / sub
JX_HD f128 add128(f128 a, f128 b) {
  uint32_t c = 0;
  uint64_t lo = addc64(a.lo, b.lo, c);
  uint64_t hi = addc64(a.hi, b.hi, c);
  // s - p
  uint32_t br = 0;
  uint64_t dlo = subb64(lo, P128_LO, br);
  uint64_t dhi = subb64(hi, P128_HI, br);
  bool take = c || !br;  // sum >= p
  return make128(take ? dlo : lo, take ? dhi : hi);
}
JX_HD f128 sub128(f128 a, f128 b) {
  uint32_t br = 0;
  uint64_t lo = subb64(a.lo, b.lo, br);
  uint64_t hi = subb64(a.hi, b.hi, br);
  if (br) {  // add p back
    uint32_t c = 0;
    lo = addc64(lo, P128_LO, c);
    hi = addc64(hi, P128_HI, c);
  }
  return make128(lo, hi);
}
JX_HD f128 neg128(f128 a) { return sub128(make128(0, 0), a); }

// full 128x128 -> 256 product, 32-bit limb schoolbook (16 v_mad_u64_u32 on gfx950)
JX_HD void mul128_full(f128 a, f128 b, uint64_t z[4]) {
  const uint32_t A[4] = {lo32(a.lo), hi32(a.lo), lo32(a.hi), hi32(a.hi)};
  const uint32_t B[4] = {lo32(b.lo), hi32(b.lo), lo32(b.hi), hi32(b.hi)};
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint64_t t = (uint64_t)A[i] * B[j] + ((uint64_t)r[i + j] + carry);
      r[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    r[i + 4] = (uint32_t)carry;
  }
  z[0] = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
  z[1] = (uint64_t)r[2] | ((uint64_t)r[3] << 32);
  z[2] = (uint64_t)r[4] | ((uint64_t)r[5] << 32);
  z[3] = (uint64_t)r[6] | ((uint64_t)r[7] << 32);
}

JX_HD uint64_t umulhi64_28(uint64_t m) {
  // floor(28*m / 2^64): 28m = 32m - 4m
  // computed exactly with 32-bit pieces
  uint64_t lo = (uint64_t)lo32(m) * 28u;
  uint64_t hi = (uint64_t)hi32(m) * 28u + (lo >> 32);
  return hi >> 32;
}

// One 64-bit Montgomery REDC step for p = 2^128 - 28*2^64 + 1 (p' = -1 mod 2^64):
// T' = (T + m*p) / 2^64 with m = -T0 mod 2^64.  m*p = m*2^128 - 28m*2^64 + m, so
// T' = T[1..] + carry(T0 != 0) + m*(2^64 - 28).
JX_HD void redc_step(uint64_t& t0, uint64_t& t1, uint64_t& t2, uint64_t& t3) {
  uint64_t m = 0 - t0;
  uint32_t c = t0 != 0;
  uint64_t v = m * 28u;          // low 64 bits of 28m
  uint64_t u = umulhi64_28(m);   // high bits of 28m
  uint64_t q_lo = 0 - v;         // m*(2^64-28) = (m - u - (v!=0)) * 2^64 + (2^64 - v)
  uint64_t q_hi = m - u - (uint64_t)(v != 0);
  // (t1, t2, t3) + (q_lo, q_hi, 0) + c
  uint64_t n0 = addc64(t1, q_lo, c);
  uint64_t n1 = addc64(t2, q_hi, c);
  uint64_t n2 = t3 + c;
  t0 = n0;
  t1 = n1;
  t2 = n2;
  t3 = 0;
}

// 32-bit add / subtract with carry (borrow) in and out: v_add_co / v_addc / v_sub_co / v_subb chains on the
// device (the 64-bit forms above compile to 64-bit adds plus 64-bit compares for the carries)
JX_HD uint32_t adc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_addc(a, b, cin, &cout);
#else
  const uint64_t s = (uint64_t)a + b + cin;
  cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}
JX_HD uint32_t sbb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_subc(a, b, bin, &bout);
#else
  const uint64_t d = (uint64_t)a - b - bin;
  bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
#endif
}
// acc += x * y (64-bit), the carry out of 2^64 counted into top. On the device one v_mad_u64_u32 with its
// carry-out SGPR pair feeding one v_addc_co_u32 (the compiler cannot see the mad's carry-out and would
// test t < acc with a 64-bit compare and a select instead).
JX_HD void mac_c(uint64_t& acc, uint32_t& top, uint32_t x, uint32_t y) {
#ifdef __HIP_DEVICE_COMPILE__
  uint64_t co;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(acc), "=s"(co) : "v"(x), "v"(y), "v"(acc));
  asm("v_addc_co_u32 %0, vcc, 0, %1, %2" : "=v"(top) : "v"(top), "s"(co) : "vcc");
#else
  const uint64_t t = (uint64_t)x * y + acc;
  top += t < acc;
  acc = t;
#endif
}

// Montgomery product a*b*2^-128 mod p, canonical output (inputs < p). The 256-bit product is formed
// column by column (product scanning: a 64-bit column sum plus a carry count, so no per-product carry
// word needs a zero-extending move), then two 64-bit REDC steps (see redc_step) and one conditional
// subtraction, all on 32-bit add/sub-with-carry chains: 71 VALU on gfx950 against 123 for the 64-bit
// formulation (mul128_full + redc_step, kept for mont128_lazy). Host-tested against Python integers
// (tests/test_device_math_host.py, the same code with portable mac_c / adc32 / sbb32).
JX_HD f128 mont128(f128 a, f128 b) {
  const uint32_t A0 = lo32(a.lo), A1 = hi32(a.lo), A2 = lo32(a.hi), A3 = hi32(a.hi);
  const uint32_t B0 = lo32(b.lo), B1 = hi32(b.lo), B2 = lo32(b.hi), B3 = hi32(b.hi);
  uint32_t t[8];
  uint64_t acc = (uint64_t)A0 * B0;
  uint32_t top;
  t[0] = (uint32_t)acc;
  acc >>= 32;
  top = 0;
  mac_c(acc, top, A0, B1);
  mac_c(acc, top, A1, B0);
  t[1] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)top << 32);
  top = 0;
  mac_c(acc, top, A0, B2);
  mac_c(acc, top, A1, B1);
  mac_c(acc, top, A2, B0);
  t[2] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)top << 32);
  top = 0;
  mac_c(acc, top, A0, B3);
  mac_c(acc, top, A1, B2);
  mac_c(acc, top, A2, B1);
  mac_c(acc, top, A3, B0);
  t[3] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)top << 32);
  top = 0;
  mac_c(acc, top, A1, B3);
  mac_c(acc, top, A2, B2);
  mac_c(acc, top, A3, B1);
  t[4] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)top << 32);
  top = 0;
  mac_c(acc, top, A2, B3);
  mac_c(acc, top, A3, B2);
  t[5] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)top << 32);
  acc = (uint64_t)A3 * B3 + acc;  // the top column: the product is < 2^256, so this sum is < 2^64
  t[6] = (uint32_t)acc;
  t[7] = (uint32_t)(acc >> 32);
  // two REDC steps of 64 bits: T' = T / 2^64 + (T0 != 0) + m (2^64 - 28), m = -T0 mod 2^64 (-1/p = -1 mod 2^64)
#pragma unroll
  for (int s = 0; s < 2; s++) {
    uint32_t c, b1, b2, k;
    const uint32_t m0 = sbb32(0u, t[0], 0u, b1);
    const uint32_t m1 = sbb32(0u, t[1], b1, c);  // c = (T0 != 0)
    const uint64_t p0 = (uint64_t)m0 * 28u;      // 28 m = u 2^64 + (v1, v0)
    const uint64_t p1 = (uint64_t)m1 * 28u + (p0 >> 32);
    const uint32_t v0 = (uint32_t)p0, v1 = (uint32_t)p1, u = (uint32_t)(p1 >> 32);
    // m (2^64 - 28) = (m - u - (v != 0)) 2^64 + (2^64 - v)
    const uint32_t ql0 = sbb32(0u, v0, 0u, b1);
    const uint32_t ql1 = sbb32(0u, v1, b1, b2);  // b2 = (v != 0)
    const uint32_t qh0 = sbb32(m0, u, b2, b1);
    const uint32_t qh1 = sbb32(m1, 0u, b1, b2);
    const uint32_t n0 = adc32(t[2], ql0, c, k);
    const uint32_t n1 = adc32(t[3], ql1, k, k);
    const uint32_t n2 = adc32(t[4], qh0, k, k);
    const uint32_t n3 = adc32(t[5], qh1, k, k);
    const uint32_t n4 = adc32(t[6], 0u, k, k);
    const uint32_t n5 = t[7] + k;
    t[0] = n0;
    t[1] = n1;
    t[2] = n2;
    t[3] = n3;
    t[4] = n4;
    t[5] = n5;
    t[6] = 0;
    t[7] = 0;
  }
  // (t0..t3) + t4 2^128 < 2p: subtract p = (1, 0, 2^32 - 28, 2^32 - 1) once if the value is >= p
  uint32_t br;
  const uint32_t d0 = sbb32(t[0], 1u, 0u, br);
  const uint32_t d1 = sbb32(t[1], 0u, br, br);
  const uint32_t d2 = sbb32(t[2], 0xFFFFFFE4u, br, br);
  const uint32_t d3 = sbb32(t[3], 0xFFFFFFFFu, br, br);
  const bool take = t[4] != 0 || !br;
  return make128(take ? ((uint64_t)d1 << 32 | d0) : ((uint64_t)t[1] << 32 | t[0]),
                 take ? ((uint64_t)d3 << 32 | d2) : ((uint64_t)t[3] << 32 | t[2]));
}

// Montgomery product without the final subtraction: result < 2p, returned as
// (lo, hi, top) with top in {0,1}. For lazy accumulation.
JX_HD void mont128_lazy(f128 a, f128 b, uint64_t& lo, uint64_t& hi, uint32_t& top) {
  uint64_t z[4];
  mul128_full(a, b, z);
  uint64_t t0 = z[0], t1 = z[1], t2 = z[2], t3 = z[3];
  redc_step(t0, t1, t2, t3);
  redc_step(t0, t1, t2, t3);
  lo = t0;
  hi = t1;
  top = (uint32_t)t2;
}

// R^2 mod p (R = 2^128), for to_mont
constexpr uint64_t R2_128_LO = 0xfffffffffffffcf1ull;  // 2^256 mod p (checked in tests)
constexpr uint64_t R2_128_HI = 0x0000000000005587ull;
// R mod p = 2^128 - p = 28*2^64 - 1 : Montgomery form of 1
constexpr uint64_t R1_128_LO = 0xffffffffffffffffull;
constexpr uint64_t R1_128_HI = 0x000000000000001bull;

JX_HD f128 to_mont128(f128 a) { return mont128(a, make128(R2_128_LO, R2_128_HI)); }

JX_HD f128 from_mont128(f128 a) { return mont128(a, make128(1, 0)); }

// Modular reduction of a value < 2^192 (three 64-bit words) to canonical.
// 2^128 == 28*2^64 - 1 (mod p).
JX_HD f128 reduce192(uint64_t w0, uint64_t w1, uint64_t w2) {
  // v = w0 + w1*2^64 + w2*2^128 == w0 + w1*2^64 + w2*(28*2^64 - 1)
  //   = (w0 - w2) + 2^64*(w1 + 28*w2)
  // w2 < 2^64: 28*w2 < 2^69.  Iterate until the top word is zero.
#pragma unroll 1
  for (int it = 0; it < 4 && w2 != 0; it++) {
    uint64_t m_lo = w2 * 28u;
    uint64_t m_hi = umulhi64_28(w2);  // 28*w2 = m_hi*2^64 + m_lo
    uint32_t br = 0;
    uint64_t a0 = subb64(w0, w2, br);  // w0 - w2, borrow into the 2^64 column
    uint32_t c = 0;
    uint64_t a1 = addc64(w1, m_lo, c);
    uint64_t a2 = m_hi + c;
    // subtract borrow from (a1, a2)
    uint32_t br2 = br;
    a1 = subb64(a1, 0, br2);
    a2 = a2 - br2;
    w0 = a0;
    w1 = a1;
    w2 = a2;
  }
  f128 v = make128(w0, w1);
  // v < 2^128 now; at most two subtractions of p
  if (ge_p128(v)) {
    uint32_t br = 0;
    v.lo = subb64(v.lo, P128_LO, br);
    v.hi = subb64(v.hi, P128_HI, br);
  }
  if (ge_p128(v)) {
    uint32_t br = 0;
    v.lo = subb64(v.lo, P128_LO, br);
    v.hi = subb64(v.hi, P128_HI, br);
  }
  return v;
}

// 192-bit lazy accumulator (sums of < 2^129 values; safe for < 2^63 terms)
struct acc192 {
  uint64_t w0, w1, w2;
};
JX_HD void acc_zero(acc192& a) { a.w0 = a.w1 = a.w2 = 0; }
JX_HD void acc_add(acc192& a, uint64_t lo, uint64_t hi, uint32_t top) {
  uint32_t c = 0;
  a.w0 = addc64(a.w0, lo, c);
  a.w1 = addc64(a.w1, hi, c);
  a.w2 += (uint64_t)top + c;
}
// reduce192 for a top word w2 < 2^32 (the output-share truncation: V < 2^(128 + bits)), branch-free:
// one fold of w2 (2^128 == 28*2^64 - 1), one fold of its carry, one conditional subtraction of p.
JX_HD f128 reduce192_small(uint64_t w0, uint64_t w1, uint64_t w2) {
  uint32_t b = 0;
  uint64_t a0 = subb64(w0, w2, b);
  uint32_t c = 0;
  uint64_t a1 = addc64(w1, w2 * 28u, c);  // w1 + 28 w2 (28 w2 < 2^37)
  uint32_t b1 = b;
  a1 = subb64(a1, 0, b1);  // - the borrow of w0 - w2; w1 + 28 w2 - b >= 0, so c - b1 is 0 or 1
  const uint64_t k = (uint64_t)(c - b1);
  uint32_t b2 = 0;
  a0 = subb64(a0, k, b2);  // k * 2^128 == k * (28 * 2^64 - 1); a1 < 2^37 here when k = 1: no carry
  a1 = a1 + 28u * k - b2;
  f128 v = make128(a0, a1);
  uint32_t br = 0;
  const uint64_t lo = subb64(v.lo, P128_LO, br);
  const uint64_t hi = subb64(v.hi, P128_HI, br);
  return ge_p128(v) ? make128(lo, hi) : v;  // v < 2^128 < 2p: one subtraction at most
}
JX_HD void acc_add128(acc192& a, f128 v) { acc_add(a, v.lo, v.hi, 0); }
JX_HD f128 acc_reduce(const acc192& a) { return reduce192(a.w0, a.w1, a.w2); }

// ----------------------------------------------------------------------------
// Wide lazy dot products for the FLP wire sums  sum_k x_k * c_k  (thousands of terms per
// report). Operands are split into five 26-bit limbs; one limb product is < 2^52, so nine
// 64-bit column accumulators absorb every partial product with a single v_mad_u64_u32 and
// no carry handling for up to 4096 / 5 terms per column between normalisations. The sum is
// reduced mod p once, at the end.

struct limbs26 {
  uint32_t l[5];
};
JX_HD limbs26 to_limbs26(f128 a) {
  const uint32_t M = (1u << 26) - 1;
  const uint32_t w0 = lo32(a.lo), w1 = hi32(a.lo), w2 = lo32(a.hi), w3 = hi32(a.hi);
  limbs26 r;
  r.l[0] = w0 & M;
  r.l[1] = (uint32_t)(((((uint64_t)w1) << 32) | w0) >> 26) & M;
  r.l[2] = (uint32_t)(((((uint64_t)w2) << 32) | w1) >> 20) & M;
  r.l[3] = (uint32_t)(((((uint64_t)w3) << 32) | w2) >> 14) & M;
  r.l[4] = w3 >> 8;
  return r;
}

struct wacc26 {
  uint64_t col[9];  // value = sum_s col[s] * 2^(26 s)
};
JX_HD void wacc_zero(wacc26& a) {
#pragma unroll
  for (int s = 0; s < 9; s++) a.col[s] = 0;
}
JX_HD void wacc_mac(wacc26& a, const limbs26& x, const limbs26& c) {
#pragma unroll
  for (int i = 0; i < 5; i++)
#pragma unroll
    for (int j = 0; j < 5; j++) {
      a.col[i + j] += (uint64_t)x.l[i] * c.l[j];
#ifdef __HIP_DEVICE_COMPILE__
      // keeps every product accumulating straight into its column (one v_mad_u64_u32 each);
      // without it the compiler sums a column's products in a side chain and adds that with
      // an extra 64-bit add per column
      asm("" : "+v"(a.col[i + j]));
#endif
    }
}
// carry-propagate so that col[0..7] < 2^26 (keeps headroom for further terms)
JX_HD void wacc_normalize(wacc26& a) {
  const uint64_t M = (1ull << 26) - 1;
#pragma unroll
  for (int s = 0; s < 8; s++) {
    a.col[s + 1] += a.col[s] >> 26;
    a.col[s] &= M;
  }
}
// value mod p (canonical), for values < 2^320
JX_HD f128 wacc_reduce(wacc26 a) {
  wacc_normalize(a);
  // pack the 26-bit limbs (top limb wider) into five 64-bit words
  uint64_t o[5] = {0, 0, 0, 0, 0};
  int oi = 0, nb = 0;
  uint64_t buf_lo = 0, buf_hi = 0;  // 128-bit bit buffer
#pragma unroll
  for (int s = 0; s < 9; s++) {
    const uint64_t v = a.col[s];
    // buf |= v << nb  (nb < 64)
    buf_lo |= v << nb;
    buf_hi |= nb ? (v >> (64 - nb)) : 0;
    nb += 26;
    if (nb >= 64) {
      o[oi++] = buf_lo;
      buf_lo = buf_hi;
      buf_hi = 0;
      nb -= 64;
    }
  }
  // flush: the top limb may hold up to 64 bits beyond position 208
  if (oi < 5) o[oi++] = buf_lo;
  if (oi < 5) o[oi++] = buf_hi;
  // Straight-line fold (value < 2^272, so o4 < 2^16). Mod p, 2^128 = 28 2^64 - 1, 2^192 = 783 2^64 - 28,
  // 2^256 = 21896 2^64 - 783, hence
  //   V = (o0 - S) + 2^64 H,  S = o2 + 28 o3 + 783 o4 (< 2^70),  H = o1 + 28 o2 + 783 o3 + 21896 o4 (< 2^74);
  // T = H 2^64 + o0 - S is >= 0 (H 2^64 >= S whenever S > 0) and < 2^139; folding T's bits >= 2^128 (t2 <
  // 2^11) once more leaves U < 2^128 + 2^80 < 2p, and one conditional subtraction makes it canonical. (The
  // Horner form with reduce192's data-dependent loop cost ~250 VALU; this ~70.)
  typedef unsigned __int128 u128;
  const u128 S = (u128)o[2] + (u128)o[3] * 28u + (u128)o[4] * 783u;
  const u128 H = (u128)o[1] + (u128)o[2] * 28u + (u128)o[3] * 783u + (u128)o[4] * 21896u;
  const u128 Tlo = ((u128)(uint64_t)H << 64) | o[0];  // H 2^64 + o0 = t2 2^128 + Tlo
  uint64_t t2 = (uint64_t)(H >> 64);
  const u128 T = Tlo - S;
  t2 -= (uint64_t)(Tlo < S);
  const u128 add = (u128)(28u * t2) << 64;  // t2 2^128 = 28 t2 2^64 - t2
  u128 U = T + add;
  uint32_t top = U < add;
  const u128 U2 = U - t2;
  top -= (uint32_t)(U < (u128)t2);
  const u128 P = ((u128)P128_HI << 64) | P128_LO;
  const u128 D = U2 - P;
  const u128 R = (top || U2 >= P) ? D : U2;
  return make128((uint64_t)R, (uint64_t)(R >> 64));
}

// ----------------------------------------------------------------------------
// Field64 (Goldilocks) p = 2^64 - 2^32 + 1, canonical representation

constexpr uint64_t P64 = 0xFFFFFFFF00000001ull;

JX_HD uint64_t add64(uint64_t a, uint64_t b) {
  uint64_t s = a + b;
  bool c = s < a;
  // if carry: s + 2^64 - p = s + 2^32 - 1
  if (c) s += 0xFFFFFFFFull;  // cannot overflow again since s < p - 2^32... handled by final check
  if (s >= P64) s -= P64;
  return s;
}
JX_HD uint64_t sub64(uint64_t a, uint64_t b) { return a >= b ? a - b : a + (P64 - b); }
JX_HD uint64_t mul64(uint64_t a, uint64_t b) {
  // 128-bit product
  uint64_t a0 = lo32(a), a1 = hi32(a), b0 = lo32(b), b1 = hi32(b);
  uint64_t p00 = a0 * b0, p01 = a0 * b1, p10 = a1 * b0, p11 = a1 * b1;
  uint64_t mid = (p00 >> 32) + (uint32_t)p01 + (uint32_t)p10;
  uint64_t lo = (uint32_t)p00 | (mid << 32);
  uint64_t hi = p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
  // x = lo + hi*2^64; 2^64 == 2^32 - 1; 2^96 == -1
  uint64_t hh = hi >> 32, hl = hi & 0xFFFFFFFFull;
  uint64_t t = lo - hh;
  if (lo < hh) t += P64;  // borrow: add p (t = lo - hh + p, fits since lo - hh + p < p)
  uint64_t u = hl * 0xFFFFFFFFull;  // < 2^64
  uint64_t r = t + u;
  if (r < t) r += 0xFFFFFFFFull;  // carry: 2^64 == 2^32 - 1
  if (r >= P64) r -= P64;
  return r;
}


// 192-bit value w0 + w1 2^64 + w2 2^128 mod p64 (2^64 == 2^32 - 1, 2^128 == -2^32)
JX_HD uint64_t reduce192_p64(uint64_t w0, uint64_t w1, uint64_t w2) {
  const uint64_t a = w0 >= P64 ? w0 - P64 : w0;
  const uint64_t b = w1 >= P64 ? w1 - P64 : w1;
  const uint64_t d = w2 >= P64 ? w2 - P64 : w2;
  return add64(add64(a, mul64(b, 0xFFFFFFFFull)), mul64(d, P64 - 0x100000000ull));
}

// Field64 wire sums without per-product reduction (the multiproof SumVec FLP): x < 2^64 as two
// 32-bit limbs, the coefficient c < 2^64 as 22/22/20-bit limbs; each of the six limb products
// (< 2^54) goes into its own 64-bit column with one v_mad_u64_u32, exact for up to 1024 products
// per column; column weights 2^0, 2^22, 2^44 (x0) and 2^32, 2^54, 2^76 (x1).
struct c64limbs {
  uint32_t l0, l1, l2;
};
JX_HD c64limbs to_c64limbs(uint64_t c) {
  c64limbs r;
  r.l0 = (uint32_t)c & 0x3FFFFFu;
  r.l1 = (uint32_t)(c >> 22) & 0x3FFFFFu;
  r.l2 = (uint32_t)(c >> 44);
  return r;
}
struct wacc64 {
  uint64_t w[6];
};
constexpr uint32_t WACC64_MAX_TERMS = 1024;
JX_HD void wacc64_zero(wacc64& a) {
#pragma unroll
  for (int i = 0; i < 6; i++) a.w[i] = 0;
}
JX_HD void wacc64_mac(wacc64& a, uint64_t x, const c64limbs& c) {
  const uint32_t x0 = lo32(x), x1 = hi32(x);
  a.w[0] += (uint64_t)x0 * c.l0;
  a.w[1] += (uint64_t)x0 * c.l1;
  a.w[2] += (uint64_t)x0 * c.l2;
  a.w[3] += (uint64_t)x1 * c.l0;
  a.w[4] += (uint64_t)x1 * c.l1;
  a.w[5] += (uint64_t)x1 * c.l2;
}
// the column sum as a canonical Field64 element
JX_HD uint64_t wacc64_reduce(const wacc64& a) {
  uint64_t w0 = 0, w1 = 0, w2 = 0;
  auto add = [&](uint64_t lo, uint64_t hi, uint64_t top) {
    uint32_t c = 0;
    w0 = addc64(w0, lo, c);
    w1 = addc64(w1, hi, c);
    w2 += top + c;
  };
  add(a.w[0], 0, 0);
  add(a.w[1] << 22, a.w[1] >> 42, 0);
  add(a.w[2] << 44, a.w[2] >> 20, 0);
  add(a.w[3] << 32, a.w[3] >> 32, 0);
  add(a.w[4] << 54, a.w[4] >> 10, 0);
  add(0, a.w[5] << 12, a.w[5] >> 52);
  return reduce192_p64(w0, w1, w2);
}
JX_HD uint64_t pow64_h(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mul64(r, a);
    a = mul64(a, a);
    e >>= 1;
  }
  return r;
}

}  // namespace jx
