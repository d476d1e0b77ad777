// Host build of the device arithmetic headers (janus_amd/csrc/jx_*.h), so the exact
// field / Keccak / SHA-256 code the kernels inline is checked against the oracle on
// the CPU (tests/test_device_math_host.py). Test-only; not part of the product.
#include <stdint.h>
#include <string.h>

#include "../../janus_amd/csrc/jx_field.h"
#include "../../janus_amd/csrc/jx_keccak.h"
#include "../../janus_amd/csrc/jx_sha256.h"
#include "../../janus_amd/csrc/jx_hpke.h"
#include "../../janus_amd/csrc/jx_sha_aes.h"

using namespace jx;

static f128 ld(const uint8_t* p) {
  uint64_t lo, hi;
  memcpy(&lo, p, 8);
  memcpy(&hi, p + 8, 8);
  return make128(lo, hi);
}
static void st(uint8_t* p, f128 v) {
  memcpy(p, &v.lo, 8);
  memcpy(p + 8, &v.hi, 8);
}

extern "C" {
// op: 0 add, 1 sub, 2 mont, 3 to_mont, 4 from_mont, 5 neg
void ht_f128(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  f128 x = ld(a), y = b ? ld(b) : make128(0, 0), r;
  switch (op) {
    case 0: r = add128(x, y); break;
    case 1: r = sub128(x, y); break;
    case 2: r = mont128(x, y); break;
    case 3: r = to_mont128(x); break;
    case 4: r = from_mont128(x); break;
    default: r = neg128(x); break;
  }
  st(out, r);
}
void ht_reduce192(const uint64_t w[3], uint8_t* out) { st(out, reduce192(w[0], w[1], w[2])); }
// wacc_reduce of nine raw column sums (each < 2^63, the wire-sum bound)
void ht_wacc_reduce(const uint64_t cols[9], uint8_t* out) {
  wacc26 a;
  for (int s = 0; s < 9; s++) a.col[s] = cols[s];
  st(out, wacc_reduce(a));
}
void ht_reduce192_small(const uint64_t w[3], uint8_t* out) { st(out, reduce192_small(w[0], w[1], w[2])); }
void ht_mont_lazy(const uint8_t* a, const uint8_t* b, uint64_t out[3]) {
  uint64_t lo, hi;
  uint32_t top;
  mont128_lazy(ld(a), ld(b), lo, hi, top);
  out[0] = lo;
  out[1] = hi;
  out[2] = top;
}
// sum_k xs[k] * cs[k] mod p through the 26-bit-limb column accumulator, normalising every
// `norm_every` terms (the FLP kernel normalises every 512 calls)
void ht_wide_dot(const uint8_t* xs, const uint8_t* cs, int n, int norm_every, uint8_t* out) {
  wacc26 a;
  wacc_zero(a);
  for (int k = 0; k < n; k++) {
    wacc_mac(a, to_limbs26(ld(xs + 16 * k)), to_limbs26(ld(cs + 16 * k)));
    if (norm_every > 0 && (k + 1) % norm_every == 0) wacc_normalize(a);
  }
  st(out, wacc_reduce(a));
}
// ---- HPKE primitives (jx_hpke.h)
void ht_x25519(const uint8_t k[32], const uint8_t u[32], uint8_t out[32]) {
  uint8_t kc[32];
  memcpy(kc, k, 32);
  kc[0] &= 248;
  kc[31] &= 127;
  kc[31] |= 64;
  uint32_t kw[8], uw[8], ow[8];
  memcpy(kw, kc, 32);
  memcpy(uw, u, 32);
  x25519_ladder(ow, kw, uw);
  memcpy(out, ow, 32);
}
// op: 0 mul, 1 sq, 2 sub, 3 invert, 4 mul_small(121665); inputs/outputs canonical 32-byte LE
void ht_fe(int op, const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  uint32_t aw[8], bw[8], ow[8];
  memcpy(aw, a, 32);
  memcpy(bw, b, 32);
  fe x, y, r;
  fe_from_bytes(x, aw);
  fe_from_bytes(y, bw);
  switch (op) {
    case 0: fe_mul(r, x, y); break;
    case 1: fe_sq(r, x); break;
    case 2: fe_sub(r, x, y); break;
    case 3: fe_invert(r, x); break;
    default: fe_mul_small(r, x, 121665); break;
  }
  fe_to_bytes(ow, r);
  memcpy(out, ow, 32);
}
// op 0 mul, 1 sq, 4 mul_small(121665) on raw limbs (loosely reduced inputs up to 2^28 - 1, as fe_sub / fe_add
// produce them inside the ladder); the output limbs as the reduction leaves them (bounds checked by the test)
void ht_fe_limbs(int op, const uint32_t a[10], const uint32_t b[10], uint32_t out[10]) {
  fe x, y, r;
  for (int i = 0; i < 10; i++) {
    x.v[i] = a[i];
    y.v[i] = b[i];
  }
  switch (op) {
    case 0: fe_mul(r, x, y); break;
    case 1: fe_sq(r, x); break;
    default: fe_mul_small(r, x, 121665); break;
  }
  for (int i = 0; i < 10; i++) out[i] = r.v[i];
}
static uint8_t HT_SBOX[256];
static void ht_sbox_init() {
  // FIPS 197 S-box generated from GF(2^8) inverses (independent of the kernel's table)
  uint8_t inv[256] = {0};
  for (int x = 1; x < 256; x++)
    for (int y = 1; y < 256; y++) {
      int a = x, b = y, r = 0;
      for (int i = 0; i < 8; i++) {
        if (b & 1) r ^= a;
        int hi = a & 0x80;
        a = (a << 1) & 0xff;
        if (hi) a ^= 0x1b;
        b >>= 1;
      }
      if (r == 1) {
        inv[x] = (uint8_t)y;
        break;
      }
    }
  for (int x = 0; x < 256; x++) {
    int b = inv[x], s = b;
    for (int i = 1; i < 5; i++) s ^= ((b << i) | (b >> (8 - i))) & 0xff;
    HT_SBOX[x] = (uint8_t)(s ^ 0x63);
  }
}
void ht_aes128(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
  ht_sbox_init();
  uint32_t k[4], rk[44], i4[4], o4[4];
  memcpy(k, key, 16);
  memcpy(i4, in, 16);
  aes128_expand_key(HT_SBOX, k, rk);
  aes128_encrypt(HT_SBOX, rk, i4, o4);
  memcpy(out, o4, 16);
}
// x, h: 16-byte blocks; out = x * h in GF(2^128) (GCM bit order)
void ht_ghash_mul(const uint8_t x[16], const uint8_t h[16], uint8_t out[16]) {
  uint32_t xw[4], hw[4];
  for (int i = 0; i < 4; i++) {
    xw[i] = (uint32_t)x[4 * i] << 24 | (uint32_t)x[4 * i + 1] << 16 | (uint32_t)x[4 * i + 2] << 8 | x[4 * i + 3];
    hw[i] = (uint32_t)h[4 * i] << 24 | (uint32_t)h[4 * i + 1] << 16 | (uint32_t)h[4 * i + 2] << 8 | h[4 * i + 3];
  }
  ghash_mul(xw, hw);
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(xw[i] >> (24 - 8 * k));
}
// HMAC-SHA256 with a 32-byte key over msg (len <= 119) through hmac_pads/sha256_finish64/hmac_outer
void ht_hmac32(const uint8_t key[32], const uint8_t* msg, int len, uint8_t out[32]) {
  uint32_t kb[8], ist[8], ost[8], inner[8], o[8];
  for (int i = 0; i < 8; i++)
    kb[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 | (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
  hmac_pads(kb, ist, ost);
  Msg128 m;
  m_zero(m);
  for (int i = 0; i < len; i++) m_byte(m, i, msg[i]);
  sha256_finish64(inner, ist, m, len);
  hmac_outer(o, ost, inner);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(o[i] >> (24 - 8 * k));
}
// op: 0 add, 1 sub, 2 mul
uint64_t ht_f64(int op, uint64_t a, uint64_t b) {
  switch (op) {
    case 0: return add64(a, b);
    case 1: return sub64(a, b);
    default: return mul64(a, b);
  }
}
void ht_keccak_p12(uint64_t st64[25]) {
  uint32_t s[50];
  for (int i = 0; i < 25; i++) {
    s[2 * i] = (uint32_t)st64[i];
    s[2 * i + 1] = (uint32_t)(st64[i] >> 32);
  }
  keccak_p12(s);
  for (int i = 0; i < 25; i++) st64[i] = (uint64_t)s[2 * i] | ((uint64_t)s[2 * i + 1] << 32);
}
void ht_sha256_16(const uint8_t id[16], uint8_t out[32]) {
  uint32_t w[4], d[8];
  memcpy(w, id, 16);
  sha256_16(w, d);
  memcpy(out, d, 32);
}
// XOF prefix block builder: returns the 42 words of a one-block message
// prefix(algo, usage, seed) || binder (<= 142 bytes), padded.
void ht_xof_block(uint32_t algo, uint32_t usage, const uint8_t seed[16], const uint8_t* binder, int blen,
                  uint32_t out[42]) {
  Block b;
  blk_zero(b);
  uint32_t sw[4];
  memcpy(sw, seed, 16);
  int pos = blk_xof_prefix(b, algo, usage, sw);
  for (int i = 0; i < blen; i++) blk_put_byte(b, pos + i, binder[i]);
  blk_pad(b, pos + blen);
  memcpy(out, b.w, sizeof b.w);
}
// T-table AES of the XofHmacSha256Aes128 kernels (jx_sha_aes.h): otf = 0 expands the 44-word
// schedule first, otf = 1 computes it on the fly
void ht_aes128_t(int otf, const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
  ht_sbox_init();
  static uint32_t t0[256];
  for (int x = 0; x < 256; x++) t0[x] = aes_t0_entry(HT_SBOX[x]);
  auto T = [&](uint32_t x) { return t0[x]; };
  uint32_t k[4], rk[44], i4[4], o4[4];
  memcpy(k, key, 16);
  memcpy(i4, in, 16);
  if (otf) {
    aes128_encrypt_t_otf(T, k, i4, o4);
  } else {
    aes128_expand_key_t(T, k, rk);
    aes128_encrypt_t(T, rk, i4, o4);
  }
  memcpy(out, o4, 16);
}
uint32_t ht_be_word_shift16(uint32_t lo, uint32_t hi) { return be_word_shift16(lo, hi); }
// sum_k xs[k] * cs[k] mod p64 through the Field64 limb column accumulator (folding every 1024 terms)
uint64_t ht_wacc64_dot(const uint64_t* xs, const uint64_t* cs, int n) {
  wacc64 a;
  wacc64_zero(a);
  uint64_t acc = 0;
  for (int k = 0; k < n; k++) {
    wacc64_mac(a, xs[k], to_c64limbs(cs[k]));
    if ((k + 1) % (int)WACC64_MAX_TERMS == 0) {
      acc = add64(acc, wacc64_reduce(a));
      wacc64_zero(a);
    }
  }
  return add64(acc, wacc64_reduce(a));
}
uint64_t ht_reduce192_p64(const uint64_t w[3]) { return reduce192_p64(w[0], w[1], w[2]); }
}
