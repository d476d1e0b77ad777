// Host build of the device arithmetic headers (janus_amd/csrc/jx_*.h), so the exact
// field / Keccak / SHA-256 code the kernels inline is checked against the oracle on
// the CPU (tests/test_device_math_host.py). Test-only; not part of the product.
#include <stdint.h>
#include <string.h>

#include "../../janus_amd/csrc/jx_field.h"
#include "../../janus_amd/csrc/jx_keccak.h"
#include "../../janus_amd/csrc/jx_sha256.h"

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
}
