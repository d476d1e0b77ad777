// jx_kernels.hip — gfx950 kernels for batched Prio3 helper preparation + aggregation.
//
// The per-report work Janus does at aggregator/src/aggregator.rs:1945-1967
// (prio 0.16.1 ping-pong helper_initialized + evaluate) is split into three
// launches over a batch of reports:
//
//   K1 xof_kernel      one report per lane. TurboSHAKE128 expansion of the helper
//                      measurement share (fused with the joint_rand_part absorb of the
//                      same bytes) and proof share; joint_rand_seed, joint_rands,
//                      query_rands, the prepare-message seed; per-report FLP
//                      coefficients (barycentric weights, batch-inverted).
//   K3 flp_*_kernel    FLP query on the helper share + add the leader's verifier
//                      share + decide + prepare_next check -> verdict byte.
//   K4 accumulate      masked/segmented field sum of output shares (+count, +checksum),
//                      i.e. BatchAggregation::merged_with (models.rs:1275-1330).
//
// Prio3Count (Field64, 3 permutations) runs as one lane-per-report kernel.
// Algorithm: draft-irtf-cfrg-vdaf-08 as implemented by prio 0.16.1; see DESIGN.md.
#include <cstdlib>
#include <stdlib.h>

#include <type_traits>

#include "jx_field.h"
#include "jx_kernels.h"
#include "jx_keccak.h"
#include "jx_sha256.h"

namespace jx {

// ---------------------------------------------------------------------------- helpers

__device__ __forceinline__ f128 u4_to_f(uint4 v) {
  return make128((uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z | ((uint64_t)v.w << 32));
}
__device__ __forceinline__ uint4 f_to_u4(f128 a) { return make_uint4(lo32(a.lo), hi32(a.lo), lo32(a.hi), hi32(a.hi)); }
__device__ __forceinline__ f128 w4_to_f(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return make128((uint64_t)a | ((uint64_t)b << 32), (uint64_t)c | ((uint64_t)d << 32));
}
// interleaved staging address
__device__ __forceinline__ uint64_t il_idx(uint64_t blk, uint32_t len, uint32_t e, uint32_t lane) {
  return (blk * len + e) * IL + lane;
}
// (the staging is global memory: the address-space casts keep these global_load/store even inside the
// non-inlined XOF tail, where a generic pointer would make them flat accesses that wait with vmcnt(0) and
// lgkmcnt(0) each)
// global (not flat) pointers for the staging in the non-inlined XOF tail: flat accesses count in both
// vmcnt and lgkmcnt and force full waits; the host pass of hipcc keeps plain pointers
#ifdef __HIP_DEVICE_COMPILE__
typedef __attribute__((address_space(1))) uint4 g_uint4;
#else
typedef uint4 g_uint4;
#endif
__device__ __forceinline__ f128 ld_il(const uint4* base, uint64_t blk, uint32_t len, uint32_t e, uint32_t lane) {
  return u4_to_f(((const g_uint4*)base)[il_idx(blk, len, e, lane)]);
}
__device__ __forceinline__ void st_il(uint4* base, uint64_t blk, uint32_t len, uint32_t e, uint32_t lane, f128 v) {
  ((g_uint4*)base)[il_idx(blk, len, e, lane)] = f_to_u4(v);
}
// The measurement share as the FLP kernels read it: the interleaved staging (element e of the lane's
// report at p[e * IL]) or, for the leader, its explicit input share in place (p[e], report-major).
struct MeasView {
  const uint4* p;
  uint32_t es;  // element stride in uint4
  __device__ __forceinline__ const uint4& operator[](uint64_t e) const { return p[e * es]; }
};
__device__ __forceinline__ MeasView meas_view(const Cfg& c, const Bufs& b, uint64_t blk, uint32_t lane) {
  if (b.meas_rs) {
    const uint64_t r0 = blk * 64 + lane, r = r0 < b.n ? r0 : b.n - 1;
    return MeasView{reinterpret_cast<const uint4*>(b.meas_src + r * b.meas_rs), 1u};
  }
  return MeasView{b.meas + il_idx(blk, c.meas_len, 0, lane), (uint32_t)IL};
}
__device__ __forceinline__ void load16(const uint8_t* p, uint32_t w[4]) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
}

// the verify key of report r: its row of the per-report keys of a coalesced launch, or the engine's
__device__ __forceinline__ void load_vk(const Cfg& c, const Bufs& b, uint64_t r, uint32_t vk[4]) {
  if (b.vkeys) {
    load16(b.vkeys + 16 * r, vk);
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++) vk[i] = c.vk[i];
  }
}

// Montgomery exponentiation, uniform exponent
__device__ f128 mpow(f128 aR, uint32_t e) {
  f128 r = make128(R1_128_LO, R1_128_HI);
  while (e) {
    if (e & 1) r = mont128(r, aR);
    aR = mont128(aR, aR);
    e >>= 1;
  }
  return r;
}
__device__ __forceinline__ f128 msqr_n(f128 a, int n) {
  for (int i = 0; i < n; i++) a = mont128(a, a);
  return a;
}
// Montgomery inverse: (aR)^(p-2) via an addition chain for p-2 = (2^64-29)*2^64 + (2^64-1)
__device__ f128 minv(f128 a) {
  f128 x2 = mont128(mont128(a, a), a);    // 2^2-1
  f128 x4 = mont128(msqr_n(x2, 2), x2);   // 2^4-1
  f128 x8 = mont128(msqr_n(x4, 4), x4);   // 2^8-1
  f128 x16 = mont128(msqr_n(x8, 8), x8);  // 2^16-1
  f128 x32 = mont128(msqr_n(x16, 16), x16);
  f128 x64 = mont128(msqr_n(x32, 32), x32);
  f128 x48 = mont128(msqr_n(x32, 16), x16);
  f128 y = mont128(msqr_n(x48, 8), x8);  // 2^56-1
  // append the 8 low bits of 0xE3 = 1110 0011
  const uint32_t tail = 0xE3u;
  for (int i = 7; i >= 0; i--) {
    y = mont128(y, y);
    if ((tail >> i) & 1) y = mont128(y, a);
  }
  // y = a^(2^64 - 29); result = y^(2^64) * a^(2^64-1)
  y = msqr_n(y, 64);
  return mont128(y, x64);
}

// ---------------------------------------------------------------------------- Field64 helpers (Count)

__device__ uint64_t pow64(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mul64(r, a);
    a = mul64(a, a);
    e >>= 1;
  }
  return r;
}

// first N accepted Field64 samples from a stream whose first block is in S
template <int N>
__device__ void sample64(uint32_t* S, uint64_t out[N]) {
  int cnt = 0;
#pragma unroll 1
  for (int guard = 0; guard < 64; guard++) {
#pragma unroll
    for (int ci = 0; ci < 21; ci++) {
      uint64_t x = (uint64_t)S[2 * ci] | ((uint64_t)S[2 * ci + 1] << 32);
      bool acc = x < P64;
#pragma unroll
      for (int i = 0; i < N; i++)
        if (acc && cnt == i) out[i] = x;
      cnt += acc ? 1 : 0;
    }
    if (cnt >= N) break;
    keccak_p12(S);
  }
}

// ---------------------------------------------------------------------------- K0: Prio3Count

// LEADER: prepare_init with agg_id 0 on the explicit leader input share (meas || proofs, Field64);
// writes the leader's verifier share [v, W0, W1, G] as its prep share.
template <bool LEADER>
__global__ __launch_bounds__(256) void count_kernel(Cfg c, Bufs b) {
  const uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nblk = (b.n + 63) / 64;
  if (r0 >= nblk * 64) return;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint64_t blk = r0 / 64;
  const uint32_t lane = r0 % 64;
  uint32_t nonce[4], kmeas[4], kproof[4], S[50];
  load16(b.nonces + 16 * r, nonce);
  uint64_t x[1], proof[5], t[1];
  bool bad = false;
  if (LEADER) {
    const uint2* ls = reinterpret_cast<const uint2*>(b.lis + b.lis_rs * r);
    uint2 q = ls[0];
    x[0] = (uint64_t)q.x | ((uint64_t)q.y << 32);
    bad |= x[0] >= P64;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      q = ls[1 + i];
      proof[i] = (uint64_t)q.x | ((uint64_t)q.y << 32);
      bad |= proof[i] >= P64;
    }
  } else {
  load16(b.his + (uint64_t)c.his_bytes * r, kmeas);
  load16(b.his + (uint64_t)c.his_bytes * r + 16, kproof);
  {  // helper_meas_share: XOF(k_meas, DST(usage 1), [agg_id=1])
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, ALGO_COUNT, 1, kmeas);
    blk_put_byte(m, pos, 1);
    blk_pad(m, pos + 1);
    sponge_oneblock(S, m);
    sample64<1>(S, x);
  }
  {  // helper_proofs_share: XOF(k_proofs, DST(usage 2), [PROOFS=1, agg_id=1])
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, ALGO_COUNT, 2, kproof);
    blk_put_byte(m, pos, 1);
    blk_put_byte(m, pos + 1, 1);
    blk_pad(m, pos + 2);
    sponge_oneblock(S, m);
    sample64<5>(S, proof);
  }
  }
  {  // query_rands: XOF(verify_key, DST(usage 5), [PROOFS=1] || nonce)
    Block m;
    blk_zero(m);
    uint32_t vk[4];
    load_vk(c, b, r, vk);
    int pos = blk_xof_prefix(m, ALGO_COUNT, 5, vk);
    blk_put_byte(m, pos, 1);
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(m, pos + 1 + 4 * i, nonce[i]);
    blk_pad(m, pos + 17);
    sponge_oneblock(S, m);
    sample64<1>(S, t);
  }
  // FLP query, gadget Mul (arity 2), 1 call, P = 2, alpha = -1
  const uint64_t one = 1, minus1 = P64 - 1;
  uint64_t tt = t[0];
  uint64_t t2 = mul64(tt, tt);
  uint32_t verdict = 0;
  if (t2 == one) verdict = 1;  // prepare_init_failure
  uint64_t dm = sub64(tt, one), dp = add64(tt, one);
  uint64_t inv = pow64(mul64(dm, dp), P64 - 2);
  uint64_t c0 = mul64(inv, dp);                  // 1/(t-1)
  uint64_t c1 = mul64(minus1, mul64(inv, dm));   // -1/(t+1) = alpha^1/(t - alpha^1)
  uint64_t inv2 = (P64 + 1) / 2;
  uint64_t L = mul64(sub64(t2, one), inv2);
  uint64_t xm = x[0];
  uint64_t W0 = mul64(L, add64(mul64(c0, proof[0]), mul64(c1, xm)));
  uint64_t W1 = mul64(L, add64(mul64(c0, proof[1]), mul64(c1, xm)));
  // circuit: Mul(x,x) - x with the gadget replaced by gadget_poly(alpha^1) = g0 - g1 + g2
  uint64_t v = sub64(add64(sub64(proof[2], proof[3]), proof[4]), xm);
  uint64_t G = add64(proof[2], mul64(tt, add64(proof[3], mul64(tt, proof[4]))));
  if (LEADER) {
    if (r0 < b.n) {
      uint2* o = reinterpret_cast<uint2*>(b.lps_out + (uint64_t)c.lps_bytes * r);
      o[0] = make_uint2(lo32(v), hi32(v));
      o[1] = make_uint2(lo32(W0), hi32(W0));
      o[2] = make_uint2(lo32(W1), hi32(W1));
      o[3] = make_uint2(lo32(G), hi32(G));
      b.verdicts[r0] = (uint8_t)((verdict || bad) ? 1 : 0);
    }
    b.outs[il_idx(blk, 1, 0, lane)] = make_uint4(lo32(xm), hi32(xm), 0, 0);
    return;
  }
  // leader verifier share: [v, W0, W1, G] as 4 x 8-byte LE
  const uint8_t* lp = b.lps + (uint64_t)c.lps_bytes * r;
  uint64_t lv[4];
  bool dfail = false;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint2 q = *reinterpret_cast<const uint2*>(lp + 8 * i);
    lv[i] = (uint64_t)q.x | ((uint64_t)q.y << 32);
    dfail |= lv[i] >= P64;
  }
  if (verdict == 0 && dfail) verdict = 2;
  if (verdict == 0) {
    uint64_t V0 = add64(v, lv[0]), V1 = add64(W0, lv[1]), V2 = add64(W1, lv[2]), VG = add64(G, lv[3]);
    if (V0 != 0 || mul64(V1, V2) != VG) verdict = 3;
  }
  if (r0 < b.n) b.verdicts[r0] = (uint8_t)verdict;
  b.outs[il_idx(blk, 1, 0, lane)] = make_uint4(lo32(xm), hi32(xm), 0, 0);
}

// ---------------------------------------------------------------------------- K1: XOF stage (Field128)

struct Trunc {
  acc192 a;
  uint32_t j, i;
};

// 192-bit add of x << sh (sh < 64) into the accumulator
__device__ __forceinline__ void trunc_add(acc192& a, f128 x, uint32_t sh) {
  uint64_t w0 = x.lo << sh;
  uint64_t w1 = sh ? ((x.hi << sh) | (x.lo >> (64 - sh))) : x.hi;
  uint64_t w2 = sh ? (x.hi >> (64 - sh)) : 0;
  uint32_t cc = 0;
  a.w0 = addc64(a.w0, w0, cc);
  a.w1 = addc64(a.w1, w1, cc);
  a.w2 = a.w2 + w2 + cc;
}

// A value the optimizer cannot see through (no instruction is emitted): keeps x * 2^j a single
// v_mad_u64_u32 (x * 2^j + T) instead of the zero-extend + 64-bit shift + 64-bit add it would
// strength-reduce the multiply to.
__device__ __forceinline__ uint32_t opaque_u32(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Output-share truncation in the fast XOF kernel (SumVec / Sum):
//   out_i = sum_{j<bits} 2^j x_{bits*i+j} mod p.
// Word columns T_w = sum_j x_{j,w} 2^j (< 2^(32+bits) <= 2^64) cost one v_mad_u64_u32 per 32-bit
// word of each element; the <= 160-bit total is reduced once per output element.
struct TruncW {
  uint64_t T[4];
  uint32_t j, i;
};
__device__ __forceinline__ void truncw_zero(TruncW& t) {
#pragma unroll
  for (int w = 0; w < 4; w++) t.T[w] = 0;
}
__device__ __forceinline__ f128 truncw_value(const TruncW& t) {
  // V = T0 + T1 2^32 + T2 2^64 + T3 2^96
  uint32_t c = 0;
  const uint64_t w0 = addc64(t.T[0], t.T[1] << 32, c);
  const uint64_t w1 = addc64(t.T[2], (t.T[1] >> 32) | (t.T[3] << 32), c);
  const uint64_t w2 = (t.T[3] >> 32) + c;
  return reduce192_small(w0, w1, w2);  // V < 2^(128 + bits), bits <= 32
}
// Conservative ">= p" screen for a sampled Field128 element: true for every x >= p (and for
// the 2^-59-probable x in [2^128 - 2^69, p), which the slow kernel then redoes exactly).
// Tracked as a running max so that one compare per block decides.
__device__ __forceinline__ uint32_t ge_screen(uint4 v) { return v.w & (v.z | 0x1Fu); }

// h * 2^32 mod p (the high half of a > 32-bit truncation)
__device__ __forceinline__ f128 shl32_mod(f128 h) {
  return reduce192(h.lo << 32, (h.hi << 32) | (h.lo >> 32), h.hi >> 32);
}

// one measurement element at static stream position e (fast path: no rejections)
// WIDE (bits in (32, 64], Sum / SumVec): the word columns of bits 0..31 are folded into `lo` at
// bit 32 and restart for the bits 32.. (weights 2^(j-32) < 2^32); out = lo + 2^32 * high.
template <bool WIDE, bool STORE = true>
__device__ __forceinline__ void emit_meas(const Cfg& c, uint4* mp, uint4* op, uint32_t e, uint4 v, uint32_t& gmax,
                                          TruncW& tr, f128& lo) {
  // e is uniform. Straight-line except for the store guard and the once-per-output-element finish:
  // elements past the share (last block) or not truncated (Histogram; FixedPoint's trailing norm
  // bits) add with weight 0 instead of branching around the column sums.
  const bool in = e < c.meas_len;
  if (STORE && in) mp[(uint64_t)e * IL] = v;
  gmax = max(gmax, in ? ge_screen(v) : 0u);
  const bool tin = !c.out_is_meas && e < c.trunc_len;
  const uint32_t sh = opaque_u32(tin ? 1u << (WIDE ? (tr.j & 31u) : tr.j) : 0u);
  tr.T[0] += (uint64_t)v.x * sh;
  tr.T[1] += (uint64_t)v.y * sh;
  tr.T[2] += (uint64_t)v.z * sh;
  tr.T[3] += (uint64_t)v.w * sh;
  tr.j += tin ? 1u : 0u;
  if (WIDE && tin && tr.j == 32 && c.bits > 32) {
    lo = truncw_value(tr);
    truncw_zero(tr);
  }
  if (tin && tr.j == c.bits) {
    f128 val = truncw_value(tr);
    if (WIDE && c.bits > 32) val = add128(lo, shl32_mod(val));
    op[(uint64_t)tr.i * IL] = f_to_u4(val);
    truncw_zero(tr);
    tr.j = 0;
    tr.i++;
  }
}
__device__ __forceinline__ void emit_proof(const Cfg& c, uint4* pp, uint32_t e, uint4 v, uint32_t& gmax) {
  if (e >= c.proof_len) return;
  gmax = max(gmax, ge_screen(v));
  pp[(uint64_t)e * IL] = v;
}

// Barycentric weights of one gadget on the P-th roots of unity w^k (Montgomery form):
//   c_k = w^k / (t - w^k) for k = 1..C at slot sk + stride*(k-1), c_0 = 1/(t - 1) at slot s0,
// by one batch inversion (prefix products parked in the c_k slots, then one inversion chain).
// With with_d (ParallelSum gadget 0, stride 2; rcR = r^chunk R): also d_k = c_k rc^(k-1) at slot sk + 2(k-1) + 1, rc = r^chunk,
// in the same backward pass: rc joins the inverted product, so 1/rc costs two products, and the powers
// descend from rc^(C-1). The backward pass keeps four prefix-product loads in flight (a prefix in slot k-1
// is overwritten only at step k-1, after its read). Returns sum_{k>=1} c_k.
__device__ f128 bary_coeffs(uint4* coef, uint64_t blk, uint32_t NC, uint32_t lane, f128 tR, const uint4* omega,
                            uint32_t C, uint32_t s0, uint32_t sk, uint32_t stride, bool with_d = false,
                            f128 rcR = f128{0, 0}) {
  auto slot = [&](uint32_t k) { return k == 0 ? s0 : sk + stride * (k - 1); };
  const g_uint4* gom = (const g_uint4*)omega;
  f128 acc = sub128(tR, u4_to_f(gom[0]));
  st_il(coef, blk, NC, slot(0), lane, acc);
  for (uint32_t k = 1; k <= C; k++) {
    acc = mont128(acc, sub128(tR, u4_to_f(gom[k])));
    st_il(coef, blk, NC, slot(k), lane, acc);
  }
  f128 inv, rp = make128(R1_128_LO, R1_128_HI), rinv = rp;
  if (with_d) {
    const f128 ie = minv(mont128(acc, rcR));  // 1 / (prefix * rc)
    inv = mont128(ie, rcR);                     // 1 / prefix
    rinv = mont128(ie, acc);                    // 1 / rc
    rp = mpow(rcR, C - 1);                      // rc^(C-1)
  } else {
    inv = minv(acc);
  }
  f128 sumc = make128(0, 0);
  // step k needs the prefix of slot k-1 and w^k: both loaded four steps ahead (vmcnt counts in order, so a
  // load issued just before its use would also wait for every prefetch)
  auto pref = [&](int k) { return k >= 1 ? ld_il(coef, blk, NC, slot((uint32_t)k - 1), lane) : make128(0, 0); };
  auto wk = [&](int k) { return k >= 1 ? u4_to_f(gom[k]) : make128(0, 0); };
  const int Ci = (int)C;
  f128 q0 = pref(Ci), q1 = pref(Ci - 1), q2 = pref(Ci - 2), q3 = pref(Ci - 3);
  f128 o0 = wk(Ci), o1 = wk(Ci - 1), o2 = wk(Ci - 2), o3 = wk(Ci - 3);
  for (uint32_t k = C; k >= 1; k--) {
    const f128 pre = q0, w = o0;
    q0 = q1;
    q1 = q2;
    q2 = q3;
    o0 = o1;
    o1 = o2;
    o2 = o3;
    // unconditional loads (a clamped index past the end: the value is never used) keep the loop
    // branch-free, so the wait before the first use counts only the older loads
    const uint32_t kn = k > 4 ? k - 4 : 1;
    q3 = ld_il(coef, blk, NC, slot(kn - 1), lane);
    o3 = u4_to_f(gom[kn]);
    f128 invden = mont128(inv, pre);
    inv = mont128(inv, sub128(tR, w));
    f128 ck = mont128(w, invden);
    st_il(coef, blk, NC, slot(k), lane, ck);
    if (with_d) {
      st_il(coef, blk, NC, slot(k) + 1, lane, mont128(ck, rp));
      rp = mont128(rp, rinv);
    }
    sumc = add128(sumc, ck);
  }
  st_il(coef, blk, NC, s0, lane, inv);  // c_0 = 1/(t - 1)
  return sumc;
}

// `cnt` (<= 2) Field128 samples from an XOF stream whose first block is in S. Fast path: the first
// two 16-byte chunks, FLAG_SLOW if one is >= p; slow path: rejection sampling (a rejection stays in
// the first block except with probability ~2^-600, beyond which chunks straddling blocks are skipped).
// Every index is static (the chunks are unrolled and a sample lands in out[0] / out[1] by select), so
// the state and the samples stay in registers: a data-dependent index would put both in scratch.
__device__ __forceinline__ void sample2_f128(uint32_t* S, f128 out[2], uint32_t cnt, bool slow, uint32_t& flags) {
  if (!slow) {
    out[0] = w4_to_f(S[0], S[1], S[2], S[3]);
    out[1] = w4_to_f(S[4], S[5], S[6], S[7]);
    if (ge_p128(out[0]) || (cnt > 1 && ge_p128(out[1]))) flags |= FLAG_SLOW;
    return;
  }
  f128 o0 = make128(0, 0), o1 = make128(0, 0);
  uint32_t k = 0;
  for (int guard = 0; guard < 64 && k < cnt; guard++) {
#pragma unroll
    for (int ci = 0; ci < 10; ci++) {
      const f128 v = w4_to_f(S[4 * ci], S[4 * ci + 1], S[4 * ci + 2], S[4 * ci + 3]);
      const bool take = k < cnt && !ge_p128(v);
      if (take && k == 0) o0 = v;
      if (take && k == 1) o1 = v;
      k += take ? 1u : 0u;
    }
    if (k < cnt) keccak_p12(S);
  }
  out[0] = o0;
  out[1] = o1;
}

// Tail of the XOF stage shared by the fast and slow kernels: joint randomness,
// prepare-message seed, query randomness, FLP coefficients.
// part_h: the helper's joint_rand_part. Writes msgs / flags / coef.
// Returns flags (with FLAG_SLOW set if a rejected sample was hit and slow == false).
// INL: the barycentric coefficient chains are inlined instead of called (the lane-split kernel, whose
// registers have room for them: a call's frame and the registers saved around it cost it 80 B of scratch)
template <bool INL = false>
__device__ uint32_t xof_tail(const Cfg& c, const Bufs& b, uint64_t blk, uint32_t lane, uint64_t r, bool write_msg,
                             const uint32_t nonce[4], const uint32_t part_l[4], const uint32_t lead_part[4],
                             const uint32_t part_h[4], uint32_t flags, bool slow) {
  uint32_t S[50];
  const uint32_t zero[4] = {0, 0, 0, 0};
  // corrected joint-rand seed = XOF(0^16, DST(6), part_L || part_H)[0:16]
  uint32_t corr[4];
  {
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 6, zero);
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(m, pos + 4 * i, part_l[i]);
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(m, pos + 16 + 4 * i, part_h[i]);
    blk_pad(m, pos + 32);
    sponge_oneblock(S, m);
#pragma unroll
    for (int i = 0; i < 4; i++) corr[i] = S[i];
  }
  // joint_rands = expand(corrected, DST(3), [PROOFS=1], JR_LEN)
  f128 jr[2];
  {
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 3, corr);
    blk_put_byte(m, pos, 1);
    blk_pad(m, pos + 1);
    sponge_oneblock(S, m);
    sample2_f128(S, jr, c.jr_len, slow, flags);
  }
  // prepare message = XOF(0^16, DST(6), leader's part || part_H); equals corr when the
  // leader's part matches the public share.
  bool same = part_l[0] == lead_part[0] && part_l[1] == lead_part[1] && part_l[2] == lead_part[2] &&
              part_l[3] == lead_part[3];
  uint32_t msg[4] = {corr[0], corr[1], corr[2], corr[3]};
  if (!same) {
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 6, zero);
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(m, pos + 4 * i, lead_part[i]);
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(m, pos + 16 + 4 * i, part_h[i]);
    blk_pad(m, pos + 32);
    sponge_oneblock(S, m);
#pragma unroll
    for (int i = 0; i < 4; i++) msg[i] = S[i];
    if (msg[0] != corr[0] || msg[1] != corr[1] || msg[2] != corr[2] || msg[3] != corr[3]) flags |= FLAG_NEXT_FAIL;
  }
  if (write_msg) *reinterpret_cast<uint4*>(b.msgs + 16 * r) = make_uint4(msg[0], msg[1], msg[2], msg[3]);
  // query_rands = expand(verify_key, DST(5), [PROOFS=1] || nonce, QR_LEN): one t per gadget
  f128 tq[2];
  {
    Block m;
    blk_zero(m);
    uint32_t vk[4];
    load_vk(c, b, r, vk);
    int pos = blk_xof_prefix(m, c.dst_id, 5, vk);
    blk_put_byte(m, pos, 1);
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(m, pos + 1 + 4 * i, nonce[i]);
    blk_pad(m, pos + 17);
    sponge_oneblock(S, m);
    sample2_f128(S, tq, c.qr_len, slow, flags);
  }
  const f128 t = tq[0];
  // ---- FLP coefficients (Montgomery form). Barycentric weights on the P-th roots:
  //   wire_j(t) = L * sum_k c_k * wire_j[k],  c_k = w^k / (t - w^k),  L = (t^P - 1)/P
  const uint4* omega = b.consts + c.c_omega;
  const uint4* misc = b.consts + c.c_misc;
  const f128 R1 = make128(R1_128_LO, R1_128_HI);
  f128 tR = to_mont128(t);
  f128 tp = tR;
  for (uint32_t i = 0; i < c.logP; i++) tp = mont128(tp, tp);
  if (eq128(tp, R1)) flags |= FLAG_INIT_FAIL;
  f128 LR = mont128(sub128(tp, R1), u4_to_f(misc[0]));
  uint4* coef = b.coef;
  const uint32_t NC = c.ncoef;
  st_il(coef, blk, NC, COEF_L, lane, LR);
  st_il(coef, blk, NC, COEF_T, lane, tR);
  f128 rR = to_mont128(jr[0]);
  st_il(coef, blk, NC, COEF_R, lane, rR);
  st_il(coef, blk, NC, COEF_R2, lane, to_mont128(jr[1]));
  // batch inversion of den_k = t - w^k, k = 0..calls
  const uint32_t C = c.calls;
  const uint32_t stride = c.algo == ALGO_SUM ? 1u : 2u;
  const f128 rcR = mpow(rR, c.chunk);  // r^chunk (ParallelSum's d_k = c_k r^((k-1) chunk))
  f128 sumc;
  if constexpr (INL) {
    [[clang::always_inline]] sumc =
        bary_coeffs(coef, blk, NC, lane, tR, omega, C, COEF_C0, COEF_K, stride, c.algo != ALGO_SUM, rcR);
  } else {
    sumc = bary_coeffs(coef, blk, NC, lane, tR, omega, C, COEF_C0, COEF_K, stride, c.algo != ALGO_SUM, rcR);
  }
  if (c.algo == ALGO_SUM) {
    // (1/2) * sum c_k, canonical: mont(sumc*R, 1/2) = sumc/2
    st_il(coef, blk, NC, COEF_HALFSUM, lane, mont128(sumc, u4_to_f(misc[1])));
  } else {
    // the ParallelSum group finish (psum_group_finish) takes its constants scaled by L, so a wire at t costs
    // two products instead of three: COEF_C0 <- c_0 L R, COEF_L <- L canonical, COEF_HALFSUM <- L (sum c_k)/2
    // canonical; below, its power table holds L r^(j+1) (the chain starts from L r: mont(L R, r) = L r)
    const f128 c0R = ld_il(coef, blk, NC, COEF_C0, lane);
    st_il(coef, blk, NC, COEF_C0, lane, mont128(c0R, LR));
    st_il(coef, blk, NC, COEF_L, lane, mont128(LR, make128(1, 0)));
    st_il(coef, blk, NC, COEF_HALFSUM, lane, mont128(mont128(sumc, LR), u4_to_f(misc[1])));
  }
  if (c.algo != ALGO_SUM) {
    // power tables of the ParallelSum group finish: L r^(j+1) canonical for the even wires of slot j (a chain
    // of mont products from L r), and t^(g * per) R for group g's share of G(t)
    f128 rj = mont128(LR, jr[0]);
    for (uint32_t j = 0; j < c.chunk; j++) {
      st_il(coef, blk, NC, c.c_rpow + j, lane, rj);
      rj = mont128(rj, rR);
    }
    const uint32_t per = (c.gpoly_len + c.ngroups - 1) / c.ngroups;
    const f128 tstep = mpow(tR, per);
    f128 tg = R1;
    for (uint32_t g = 0; g < c.ngroups; g++) {
      st_il(coef, blk, NC, c.c_tpow + g, lane, tg);
      tg = mont128(tg, tstep);
    }
  }
  if (c.algo == ALGO_FIXEDPOINT_L2) {
    // gadget 1 (the norm's ParallelSum(PolyEval)): its own query randomness t1 and P1-th roots
    const f128 t1R = to_mont128(tq[1]);
    f128 tp1 = t1R;
    for (uint32_t i = 0; i < c.logP1; i++) tp1 = mont128(tp1, tp1);
    if (eq128(tp1, R1)) flags |= FLAG_INIT_FAIL;
    const uint32_t B = c.coef1;
    st_il(coef, blk, NC, B + G1_L, lane, mont128(sub128(tp1, R1), u4_to_f(misc[7])));
    st_il(coef, blk, NC, B + G1_T, lane, t1R);
    if constexpr (INL) {
      [[clang::always_inline]] (void)bary_coeffs(coef, blk, NC, lane, t1R, b.consts + c.c_omega1, c.calls1, B + G1_C0,
                                                  B + G1_K, 1);
    } else {
      (void)bary_coeffs(coef, blk, NC, lane, t1R, b.consts + c.c_omega1, c.calls1, B + G1_C0, B + G1_K, 1);
    }
  }
  return flags;
}

// Exact ">= p" test (decoding an explicit Field128 element, VDAF-08 decode rejects x >= p).
__device__ __forceinline__ bool ge_exact(uint4 v) {
  return v.w == 0xFFFFFFFFu && (v.z > 0xFFFFFFE4u || (v.z == 0xFFFFFFE4u && (v.x | v.y) != 0u));
}

// K1, helper (agg_id 1, aggregator.rs:1947), large launches: the measurement and proof shares are
// expanded from seeds by TurboSHAKE128 and the squeeze runs alongside the joint_rand_part absorb, one
// report per lane with both sponges in VGPRs (2 waves/SIMD). The leader (agg_id 0) has its own
// one-sponge kernel (xof_leader_kernel); launches under one fused wave per SIMD take the lane-split
// kernel (xof_lanes_kernel). Variants measured slower and removed: squeeze-only +
// absorb-only launches, sequential S/J permutations at 3 waves/SIMD.
constexpr uint32_t K1_WAVES = 4;  // waves (64-report blocks) per K1 workgroup
// PROBE (measurement variants, instantiated only by tools/kernel_probe.hip, never by the library):
// 1 = the measurement-share staging stores skipped at run time by a uniform branch the compiler cannot
// resolve (everything else as built), 2 = no per-block emission at all (stores, truncation, >= p screen),
// 3 = the stores without the truncation and the screen. The variants write a sink to flags so nothing is dead.
template <bool WIDE = false, int PROBE = 0>
__global__ __launch_bounds__(64 * K1_WAVES, 1) void xof_kernel(Cfg c, Bufs b) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t blk = (uint64_t)blockIdx.x * K1_WAVES + (threadIdx.x >> 6);
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint64_t r0 = blk * 64 + lane;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;

  const uint8_t* hs = b.his + (uint64_t)c.his_bytes * r;
  uint32_t flags = 0;
  const uint32_t MB = c.meas_len * 16;
  const uint32_t ML = 42 + MB;
  const uint32_t NM = (MB + 167) / 168;  // measurement-share blocks of 168 bytes
  const uint32_t b_last = ML / 168;      // last absorbed block (b_last <= NM)

  // ---- measurement share fused with the joint_rand_part absorb --------------------
  // S: XOF(k_meas, DST(1), [1]) squeezed 168 bytes (block m of the measurement share) per block.
  // J: XOF(k_blind, DST(7), [agg_id] || nonce || enc(meas_share))   (absorbing those bytes)
  // J's message block m is meas bytes [168m - 42, 168m + 126): the 42-byte header makes it a
  // 16-bit funnel shift (v_alignbit_b32) of the words of blocks m-1 and m. After block m is
  // consumed S (-> block m+1) and J (absorb block m) permute together: two independent streams
  // (keccak_p12_x2).
  uint32_t S[50], J[50];
  {
    uint32_t kmeas[4];
    load16(hs, kmeas);
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 1, kmeas);
    blk_put_byte(m, pos, 1);
    blk_pad(m, pos + 1);
    sponge_oneblock(S, m);
  }
  uint32_t hdr[11];
  {
    uint32_t nonce[4], kblind[4];
    load16(b.nonces + 16 * r, nonce);
    load16(hs + 32, kblind);
    Block h;
    blk_zero(h);
    int pos = blk_xof_prefix(h, c.dst_id, 7, kblind);
    blk_put_byte(h, pos, 1);  // agg_id
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(h, pos + 1 + 4 * i, nonce[i]);
#pragma unroll
    for (int w = 0; w < 11; w++) hdr[w] = h.w[w];  // 42 header bytes
  }
  uint32_t prev[11];
  uint32_t carry0 = 0, carry1 = 0;
  uint32_t gmax = 0;  // running ge_screen over every sampled element
  TruncW tr;
  truncw_zero(tr);
  tr.j = 0;
  tr.i = 0;
  f128 trunc_lo = make128(0, 0);
  uint4* const mp = b.meas + il_idx(blk, c.meas_len, 0, lane);
  uint4* const op = b.outs + il_idx(blk, c.out_len, 0, lane);
  uint32_t sink = 0;
  auto emit = [&](uint32_t e, uint4 v) {
    if constexpr (PROBE == 1) {
      if (b.force_slow == 0x5EED5EEDu && e < c.meas_len) mp[(uint64_t)e * IL] = v;  // never true at run time
      emit_meas<WIDE, false>(c, mp, op, e, v, gmax, tr, trunc_lo);
    } else if constexpr (PROBE == 3) {
      if (e < c.meas_len) mp[(uint64_t)e * IL] = v;
    } else {
      emit_meas<WIDE>(c, mp, op, e, v, gmax, tr, trunc_lo);
    }
  };
  // emit the measurement elements of block m (10 or 11, by parity)
  auto emit_block = [&](uint32_t m) {
    if constexpr (PROBE == 2) {
      sink ^= S[0] ^ S[41];
      return;
    }
    const uint32_t e0 = 21 * (m >> 1);
    if ((m & 1) == 0) {
#pragma unroll
      for (int ci = 0; ci < 10; ci++) emit(e0 + ci, make_uint4(S[4 * ci], S[4 * ci + 1], S[4 * ci + 2], S[4 * ci + 3]));
      carry0 = S[40];
      carry1 = S[41];
    } else {
      const uint32_t c0 = carry0, c1 = carry1;
      emit(e0 + 10, make_uint4(c0, c1, S[0], S[1]));
#pragma unroll
      for (int ci = 0; ci < 10; ci++)
        emit(e0 + 11 + ci, make_uint4(S[2 + 4 * ci], S[3 + 4 * ci], S[4 + 4 * ci], S[5 + 4 * ci]));
    }
  };
  // J ^= message block m built from S (block m, if present) and prev (block m-1)
  auto absorb_block = [&](uint32_t m, bool have) {
    const uint32_t s0 = have ? S[0] : 0u;
    if (m == 0) {
#pragma unroll
      for (int w = 0; w < 10; w++) J[w] = hdr[w];
      J[10] = (hdr[10] & 0xffffu) | (s0 << 16);
#pragma unroll
      for (int w = 11; w < 50; w++) J[w] = 0;
    } else {
#pragma unroll
      for (int w = 0; w < 10; w++) J[w] ^= alignbit(prev[w + 1], prev[w], 16);
      J[10] ^= alignbit(s0, prev[10], 16);
    }
    if (have) {
#pragma unroll
      for (int w = 11; w < 42; w++) J[w] ^= alignbit(S[w - 10], S[w - 11], 16);
#pragma unroll
      for (int w = 0; w < 11; w++) prev[w] = S[31 + w];
    }
  };
  // last absorbed block m: only message bytes [168m, ML) are absorbed, then TurboSHAKE padding
  // (D = 0x01 after the message, 0x80 in byte 167)
  auto absorb_last = [&](uint32_t m, bool have) {
    const uint32_t nb = ML - 168 * m;  // message bytes in this block (< 168)
    uint32_t jw[42];
    const uint32_t s0 = have ? S[0] : 0u;
    if (m == 0) {
#pragma unroll
      for (int w = 0; w < 10; w++) jw[w] = hdr[w];
      jw[10] = (hdr[10] & 0xffffu) | (s0 << 16);
#pragma unroll
      for (int w = 0; w < 50; w++) J[w] = 0;
    } else {
#pragma unroll
      for (int w = 0; w < 10; w++) jw[w] = alignbit(prev[w + 1], prev[w], 16);
      jw[10] = alignbit(s0, prev[10], 16);
    }
#pragma unroll
    for (int w = 11; w < 42; w++) jw[w] = have ? alignbit(S[w - 10], S[w - 11], 16) : 0u;
#pragma unroll
    for (int w = 0; w < 42; w++) {
      const uint32_t lo_b = 4 * w;
      if (lo_b >= nb)
        jw[w] = 0;
      else if (lo_b + 4 > nb)
        jw[w] &= (1u << (8 * (nb - lo_b))) - 1u;
      if ((uint32_t)w == (nb >> 2)) jw[w] ^= 1u << (8 * (nb & 3));
    }
    jw[41] ^= 0x80000000u;
#pragma unroll
    for (int w = 0; w < 42; w++) J[w] ^= jw[w];
    keccak_p12(J);
  };
  // advance to block m+1: S squeezes together with J's permutation
  auto advance = [&](uint32_t m) {
    if (m + 1 < NM)
      keccak_p12_x2(S, J);
    else
      keccak_p12(J);
  };
  // blocks m = 0 .. b_last (b_last <= NM); blocks m < NM hold measurement bytes. Block 0 is
  // peeled so that the 42-byte header is dead inside the main loop.
  emit_block(0);
  if (b_last == 0) {
    absorb_last(0, true);
  } else {
    absorb_block(0, true);
    advance(0);
#pragma unroll 1
    for (uint32_t m = 1; m < b_last; m++) {  // m < b_last <= NM: block m holds measurement bytes
      emit_block(m);
      absorb_block(m, true);
      advance(m);
    }
    const bool have = b_last < NM;
    if (have) emit_block(b_last);
    absorb_last(b_last, have);
  }
  uint32_t own_part[4] = {J[0], J[1], J[2], J[3]};

  // ---- proof share: XOF(k_proofs, DST(2), [PROOFS=1, agg_id=1]) ----------------------
  uint4* const pp = b.proof + il_idx(blk, c.proof_len, 0, lane);
  {
    uint32_t kproof[4];
    load16(hs + 16, kproof);
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 2, kproof);
    blk_put_byte(m, pos, 1);
    blk_put_byte(m, pos + 1, 1);
    blk_pad(m, pos + 2);
    sponge_oneblock(S, m);
  }
  const uint32_t NP = (c.proof_len * 16 + 167) / 168;
#pragma unroll 1
  for (uint32_t m = 0; m < NP; m++) {
    if (m > 0) keccak_p12(S);
    const uint32_t e0 = 21 * (m >> 1);
    if ((m & 1) == 0) {
#pragma unroll
      for (int ci = 0; ci < 10; ci++)
        emit_proof(c, pp, e0 + ci, make_uint4(S[4 * ci], S[4 * ci + 1], S[4 * ci + 2], S[4 * ci + 3]), gmax);
      carry0 = S[40];
      carry1 = S[41];
    } else {
      emit_proof(c, pp, e0 + 10, make_uint4(carry0, carry1, S[0], S[1]), gmax);
#pragma unroll
      for (int ci = 0; ci < 10; ci++)
        emit_proof(c, pp, e0 + 11 + ci, make_uint4(S[2 + 4 * ci], S[3 + 4 * ci], S[4 + 4 * ci], S[5 + 4 * ci]), gmax);
    }
  }
  if (gmax == 0xFFFFFFFFu) flags |= FLAG_SLOW;

  uint32_t nonce[4];
  load16(b.nonces + 16 * r, nonce);
  uint32_t part_l[4], lead_part[4];
  load16(b.ps + (uint64_t)c.ps_bytes * r, part_l);
  load16(b.lps + (uint64_t)c.lps_bytes * r + c.lps_bytes - 16, lead_part);
  flags = xof_tail(c, b, blk, lane, r, r0 < b.n, nonce, part_l, lead_part, own_part, flags, false);
  if constexpr (PROBE != 0) flags = (sink ^ gmax ^ (uint32_t)tr.T[0]) & ~FLAG_SLOW;
  if (b.force_slow) flags |= FLAG_SLOW;
  if (r0 < b.n) b.flags[r0] = flags;
}

// ---------------------------------------------------------------------------- K1, lane-split helper
// A wave holds 32 reports. Lanes 0..31 (the S half) run the measurement-share squeeze of report
// (lane & 31), lanes 32..63 (the J half) the joint_rand_part absorb of the same report: a lane
// carries ONE Keccak state (<= 128 VGPRs, 4 waves/SIMD, against 2 for the two-sponge fused kernel)
// and one keccak_p12 instruction stream advances both sponges. After each permutation the S half
// emits block m (stores, truncation, >= p screen) and forms J's message words of block m (the 16-bit
// funnel shift of blocks m-1 and m); v_permlane32_swap_b32 hands them to the J half,
// which XORs them into its state (the S half XORs the swap's zeros). The J half squeezes block 0
// itself (the same sponge) to build its first message block; after the measurement every lane runs
// the proof-share squeeze (emitted by the S half) and then the J half finishes the XOF tail.

// lanes 32..63 receive lanes 0..31's v; lanes 0..31 receive 0
__device__ __forceinline__ uint32_t lower_to_upper(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(0u, v, false, false);
  return r[0];
}

// Registers: the XOF tail is inlined (xof_tail<true>) and the kernel is built for two waves per SIMD, so
// nothing spills (no scratch); how many of its workgroups share a CU is capped at launch by dynamic LDS
// it does not use (Bufs::k1_lds, jx_engine_debug option 6), the placement the two-jobs shape wants
// (chain-latency-bound waves, at most two per SIMD).
template <bool WIDE>  // WIDE (bits > 32) carries 4 more truncation words
__global__ __launch_bounds__(64 * K1_WAVES, 2) void xof_lanes_kernel(Cfg c, Bufs b) {
  const uint32_t lane = threadIdx.x & 63;
  const bool jh = lane >= 32;
  const uint64_t gw = (uint64_t)blockIdx.x * K1_WAVES + (threadIdx.x >> 6);  // 32 reports per wave
  const uint64_t blk = gw >> 1;
  const uint32_t il = ((uint32_t)gw & 1u) * 32u + (lane & 31u);  // this report's slot in its 64-report block
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint64_t r0 = blk * 64 + il;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint8_t* hs = b.his + (uint64_t)c.his_bytes * r;
  const uint32_t MB = c.meas_len * 16;
  const uint32_t ML = 42 + MB;
  const uint32_t NM = (MB + 167) / 168;
  const uint32_t b_last = ML / 168;

  uint32_t st[50];
  {  // squeeze block 0 = XOF(k_meas, DST(1), [1]) in both halves
    uint32_t kmeas[4];
    load16(hs, kmeas);
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 1, kmeas);
    blk_put_byte(m, pos, 1);
    blk_pad(m, pos + 1);
    sponge_oneblock(st, m);
  }
  uint32_t hdr[11];
  {
    uint32_t nonce[4], kblind[4];
    load16(b.nonces + 16 * r, nonce);
    load16(hs + 32, kblind);
    Block h;
    blk_zero(h);
    int pos = blk_xof_prefix(h, c.dst_id, 7, kblind);
    blk_put_byte(h, pos, 1);  // agg_id
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(h, pos + 1 + 4 * i, nonce[i]);
#pragma unroll
    for (int w = 0; w < 11; w++) hdr[w] = h.w[w];
  }
  // aux: the half-specific state carried across permutations, in the SAME registers for both halves.
  // S half: the truncation word columns T0..T3 (8 words), the element carry (2), the >= p screen
  // (1) [, WIDE: the low 32-bit truncation (4)]. J half: pv = the raw words 31..41 of the previous
  // squeezed block (the 16-bit funnel shift of J's message words 0..10 needs them).
  constexpr int NAUX = WIDE ? 15 : 11;
  uint32_t aux[NAUX];
#pragma unroll
  for (int w = 0; w < NAUX; w++) aux[w] = 0;
  uint4* const mp = b.meas + il_idx(blk, c.meas_len, 0, il);
  uint4* const op = b.outs + il_idx(blk, c.out_len, 0, il);
  // uniform truncation position (output element ti, bit tj) of the next measurement element
  uint32_t tj = 0, ti = 0;
  const uint32_t tlen = c.out_is_meas ? 0u : min(c.trunc_len, c.meas_len);
  // S half (call inside `if (!jh)`): store the elements of squeezed block m, screen them, and add
  // them into the truncation word columns; an output element is finished every `bits` elements
  auto s_emit_block = [&](uint32_t m) {
    TruncW tr;
#pragma unroll
    for (int w = 0; w < 4; w++) tr.T[w] = (uint64_t)aux[2 * w] | ((uint64_t)aux[2 * w + 1] << 32);
    tr.j = tj;
    tr.i = ti;
    uint32_t carry0 = aux[8], carry1 = aux[9], gmax = aux[10];
    f128 trunc_lo = make128(0, 0);
    if constexpr (WIDE) trunc_lo = make128((uint64_t)aux[11] | ((uint64_t)aux[12] << 32), (uint64_t)aux[13] | ((uint64_t)aux[14] << 32));
    auto emit = [&](uint32_t e, uint4 v) {
      if (e >= c.meas_len) return;
      gmax = max(gmax, ge_screen(v));
      mp[(uint64_t)e * IL] = v;
      if (e < tlen) {
        const uint32_t sh = opaque_u32(1u << (WIDE ? (tr.j & 31u) : tr.j));
        tr.T[0] += (uint64_t)v.x * sh;
        tr.T[1] += (uint64_t)v.y * sh;
        tr.T[2] += (uint64_t)v.z * sh;
        tr.T[3] += (uint64_t)v.w * sh;
        ++tr.j;
        if (WIDE && tr.j == 32 && c.bits > 32) {
          trunc_lo = truncw_value(tr);
          truncw_zero(tr);
        }
        if (tr.j == c.bits) {
          f128 val = truncw_value(tr);
          if (WIDE && c.bits > 32) val = add128(trunc_lo, shl32_mod(val));
          op[(uint64_t)tr.i * IL] = f_to_u4(val);
          truncw_zero(tr);
          tr.j = 0;
          tr.i++;
        }
      }
    };
    const uint32_t e0 = 21 * (m >> 1);
    if ((m & 1) == 0) {
#pragma unroll
      for (int ci = 0; ci < 10; ci++)
        emit(e0 + ci, make_uint4(st[4 * ci], st[4 * ci + 1], st[4 * ci + 2], st[4 * ci + 3]));
      carry0 = st[40];
      carry1 = st[41];
    } else {
      emit(e0 + 10, make_uint4(carry0, carry1, st[0], st[1]));
#pragma unroll
      for (int ci = 0; ci < 10; ci++)
        emit(e0 + 11 + ci, make_uint4(st[2 + 4 * ci], st[3 + 4 * ci], st[4 + 4 * ci], st[5 + 4 * ci]));
    }
#pragma unroll
    for (int w = 0; w < 4; w++) {
      aux[2 * w] = (uint32_t)tr.T[w];
      aux[2 * w + 1] = (uint32_t)(tr.T[w] >> 32);
    }
    aux[8] = carry0;
    aux[9] = carry1;
    aux[10] = gmax;
    if constexpr (WIDE) {
      aux[11] = (uint32_t)trunc_lo.lo;
      aux[12] = (uint32_t)(trunc_lo.lo >> 32);
      aux[13] = (uint32_t)trunc_lo.hi;
      aux[14] = (uint32_t)(trunc_lo.hi >> 32);
    }
  };
  // uniform: advance (ti, tj) past the truncated elements of block m
  auto advance_trunc = [&](uint32_t m) {
    const uint32_t e0 = 21 * (m >> 1) + ((m & 1) ? 10u : 0u);
    const uint32_t e1 = e0 + ((m & 1) ? 11u : 10u);
    const uint32_t cnt = e1 <= tlen ? e1 - e0 : (e0 < tlen ? tlen - e0 : 0u);
    tj += cnt;
    while (tj >= c.bits && cnt) {
      tj -= c.bits;
      ti++;
    }
  };
  // last absorbed block: message bytes [0, nb) of the block, then TurboSHAKE padding
  auto pad_last = [&](uint32_t* jw, uint32_t nb) {
#pragma unroll
    for (int w = 0; w < 42; w++) {
      const uint32_t lo_b = 4 * w;
      if (lo_b >= nb)
        jw[w] = 0;
      else if (lo_b + 4 > nb)
        jw[w] &= (1u << (8 * (nb - lo_b))) - 1u;
      if ((uint32_t)w == (nb >> 2)) jw[w] ^= 1u << (8 * (nb & 3));
    }
    jw[41] ^= 0x80000000u;
  };

  if (!jh) s_emit_block(0);
  advance_trunc(0);
  {
    // J's message block 0: the 42-byte header || S_0[0, 126) (the J half holds S_0 too)
    uint32_t jw[42];
#pragma unroll
    for (int w = 0; w < 10; w++) jw[w] = hdr[w];
    jw[10] = (hdr[10] & 0xffffu) | (st[0] << 16);
#pragma unroll
    for (int w = 11; w < 42; w++) jw[w] = alignbit(st[w - 10], st[w - 11], 16);
    if (b_last == 0) pad_last(jw, ML);
    if (jh) {
#pragma unroll
      for (int w = 0; w < 11; w++) aux[w] = st[31 + w];
#pragma unroll
      for (int w = 0; w < 42; w++) st[w] = jw[w];
#pragma unroll
      for (int w = 42; w < 50; w++) st[w] = 0;
    }
  }
#pragma unroll 1
  for (uint32_t m = 1; m <= b_last; m++) {
    keccak_p12(st);  // S: squeeze block m; J: absorb block m - 1 (unrolled: slower, see keccak_p12_unrolled)
    const bool have = m < NM;
    if (have) {
      if (!jh) s_emit_block(m);
      advance_trunc(m);
    }
    // S -> J: the shifted message words 11..41 of block m (formed by the S half) and the raw words 0 and
    // 31..41 (J's funnel shift of words 0..10 and its next pv). v_permlane32_swap moves lanes 0..31 of
    // its second operand into lanes 32..63 of the first; the first operand is any dead register (the
    // previous swap's clobbered source), so the shifted words cost one swap each.
    uint32_t jw[42], raw[12];
    uint32_t dead = st[0];
    if (have) {
#pragma unroll
      for (int w = 11; w < 42; w++) {
        const auto r2 = __builtin_amdgcn_permlane32_swap(dead, alignbit(st[w - 10], st[w - 11], 16), false, false);
        jw[w] = r2[0];
        dead = r2[1];
      }
      {
        const auto r2 = __builtin_amdgcn_permlane32_swap(dead, st[0], false, false);
        raw[0] = r2[0];
        dead = r2[1];
      }
#pragma unroll
      for (int k = 0; k < 11; k++) {
        const auto r2 = __builtin_amdgcn_permlane32_swap(dead, st[31 + k], false, false);
        raw[1 + k] = r2[0];
        dead = r2[1];
      }
    } else {
#pragma unroll
      for (int w = 11; w < 42; w++) jw[w] = 0;
#pragma unroll
      for (int k = 0; k < 12; k++) raw[k] = 0;
    }
    if (jh) {
#pragma unroll
      for (int w = 0; w < 10; w++) jw[w] = alignbit(aux[w + 1], aux[w], 16);
      jw[10] = alignbit(raw[0], aux[10], 16);
      if (m == b_last) pad_last(jw, ML - 168 * m);
#pragma unroll
      for (int w = 0; w < 42; w++) st[w] ^= jw[w];
#pragma unroll
      for (int k = 0; k < 11; k++) aux[k] = raw[1 + k];
    }
  }
  keccak_p12(st);  // J: absorb block b_last
  uint32_t own_part[4] = {st[0], st[1], st[2], st[3]};

  // proof share: XOF(k_proofs, DST(2), [PROOFS=1, agg_id=1]) in both halves, emitted by the S half
  uint4* const pp = b.proof + il_idx(blk, c.proof_len, 0, il);
  {
    uint32_t kproof[4];
    load16(hs + 16, kproof);
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 2, kproof);
    blk_put_byte(m, pos, 1);
    blk_put_byte(m, pos + 1, 1);
    blk_pad(m, pos + 2);
    sponge_oneblock(st, m);
  }
  uint32_t carry0 = 0, carry1 = 0, gmax = aux[10];  // S half: the measurement's screen so far
  auto emit_p = [&](uint32_t e, uint4 v) {
    if (e >= c.proof_len) return;
    gmax = max(gmax, ge_screen(v));
    if (!jh) pp[(uint64_t)e * IL] = v;
  };
  const uint32_t NP = (c.proof_len * 16 + 167) / 168;
#pragma unroll 1
  for (uint32_t m = 0; m < NP; m++) {
    if (m > 0) keccak_p12(st);
    const uint32_t e0 = 21 * (m >> 1);
    if ((m & 1) == 0) {
#pragma unroll
      for (int ci = 0; ci < 10; ci++) emit_p(e0 + ci, make_uint4(st[4 * ci], st[4 * ci + 1], st[4 * ci + 2], st[4 * ci + 3]));
      carry0 = st[40];
      carry1 = st[41];
    } else {
      emit_p(e0 + 10, make_uint4(carry0, carry1, st[0], st[1]));
#pragma unroll
      for (int ci = 0; ci < 10; ci++)
        emit_p(e0 + 11 + ci, make_uint4(st[2 + 4 * ci], st[3 + 4 * ci], st[4 + 4 * ci], st[5 + 4 * ci]));
    }
  }
  // the S half's screen (measurement + proof elements) goes to the J half, which finishes the report
  const uint32_t smax = lower_to_upper(gmax);
  if (jh) {
    uint32_t flags = smax == 0xFFFFFFFFu ? FLAG_SLOW : 0u;
    uint32_t nonce[4], part_l[4], lead_part[4];
    load16(b.nonces + 16 * r, nonce);
    load16(b.ps + (uint64_t)c.ps_bytes * r, part_l);
    load16(b.lps + (uint64_t)c.lps_bytes * r + c.lps_bytes - 16, lead_part);
    [[clang::always_inline]] flags =
        xof_tail<true>(c, b, blk, il, r, r0 < b.n, nonce, part_l, lead_part, own_part, flags, false);
    if (b.force_slow) flags |= FLAG_SLOW;
    if (r0 < b.n) b.flags[r0] = flags;
  }
}

// ---------------------------------------------------------------------------- K1, lane-pair helper
// Launches that would give the lane-split kernel at most one wave per SIMD are bound by how fast ONE
// wave issues its own dependent chain (a lone wave64 issues a VALU op every ~4-6.5 cycles, against 2
// with a partner wave, MI355X_MICROARCH.md 'vector-instruction ISSUE cost'). This kernel halves each
// sponge's chain instead: a Keccak state is split over a lane PAIR, the even lane holding the low and
// the odd lane the high 32-bit halves of the 25 64-bit words (25 VGPRs each). A 64-bit rotation is
// then one v_alignbit_b32 per lane between its own half and its partner's (fetched by a DPP quad_perm
// [1,0,3,2] move): 124 instructions per round on each lane instead of 190 on one. Four lanes per
// report: lanes 2k / 2k+1 of the lower half squeeze the measurement share (S, low / high halves),
// lanes 32+2k / 33+2k absorb the joint_rand_part (J), 16 reports per wave, twice the waves of the
// lane-split kernel and 1.45x its instructions per report, so it is the choice only below one
// lane-split wave per SIMD (FixedPointBoundedL2VecSum 16 x 10000 at <= 32,768 reports per launch).
// The S lanes emit the elements (each lane two of an element's four words), keep the truncation
// word columns of their two words, and form J's message words from their own and their partner's
// halves; v_permlane32_swap hands them to the J lanes.

// the partner lane's value (lane ^ 1)
__device__ __forceinline__ uint32_t pswap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1, 0, 3, 2]
}
__device__ __forceinline__ uint64_t pswap64(uint64_t v) {
  return (uint64_t)pswap((uint32_t)v) | ((uint64_t)pswap((uint32_t)(v >> 32)) << 32);
}
// this lane's half of rotl64(word, N) from its own and its partner's half (the same formula on both)
template <int N>
__device__ __forceinline__ uint32_t hrot(uint32_t own, uint32_t par) {
  if constexpr (N == 0)
    return own;
  else if constexpr (N < 32)
    return alignbit(own, par, 32 - N);
  else if constexpr (N == 32)
    return par;
  else
    return alignbit(par, own, 64 - N);
}
template <int I>
__device__ __forceinline__ void rho_pi_half_one(const uint32_t* s, uint32_t* B) {
  constexpr int R = RotOf<I>::value;
  if constexpr (R == 0)
    B[PiDst<I>::value] = s[I];
  else
    B[PiDst<I>::value] = hrot<R>(s[I], pswap(s[I]));
}
template <int... Is>
__device__ __forceinline__ void rho_pi_half_all(const uint32_t* s, uint32_t* B, IndexSeq<Is...>) {
  (rho_pi_half_one<Is>(s, B), ...);
}
// One Keccak-f[1600] round on this lane's half s[25]; rc = this lane's half of the round constant.
// theta parity 10 v_bitop3, partner parities 5 DPP moves, D 5 alignbit + 5 xor, D applied 25 xor,
// rho 24 DPP moves + 24 alignbit, chi 25 v_bitop3, iota 1: 124 VALU.
__device__ __forceinline__ void keccak_round_half(uint32_t* s, uint32_t rc) {
  uint32_t C[5], Cp[5], B[25];
#pragma unroll
  for (int x = 0; x < 5; x++) C[x] = xor3(xor3(s[x], s[x + 5], s[x + 10]), s[x + 15], s[x + 20]);
#pragma unroll
  for (int x = 0; x < 5; x++) Cp[x] = pswap(C[x]);
#pragma unroll
  for (int x = 0; x < 5; x++) {
    const uint32_t D = C[(x + 4) % 5] ^ hrot<1>(C[(x + 1) % 5], Cp[(x + 1) % 5]);
#pragma unroll
    for (int y = 0; y < 5; y++) s[x + 5 * y] ^= D;
  }
  rho_pi_half_all(s, B, typename MakeSeq<25>::type{});
#pragma unroll
  for (int y = 0; y < 5; y++) {
#pragma unroll
    for (int x = 0; x < 5; x++) {
      const int i = x + 5 * y, i1 = (x + 1) % 5 + 5 * y, i2 = (x + 2) % 5 + 5 * y;
      s[i] = B[i] ^ (~B[i1] & B[i2]);
    }
  }
  s[0] ^= rc;
}
__device__ __forceinline__ void keccak_p12_half(uint32_t* s, bool hi) {
#pragma unroll 1
  for (int ir = 12; ir < 24; ir++) keccak_round_half(s, hi ? KECCAK_RC_HI[ir] : KECCAK_RC_LO[ir]);
}
// the same with the rounds unrolled (round constants as literals; see keccak_p12_unrolled)
__device__ __forceinline__ void keccak_p12_half_unrolled(uint32_t* s, bool hi) {
#pragma unroll
  for (int ir = 12; ir < 24; ir++) keccak_round_half(s, hi ? KECCAK_RC_HI[ir] : KECCAK_RC_LO[ir]);
}
// a ? x1 : x0 as bit operations on an opaque all-ones / zero mask: a select between two array elements
// written `a ? v[i + 1] : v[i]` becomes an indexed load v[i + a], which puts the array in scratch
__device__ __forceinline__ uint32_t msel(uint32_t m, uint32_t x0, uint32_t x1) { return x0 ^ ((x0 ^ x1) & m); }
// state := 0; absorb one final block (42 words, this lane takes words 2i + hi); permute
__device__ __forceinline__ void sponge_oneblock_half(uint32_t* s, const Block& m, bool hi) {
  const uint32_t hm = opaque_u32(hi ? 0xFFFFFFFFu : 0u);
#pragma unroll
  for (int i = 0; i < 21; i++) s[i] = msel(hm, m.w[2 * i], m.w[2 * i + 1]);
#pragma unroll
  for (int i = 21; i < 25; i++) s[i] = 0;
  keccak_p12_half(s, hi);
}

// UNR: the rounds of the block loop unrolled (round constants as literals): 4.03 -> 3.59 ms for launches of
// at most one pair-wave per SIMD, but slower with several waves per SIMD (64 x 1,000-report coalesced jobs:
// 12.5 -> 15.2 ms per launch), so the engine picks it only for the former (prep_core, k1_split 8).
template <bool UNR>
__global__ __launch_bounds__(64 * K1_WAVES, 2) void xof_pairs_kernel(Cfg c, Bufs b) {
  const uint32_t lane = threadIdx.x & 63;
  const bool jh = lane >= 32;     // J lanes
  const bool hi = (lane & 1u) != 0;  // high halves
  const uint32_t hm = opaque_u32(hi ? 0xFFFFFFFFu : 0u);
  const uint64_t gw = (uint64_t)blockIdx.x * K1_WAVES + (threadIdx.x >> 6);  // 16 reports per wave
  const uint64_t blk = gw >> 2;
  const uint32_t il = ((uint32_t)gw & 3u) * 16u + ((lane & 31u) >> 1);  // this report's slot in its 64-report block
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint64_t r0 = blk * 64 + il;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint8_t* hs = b.his + (uint64_t)c.his_bytes * r;
  const uint32_t MB = c.meas_len * 16;
  const uint32_t ML = 42 + MB;
  const uint32_t NM = (MB + 167) / 168;
  const uint32_t b_last = ML / 168;

  uint32_t h[25];
  {  // squeeze block 0 = XOF(k_meas, DST(1), [1]) on every lane pair
    uint32_t kmeas[4];
    load16(hs, kmeas);
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 1, kmeas);
    blk_put_byte(m, pos, 1);
    blk_pad(m, pos + 1);
    sponge_oneblock_half(h, m, hi);
  }
  uint32_t hdr[11];
  {
    uint32_t nonce[4], kblind[4];
    load16(b.nonces + 16 * r, nonce);
    load16(hs + 32, kblind);
    Block hb;
    blk_zero(hb);
    int pos = blk_xof_prefix(hb, c.dst_id, 7, kblind);
    blk_put_byte(hb, pos, 1);  // agg_id
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(hb, pos + 1 + 4 * i, nonce[i]);
#pragma unroll
    for (int w = 0; w < 11; w++) hdr[w] = hb.w[w];
  }
  // S lanes: the truncation word columns of this lane's two words of an element (Ta: word 0 | 1, Tb:
  // word 2 | 3), the element carry, the >= p screen (meaningful on the high lane: w & (z | 0x1F)) and
  // the own halves 15..20 of the previous squeezed block (J's message words 0..10 need them)
  uint64_t Ta = 0, Tb = 0;
  uint32_t carry = 0, gmax = 0, pv[6];
#pragma unroll
  for (int k = 0; k < 6; k++) pv[k] = 0;
  uint32_t* const mp32 = reinterpret_cast<uint32_t*>(b.meas + il_idx(blk, c.meas_len, 0, il)) + (hi ? 1u : 0u);
  uint4* const op = b.outs + il_idx(blk, c.out_len, 0, il);
  uint32_t tj = 0, ti = 0;  // uniform truncation position of the next measurement element
  const uint32_t tlen = c.out_is_meas ? 0u : min(c.trunc_len, c.meas_len);
  // S lanes: element e's words (a, bw) = (x, z) on the low lane, (y, w) on the high lane
  auto emit = [&](uint32_t e, uint32_t a, uint32_t bw, uint32_t& tjl, uint32_t& til) {
    if (e >= c.meas_len) return;
    const uint32_t pb = pswap(bw);
    gmax = max(gmax, bw & (pb | 0x1Fu));
    mp32[(uint64_t)e * IL * 4] = a;
    mp32[(uint64_t)e * IL * 4 + 2] = bw;
    if (e < tlen) {
      const uint32_t sh = opaque_u32(1u << tjl);
      Ta += (uint64_t)a * sh;
      Tb += (uint64_t)bw * sh;
      ++tjl;
      if (tjl == c.bits) {  // V = T0 + T1 2^32 + T2 2^64 + T3 2^96, finished on the low lane
        TruncW tr;
        tr.T[0] = Ta;
        tr.T[1] = pswap64(Ta);
        tr.T[2] = Tb;
        tr.T[3] = pswap64(Tb);
        const f128 val = truncw_value(tr);
        if (!hi) op[(uint64_t)til * IL] = f_to_u4(val);
        Ta = 0;
        Tb = 0;
        tjl = 0;
        til++;
      }
    }
  };
  auto s_emit_block = [&](uint32_t m) {
    uint32_t tjl = tj, til = ti;
    const uint32_t e0 = 21 * (m >> 1);
    if ((m & 1) == 0) {
#pragma unroll
      for (int ci = 0; ci < 10; ci++) emit(e0 + ci, h[2 * ci], h[2 * ci + 1], tjl, til);
      carry = h[20];
    } else {
      emit(e0 + 10, carry, h[0], tjl, til);
#pragma unroll
      for (int ci = 0; ci < 10; ci++) emit(e0 + 11 + ci, h[1 + 2 * ci], h[2 + 2 * ci], tjl, til);
    }
  };
  // uniform: advance (ti, tj) past the truncated elements of block m
  auto advance_trunc = [&](uint32_t m) {
    const uint32_t e0 = 21 * (m >> 1) + ((m & 1) ? 10u : 0u);
    const uint32_t e1 = e0 + ((m & 1) ? 11u : 10u);
    const uint32_t cnt = e1 <= tlen ? e1 - e0 : (e0 < tlen ? tlen - e0 : 0u);
    tj += cnt;
    while (tj >= c.bits && cnt) {
      tj -= c.bits;
      ti++;
    }
  };
  // last absorbed block: message bytes [0, nb) of the block, then TurboSHAKE padding; jw[i] is this
  // lane's word 2i + hi
  auto pad_last_half = [&](uint32_t* jw, uint32_t nb) {
#pragma unroll
    for (int i = 0; i < 21; i++) {
      const uint32_t w = 2 * i + (hi ? 1u : 0u);
      const uint32_t lo_b = 4 * w;
      if (lo_b >= nb)
        jw[i] = 0;
      else if (lo_b + 4 > nb)
        jw[i] &= (1u << (8 * (nb - lo_b))) - 1u;
      if (w == (nb >> 2)) jw[i] ^= 1u << (8 * (nb & 3));
      if (w == 41) jw[i] ^= 0x80000000u;
    }
  };
  // J's message words of a block from the S stream E (the previous block's halves 15..20, then the
  // current block's): J word 2i + hi = alignbit(E_own[i - 5], E_par[i - 6 + hi], 16). Past the share
  // (the block after the last squeezed one, m == b_last == NM) the current halves are a squeezed block
  // that is not part of the message: every word they reach lies at or past byte nb, which the padding
  // of that last block clears.
  auto message = [&](uint32_t* jw) {
    uint32_t Eo[21], Ep[22];
#pragma unroll
    for (int k = 0; k < 5; k++) Eo[k] = pv[k + 1];
#pragma unroll
    for (int k = 0; k < 16; k++) Eo[5 + k] = h[k];
#pragma unroll
    for (int k = 0; k < 6; k++) Ep[k] = pswap(pv[k]);
#pragma unroll
    for (int k = 0; k < 16; k++) Ep[6 + k] = pswap(h[k]);
#pragma unroll
    for (int i = 0; i < 21; i++) jw[i] = alignbit(Eo[i], msel(hm, Ep[i], Ep[i + 1]), 16);
  };

  if (!jh) s_emit_block(0);
  advance_trunc(0);
  {
    // J's message block 0: the 42-byte header || S_0[0, 126) (the J lanes hold S_0 too)
    uint32_t Hp[16];
#pragma unroll
    for (int k = 0; k < 16; k++) Hp[k] = pswap(h[k]);
    uint32_t jw[21];
#pragma unroll
    for (int i = 0; i < 5; i++) jw[i] = msel(hm, hdr[2 * i], hdr[2 * i + 1]);
    jw[5] = msel(hm, (hdr[10] & 0xffffu) | (h[0] << 16), alignbit(h[0], Hp[0], 16));
#pragma unroll
    for (int i = 6; i < 21; i++) jw[i] = alignbit(h[i - 5], msel(hm, Hp[i - 6], Hp[i - 5]), 16);
    if (b_last == 0) pad_last_half(jw, ML);
#pragma unroll
    for (int k = 0; k < 6; k++) pv[k] = h[15 + k];
    if (jh) {
#pragma unroll
      for (int i = 0; i < 21; i++) h[i] = jw[i];
#pragma unroll
      for (int i = 21; i < 25; i++) h[i] = 0;
    }
  }
#pragma unroll 1
  for (uint32_t m = 1; m <= b_last; m++) {
    if constexpr (UNR)
      keccak_p12_half_unrolled(h, hi);  // S: squeeze block m; J: absorb block m - 1
    else
      keccak_p12_half(h, hi);
    const bool have = m < NM;
    if (have) {
      if (!jh) s_emit_block(m);
      advance_trunc(m);
    }
    uint32_t msg[21], jw[21];
    message(msg);
#pragma unroll
    for (int k = 0; k < 6; k++) pv[k] = h[15 + k];
    uint32_t dead = h[0];
#pragma unroll
    for (int i = 0; i < 21; i++) {  // S lanes -> J lanes (lane l -> l + 32, the same half)
      const auto r2 = __builtin_amdgcn_permlane32_swap(dead, msg[i], false, false);
      jw[i] = r2[0];
      dead = r2[1];
    }
    if (jh) {
      if (m == b_last) pad_last_half(jw, ML - 168 * m);
#pragma unroll
      for (int i = 0; i < 21; i++) h[i] ^= jw[i];
    }
  }
  keccak_p12_half(h, hi);  // J: absorb block b_last
  // J state words 0..3: the low J lane holds words 0, 2 and gets 1, 3 from its partner
  const uint32_t p0 = pswap(h[0]), p1 = pswap(h[1]);
  uint32_t own_part[4] = {h[0], p0, h[1], p1};

  // proof share: XOF(k_proofs, DST(2), [PROOFS=1, agg_id=1]) on every lane pair, emitted by the S lanes
  uint32_t* const pp32 = reinterpret_cast<uint32_t*>(b.proof + il_idx(blk, c.proof_len, 0, il)) + (hi ? 1u : 0u);
  {
    uint32_t kproof[4];
    load16(hs + 16, kproof);
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 2, kproof);
    blk_put_byte(m, pos, 1);
    blk_put_byte(m, pos + 1, 1);
    blk_pad(m, pos + 2);
    sponge_oneblock_half(h, m, hi);
  }
  auto emit_p = [&](uint32_t e, uint32_t a, uint32_t bw) {
    if (e >= c.proof_len) return;
    const uint32_t pb = pswap(bw);
    gmax = max(gmax, bw & (pb | 0x1Fu));
    if (!jh) {
      pp32[(uint64_t)e * IL * 4] = a;
      pp32[(uint64_t)e * IL * 4 + 2] = bw;
    }
  };
  carry = 0;
  const uint32_t NP = (c.proof_len * 16 + 167) / 168;
#pragma unroll 1
  for (uint32_t m = 0; m < NP; m++) {
    if (m > 0) keccak_p12_half(h, hi);
    const uint32_t e0 = 21 * (m >> 1);
    if ((m & 1) == 0) {
#pragma unroll
      for (int ci = 0; ci < 10; ci++) emit_p(e0 + ci, h[2 * ci], h[2 * ci + 1]);
      carry = h[20];
    } else {
      emit_p(e0 + 10, carry, h[0]);
#pragma unroll
      for (int ci = 0; ci < 10; ci++) emit_p(e0 + 11 + ci, h[1 + 2 * ci], h[2 + 2 * ci]);
    }
  }
  // the high S lane's screen -> its low partner -> the low J lane, which finishes the report
  const uint32_t smax = lower_to_upper(pswap(gmax));
  if (jh && !hi) {
    uint32_t flags = smax == 0xFFFFFFFFu ? FLAG_SLOW : 0u;
    uint32_t nonce[4], part_l[4], lead_part[4];
    load16(b.nonces + 16 * r, nonce);
    load16(b.ps + (uint64_t)c.ps_bytes * r, part_l);
    load16(b.lps + (uint64_t)c.lps_bytes * r + c.lps_bytes - 16, lead_part);
    flags = xof_tail(c, b, blk, il, r, r0 < b.n, nonce, part_l, lead_part, own_part, flags, false);
    if (b.force_slow) flags |= FLAG_SLOW;
    if (r0 < b.n) b.flags[r0] = flags;
  }
}

// ---------------------------------------------------------------------------- K1, small helper launches
// A launch of a thousand reports or fewer (Janus's 10-1,000-report aggregation jobs, one at a time or a few
// coalesced) leaves most SIMDs empty, so K1's time is ONE report's chain: 762 squeeze + 763 absorb blocks for
// SumVec 8x1000, each a Keccak-p[1600,12]. The lane-pair kernel runs that chain at 124 dependent VALU per
// round per lane (4.0 ms per launch, profiles/r05_small_launch_kernels.json). This kernel spreads each
// sponge over 25 lanes, one 64-bit word per lane (lane = x + 5y), one report per wave: lanes 0..24 squeeze
// the measurement share (S), lanes 32..56 absorb the joint_rand_part (J). A round is 26 VALU per lane and
// two exchanges through the wave's own LDS region (kw_sync at each hand-off: a wave's LDS operations complete in
// order, so no barrier instruction is needed, only a compiler fence):
//   theta: every lane writes its word into a column-major table whose columns are padded with wrap copies
//          (slot c + 1 holds column c, slot 0 column 4, slot 6 column 0), then reads columns x - 1 and
//          x + 1 as five ds_read2_b64 at offsets (k, k + 10) from one base;
//   rho:   a per-lane rotation, two v_alignbit_b32 on operands ordered once per lane;
//   pi + chi: every lane writes its rotated word at its pi destination into a row-major table with rows
//          padded by wrap copies (slots 5, 6 = 0, 1), then reads B[x], B[x+1], B[x+2] of its row.
// Measured (tools/kernel_probe sweep, profiles/r05_words_sweep.jsonl): 2.5-2.7 ms per launch up to 1,024
// reports against 3.6 ms for the lane pairs (2.7-2.9 with the rounds in a loop: the unrolled rounds take
// the round constants as literals); equal at 2,048; beyond, issue-bound and slower. One exchange
// per round instead (each lane reading columns x - 1 .. x + 3 of the chi table and computing the next
// round's parities itself, 54 VALU per round) measured 3.5-3.8 ms: a lone wave pays more for the doubled
// VALU chain than for the second LDS round trip.
// S hands each squeezed block to J through a 27-word message window in LDS (the previous block's words
// 15..20, then the block), from which J lane w forms its message word w as one 48-bit funnel shift; the
// 42-byte header sits in the window's prefix for block 0. The output-share truncation runs afterwards in
// trunc_kernel (it needs `bits` consecutive elements that lie on different lanes here).
constexpr uint32_t KW_WAVES = 4;  // waves (reports) per workgroup
// per-wave LDS region, in 8-byte words: theta tables S / J, chi tables S / J, message window, init block, sink
constexpr uint32_t KW_AS = 0, KW_AJ = 35, KW_BS = 70, KW_BJ = 105, KW_MSG = 140, KW_INIT = 167, KW_SINK = 188,
                   KW_WORDS = 189;
__constant__ uint8_t kw_rot_tab[25] = {JX_ROT_LIST};

struct KwLane {
  uint32_t aw1, aw2, ab;  // theta: write (own slot, wrap copy), read base (column x - 1)
  uint32_t bw1, bw2, bb;  // chi: write (pi destination, wrap copy), read base (B[x] of the lane's row)
  uint32_t pm, s;         // rho: operand order mask, v_alignbit amount
  uint32_t m0;            // iota: all-ones on word 0
};

// A hand-off between the lanes of one wave through its LDS region: every lane's earlier LDS writes are
// visible to every lane's later reads (and earlier reads complete before later writes). gfx950 completes a
// wave's LDS operations in order, so this emits no instruction; it forbids the compiler from moving LDS
// accesses across it, which it may otherwise do for pairs it proves distinct per thread (the C++ model does
// not order plain accesses of different lanes).
__device__ __forceinline__ void kw_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void kw_round(uint2* L, const KwLane& k, uint32_t& lo, uint32_t& hi, uint32_t rlo,
                                         uint32_t rhi) {
  L[k.aw1] = make_uint2(lo, hi);
  L[k.aw2] = make_uint2(lo, hi);
  kw_sync();  // theta table written -> read (the previous round's chi reads are behind the chi sync)
  uint2 cm[5], cp[5];
#pragma unroll
  for (int j = 0; j < 5; j++) {
    cm[j] = L[k.ab + j];
    cp[j] = L[k.ab + j + 10];
  }
  const uint32_t cml = xor3(xor3(cm[0].x, cm[1].x, cm[2].x), cm[3].x, cm[4].x);
  const uint32_t cmh = xor3(xor3(cm[0].y, cm[1].y, cm[2].y), cm[3].y, cm[4].y);
  const uint32_t cpl = xor3(xor3(cp[0].x, cp[1].x, cp[2].x), cp[3].x, cp[4].x);
  const uint32_t cph = xor3(xor3(cp[0].y, cp[1].y, cp[2].y), cp[3].y, cp[4].y);
  // D[x] = C[x - 1] ^ rotl64(C[x + 1], 1)
  lo = xor3(lo, cml, alignbit(cpl, cph, 31));
  hi = xor3(hi, cmh, alignbit(cph, cpl, 31));
  // rho: (P, Q) = the halves in the order this lane's rotation needs (see xof_words_kernel)
  const uint32_t P = msel(k.pm, hi, lo);
  const uint32_t Q = xor3(lo, hi, P);
  const uint32_t nh = alignbit(P, Q, k.s), nl = alignbit(Q, P, k.s);
  L[k.bw1] = make_uint2(nl, nh);
  L[k.bw2] = make_uint2(nl, nh);
  kw_sync();  // chi table written -> read (this round's theta reads are behind the theta sync)
  const uint2 b0 = L[k.bb], b1 = L[k.bb + 1], b2 = L[k.bb + 2];
  lo = (b0.x ^ (~b1.x & b2.x)) ^ (rlo & k.m0);
  hi = (b0.y ^ (~b1.y & b2.y)) ^ (rhi & k.m0);
}
__device__ __forceinline__ void kw_p12(uint2* L, const KwLane& k, uint32_t& lo, uint32_t& hi) {
#pragma unroll
  for (int ir = 12; ir < 24; ir++) kw_round(L, k, lo, hi, KECCAK_RC_LO[ir], KECCAK_RC_HI[ir]);
}

__global__ __launch_bounds__(64 * KW_WAVES) void xof_words_kernel(Cfg c, Bufs b) {
  __shared__ uint2 lds[KW_WAVES][KW_WORDS];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t r = (uint64_t)blockIdx.x * KW_WAVES + wv;
  if (r >= b.n) return;
  uint2* L = lds[wv];
  const uint64_t blk = r >> 6;
  const uint32_t il = (uint32_t)r & 63u;
  const bool jg = lane >= 32;         // J lanes
  const uint32_t i = lane & 31u;      // this lane's word of its sponge
  const bool act = i < 25;
  const bool sw21 = !jg && i < 21;    // S lanes holding a rate word
  const bool jw21 = jg && i < 21;     // J lanes absorbing a message word
  const uint32_t ia = act ? i : 0u, x = ia % 5u, y = ia / 5u;
  KwLane k;
  {
    const uint32_t A0 = jg ? KW_AJ : KW_AS, B0 = jg ? KW_BJ : KW_BS;
    const uint32_t xp = y, yp = (2u * x + 3u * y) % 5u;  // pi destination (column, row)
    k.aw1 = act ? A0 + (x + 1u) * 5u + y : KW_SINK;
    k.aw2 = !act ? KW_SINK : x == 4u ? A0 + y : x == 0u ? A0 + 30u + y : k.aw1;
    k.ab = A0 + x * 5u;
    k.bw1 = act ? B0 + yp * 7u + xp : KW_SINK;
    k.bw2 = !act ? KW_SINK : xp < 2u ? k.bw1 + 5u : k.bw1;
    k.bb = B0 + y * 7u + x;
    // rotl64 by R: with sw = R >= 32 and M = R mod 32, new hi = alignbit(P, Q, (32 - M) mod 32) and new lo =
    // alignbit(Q, P, ...), where P is the low half iff sw != (M == 0) (alignbit by 0 returns its second operand)
    const uint32_t R = kw_rot_tab[ia], M = R & 31u;
    k.pm = ((R >= 32u) != (M == 0u)) ? 0xFFFFFFFFu : 0u;
    k.s = (32u - M) & 31u;
    k.m0 = act && ia == 0u ? 0xFFFFFFFFu : 0u;
  }
  const uint8_t* hs = b.his + (uint64_t)c.his_bytes * r;
  const uint32_t MB = c.meas_len * 16;
  const uint32_t ML = 42 + MB;
  const uint32_t NM = (MB + 167) / 168;
  const uint32_t b_last = ML / 168;
  uint32_t lo = 0, hi = 0, gmax = 0;

  // S := the permuted one-block sponge of `m` (block word i on S lane i); J keeps its state
  auto s_init = [&](const Block& m) {
    if (lane == 0) {
#pragma unroll
      for (int w = 0; w < 21; w++) L[KW_INIT + w] = make_uint2(m.w[2 * w], m.w[2 * w + 1]);
    }
    kw_sync();  // lane 0's init block -> every S lane
    const uint2 v = L[KW_INIT + (i < 21u ? i : 0u)];
    const uint32_t jlo = lo, jhi = hi;
    lo = sw21 ? v.x : 0u;
    hi = sw21 ? v.y : 0u;
    kw_p12(L, k, lo, hi);
    if (jg) {
      lo = jlo;
      hi = jhi;
    }
  };
  // S lanes: block m's word i is stream word q = 21 m + i, half q & 1 of element q >> 1
  auto s_emit = [&](uint4* base, uint32_t len, uint32_t m) {
    if (sw21) {
      const uint32_t q = 21u * m + i, e = q >> 1;
      if (e < len) {
        reinterpret_cast<uint2*>(base + il_idx(blk, len, e, il))[q & 1u] = make_uint2(lo, hi);
        if (q & 1u) gmax = max(gmax, hi & (lo | 0x1Fu));  // ge_screen on the element's (z, w)
      }
    }
  };
  // J lanes: message word w of a block = stream bytes [8 w - 42, 8 w - 34) relative to the block = window
  // words (w, w + 1) shifted by 48 bits; the last absorbed block keeps bytes [0, nb) and takes the padding
  auto j_absorb = [&](bool last, uint32_t nb) {
    if (jw21) {
      const uint2 v0 = L[KW_MSG + i], v1 = L[KW_MSG + i + 1];
      uint32_t wd[2] = {alignbit(v1.x, v0.y, 16), alignbit(v1.y, v1.x, 16)};
      if (last) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const uint32_t d = 2u * i + (uint32_t)h, lb = 4u * d;
          if (lb >= nb)
            wd[h] = 0;
          else if (lb + 4u > nb)
            wd[h] &= (1u << (8u * (nb - lb))) - 1u;
          if (d == (nb >> 2)) wd[h] ^= 1u << (8u * (nb & 3u));
          if (d == 41u) wd[h] ^= 0x80000000u;
        }
      }
      lo ^= wd[0];
      hi ^= wd[1];
    }
  };

  {  // S: XOF(k_meas, DST(1), [1]) -> measurement-share block 0
    uint32_t kmeas[4];
    load16(hs, kmeas);
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 1, kmeas);
    blk_put_byte(m, pos, 1);
    blk_pad(m, pos + 1);
    s_init(m);
  }
  {  // the window's prefix: J's 42-byte header [agg_id || nonce after the XOF prefix] at stream bytes [-42, 0)
    uint32_t nonce[4], kblind[4];
    load16(b.nonces + 16 * r, nonce);
    load16(hs + 32, kblind);
    Block h;
    blk_zero(h);
    int pos = blk_xof_prefix(h, c.dst_id, 7, kblind);
    blk_put_byte(h, pos, 1);  // agg_id
#pragma unroll
    for (int q = 0; q < 4; q++) blk_put_word(h, pos + 1 + 4 * q, nonce[q]);
    if (lane == 0) {
      // window word t covers stream bytes [8 t - 48, 8 t - 40): header bytes 8 t - 6 ..
      L[KW_MSG + 0] = make_uint2(0u, h.w[0] << 16);
#pragma unroll
      for (int t = 1; t < 6; t++)
        L[KW_MSG + t] = make_uint2(alignbit(h.w[2 * t - 1], h.w[2 * t - 2], 16), alignbit(h.w[2 * t], h.w[2 * t - 1], 16));
    }
  }
  s_emit(b.meas, c.meas_len, 0);
  if (sw21) L[KW_MSG + 6 + i] = make_uint2(lo, hi);
  kw_sync();  // the header (lane 0) and S's block -> J's message words
  j_absorb(b_last == 0, ML);  // J's state is zero: absorbing block 0 sets it
  kw_sync();  // J's window reads complete before S overwrites the window's prefix
  if (sw21 && i >= 15u) L[KW_MSG + i - 15u] = make_uint2(lo, hi);
#pragma unroll 1
  for (uint32_t m = 1; m <= b_last; m++) {
    kw_p12(L, k, lo, hi);  // S: squeeze block m; J: absorb block m - 1
    if (m < NM) s_emit(b.meas, c.meas_len, m);
    if (sw21) L[KW_MSG + 6 + i] = make_uint2(lo, hi);
    kw_sync();  // S's block -> J's message words
    j_absorb(m == b_last, ML - 168u * m);
    kw_sync();  // J's window reads complete before S overwrites the window's prefix
    if (sw21 && i >= 15u) L[KW_MSG + i - 15u] = make_uint2(lo, hi);
  }
  kw_p12(L, k, lo, hi);  // J: absorb block b_last
  // J's joint_rand_part = its state words 0, 1 (lanes 32, 33)
  uint32_t own_part[4] = {(uint32_t)__builtin_amdgcn_readlane((int)lo, 32), (uint32_t)__builtin_amdgcn_readlane((int)hi, 32),
                          (uint32_t)__builtin_amdgcn_readlane((int)lo, 33), (uint32_t)__builtin_amdgcn_readlane((int)hi, 33)};
  {  // proof share: XOF(k_proofs, DST(2), [PROOFS=1, agg_id=1])
    uint32_t kproof[4];
    load16(hs + 16, kproof);
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 2, kproof);
    blk_put_byte(m, pos, 1);
    blk_put_byte(m, pos + 1, 1);
    blk_pad(m, pos + 2);
    s_init(m);
  }
  const uint32_t NP = (c.proof_len * 16 + 167) / 168;
  s_emit(b.proof, c.proof_len, 0);
#pragma unroll 1
  for (uint32_t m = 1; m < NP; m++) {
    kw_p12(L, k, lo, hi);
    s_emit(b.proof, c.proof_len, m);
  }
  const bool slow = __ballot(gmax == 0xFFFFFFFFu) != 0;
  if (lane == 0) {
    uint32_t flags = slow ? FLAG_SLOW : 0u;
    uint32_t nonce[4], part_l[4], lead_part[4];
    load16(b.nonces + 16 * r, nonce);
    load16(b.ps + (uint64_t)c.ps_bytes * r, part_l);
    load16(b.lps + (uint64_t)c.lps_bytes * r + c.lps_bytes - 16, lead_part);
    flags = xof_tail(c, b, blk, il, r, true, nonce, part_l, lead_part, own_part, flags, false);
    if (b.force_slow) flags |= FLAG_SLOW;
    b.flags[r] = flags;
  }
}

// The output-share truncation of the small-launch kernel, one thread per (report, output element), the
// report fastest within its 64-report block: out_i = sum_{j < bits} 2^j x_{bits i + j} mod p over the staged
// measurement share (the same word-column sums as emit_meas). Reports the slow kernel redoes get their
// output share rewritten there.
__global__ __launch_bounds__(256) void trunc_kernel(Cfg c, Bufs b, uint32_t nout) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t il = (uint32_t)(t & 63u);
  const uint64_t gi = t >> 6;
  const uint32_t i = (uint32_t)(gi % nout);
  const uint64_t blk = gi / nout;
  const uint64_t r = blk * 64 + il;
  if (r >= b.n) return;
  TruncW tr;
  truncw_zero(tr);
  for (uint32_t j = 0; j < c.bits; j++) {
    const uint4 v = b.meas[il_idx(blk, c.meas_len, i * c.bits + j, il)];
    tr.T[0] += (uint64_t)v.x << j;
    tr.T[1] += (uint64_t)v.y << j;
    tr.T[2] += (uint64_t)v.z << j;
    tr.T[3] += (uint64_t)v.w << j;
  }
  b.outs[il_idx(blk, c.out_len, i, il)] = f_to_u4(truncw_value(tr));
}

// ---------------------------------------------------------------------------- K1, leader role
// leader_initialized (aggregation_job_driver.rs:345): prepare_init with agg_id 0 on the explicit leader
// input share [meas || proofs || k_blind], one report per lane. Only the joint_rand_part absorb runs
// through Keccak; block m+1 of the share (21 8-byte loads per lane) is fetched into the block buffer
// while J permutes block m, so the loads land under the permutation. Elements >= p fail the report
// (decode). One buffer, one sponge: no spills even when a launch holds a third of a wave per SIMD
// (FixedPointBoundedL2VecSum at length 10000), where every scratch access would be exposed.
// INPLACE: the FLP kernels read the explicit share where it lies (Bufs::meas_rs), so K1 stages nothing
// of it (2.56 MB per FixedPoint 16 x 10000 report: no store traffic, no waits on the stores, and the
// staging memory goes to more reports per launch).
template <bool WIDE, bool INPLACE>
__global__ __launch_bounds__(64 * K1_WAVES) void xof_leader_kernel(Cfg c, Bufs b) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t blk = (uint64_t)blockIdx.x * K1_WAVES + (threadIdx.x >> 6);
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint64_t r0 = blk * 64 + lane;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint8_t* ls = b.lis + b.lis_rs * r;
  const uint32_t MB = c.meas_len * 16;
  const uint32_t ML = 42 + MB;
  const uint32_t NM = (MB + 167) / 168;
  const uint32_t b_last = ML / 168;

  uint32_t buf[42];  // block m of the explicit measurement share (words past the share read as 0)
  auto load_block = [&](uint32_t m) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 21; q++) {
      const uint32_t off = 168 * m + 8 * q;
      uint2 v = make_uint2(0, 0);
      if (off < MB) v = *reinterpret_cast<const uint2*>(ls + off);
      buf[2 * q] = v.x;
      buf[2 * q + 1] = v.y;
    }
  };
  // a block wholly inside the share: no per-word guard, so nothing consumes the loaded words before
  // the next iteration and the loads stay in flight under the permutation (a guard's select would
  // make the compiler wait for them before it)
  auto load_block_full = [&](uint32_t m) __attribute__((always_inline)) {
    const uint2* src = reinterpret_cast<const uint2*>(ls + 168 * m);
#pragma unroll
    for (int q = 0; q < 21; q++) {
      const uint2 v = src[q];
      buf[2 * q] = v.x;
      buf[2 * q + 1] = v.y;
    }
  };
  const uint32_t NF = MB / 168;  // blocks 0 .. NF-1 lie wholly inside the share
  uint32_t carry0 = 0, carry1 = 0, unused_screen = 0;
  bool bad = false;
  TruncW tr;
  truncw_zero(tr);
  tr.j = 0;
  tr.i = 0;
  f128 trunc_lo = make128(0, 0);
  uint4* const mp = b.meas + il_idx(blk, c.meas_len, 0, lane);
  uint4* const op = b.outs + il_idx(blk, c.out_len, 0, lane);
  auto emit = [&](uint32_t e, uint4 v) __attribute__((always_inline)) {
    if (e < c.meas_len) bad |= ge_exact(v);
    emit_meas<WIDE, !INPLACE>(c, mp, op, e, v, unused_screen, tr, trunc_lo);
  };
  auto emit_block = [&](uint32_t m) __attribute__((always_inline)) {
    const uint32_t e0 = 21 * (m >> 1);
    if ((m & 1) == 0) {
#pragma unroll
      for (int ci = 0; ci < 10; ci++)
        emit(e0 + ci, make_uint4(buf[4 * ci], buf[4 * ci + 1], buf[4 * ci + 2], buf[4 * ci + 3]));
      carry0 = buf[40];
      carry1 = buf[41];
    } else {
      emit(e0 + 10, make_uint4(carry0, carry1, buf[0], buf[1]));
#pragma unroll
      for (int ci = 0; ci < 10; ci++)
        emit(e0 + 11 + ci, make_uint4(buf[2 + 4 * ci], buf[3 + 4 * ci], buf[4 + 4 * ci], buf[5 + 4 * ci]));
    }
  };
  uint32_t hdr[11];
  {
    uint32_t nonce[4], kblind[4];
    load16(b.nonces + 16 * r, nonce);
    load16(ls + MB + 16 * c.proof_len, kblind);
    Block h;
    blk_zero(h);
    int pos = blk_xof_prefix(h, c.dst_id, 7, kblind);
    blk_put_byte(h, pos, 0);  // agg_id
#pragma unroll
    for (int i = 0; i < 4; i++) blk_put_word(h, pos + 1 + 4 * i, nonce[i]);
#pragma unroll
    for (int w = 0; w < 11; w++) hdr[w] = h.w[w];
  }
  uint32_t J[50], prev[11];
  // J's message words of block m from prev (block m-1) and buf (block m, if present); block 0 starts
  // with the header
  auto message = [&](uint32_t m, bool have, uint32_t* jw) __attribute__((always_inline)) {
    const uint32_t s0 = have ? buf[0] : 0u;
    if (m == 0) {
#pragma unroll
      for (int w = 0; w < 10; w++) jw[w] = hdr[w];
      jw[10] = (hdr[10] & 0xffffu) | (s0 << 16);
    } else {
#pragma unroll
      for (int w = 0; w < 10; w++) jw[w] = alignbit(prev[w + 1], prev[w], 16);
      jw[10] = alignbit(s0, prev[10], 16);
    }
#pragma unroll
    for (int w = 11; w < 42; w++) jw[w] = have ? alignbit(buf[w - 10], buf[w - 11], 16) : 0u;
  };
  load_block(0);
  emit_block(0);
  if (b_last == 0) {
    uint32_t jw[42];
    message(0, true, jw);
    const uint32_t nb = ML;
#pragma unroll
    for (int w = 0; w < 42; w++) {
      const uint32_t lo_b = 4 * w;
      if (lo_b >= nb)
        jw[w] = 0;
      else if (lo_b + 4 > nb)
        jw[w] &= (1u << (8 * (nb - lo_b))) - 1u;
      if ((uint32_t)w == (nb >> 2)) jw[w] ^= 1u << (8 * (nb & 3));
    }
    jw[41] ^= 0x80000000u;
#pragma unroll
    for (int w = 0; w < 42; w++) J[w] = jw[w];
#pragma unroll
    for (int w = 42; w < 50; w++) J[w] = 0;
    keccak_p12(J);
  } else {
    {
      uint32_t jw[42];
      message(0, true, jw);
#pragma unroll
      for (int w = 0; w < 42; w++) J[w] = jw[w];
#pragma unroll
      for (int w = 42; w < 50; w++) J[w] = 0;
#pragma unroll
      for (int w = 0; w < 11; w++) prev[w] = buf[31 + w];
    }
    if (1 < NF)
      load_block_full(1);
    else if (1 < NM)
      load_block(1);
    keccak_p12(J);
    auto step = [&](uint32_t m) __attribute__((always_inline)) {  // block m < b_last <= NM holds measurement bytes
      emit_block(m);
      uint32_t jw[42];
      message(m, true, jw);
#pragma unroll
      for (int w = 0; w < 42; w++) J[w] ^= jw[w];
#pragma unroll
      for (int w = 0; w < 11; w++) prev[w] = buf[31 + w];
    };
    uint32_t m = 1;
#pragma unroll 1
    for (; m < b_last && m + 1 < NF; m++) {  // the next block is wholly inside the share
      step(m);
      load_block_full(m + 1);
      keccak_p12(J);  // (unrolled: slower, see keccak_p12_unrolled)
    }
#pragma unroll 1
    for (; m < b_last; m++) {
      step(m);
      if (m + 1 < NM) load_block(m + 1);
      keccak_p12(J);
    }
    const bool have = b_last < NM;
    if (have) emit_block(b_last);
    uint32_t jw[42];
    message(b_last, have, jw);
    const uint32_t nb = ML - 168 * b_last;
#pragma unroll
    for (int w = 0; w < 42; w++) {
      const uint32_t lo_b = 4 * w;
      if (lo_b >= nb)
        jw[w] = 0;
      else if (lo_b + 4 > nb)
        jw[w] &= (1u << (8 * (nb - lo_b))) - 1u;
      if ((uint32_t)w == (nb >> 2)) jw[w] ^= 1u << (8 * (nb & 3));
    }
    jw[41] ^= 0x80000000u;
#pragma unroll
    for (int w = 0; w < 42; w++) J[w] ^= jw[w];
    keccak_p12(J);
  }
  uint32_t own_part[4] = {J[0], J[1], J[2], J[3]};
  // proof share: explicit, decoded (>= p fails)
  uint4* const pp = b.proof + il_idx(blk, c.proof_len, 0, lane);
  const uint4* src = reinterpret_cast<const uint4*>(ls + MB);
#pragma unroll 1
  for (uint32_t e = 0; e < c.proof_len; e++) {
    const uint4 v = src[e];
    bad |= ge_exact(v);
    pp[(uint64_t)e * IL] = v;
  }
  uint32_t nonce[4], part_h[4];
  load16(b.nonces + 16 * r, nonce);
  // corrected seed = XOF(0, DST(6), own part || helper's part from the public share): the leader's
  // prepare state (written to msgs), and own part goes out in the prep share
  load16(b.ps + (uint64_t)c.ps_bytes * r + 16, part_h);
  uint32_t flags = xof_tail(c, b, blk, lane, r, r0 < b.n, nonce, own_part, own_part, part_h, 0u, false);
  if (flags & FLAG_SLOW)  // a rejected joint/query randomness sample (~2^-120): redo exactly
    flags = xof_tail(c, b, blk, lane, r, r0 < b.n, nonce, own_part, own_part, part_h, flags & ~FLAG_SLOW, true);
  if (bad) flags |= FLAG_INPUT_FAIL;
  if (r0 < b.n) {
    *reinterpret_cast<uint4*>(b.lps_out + (uint64_t)c.lps_bytes * r + c.lps_bytes - 16) =
        make_uint4(own_part[0], own_part[1], own_part[2], own_part[3]);
    b.flags[r0] = flags;
  }
}

// ---------------------------------------------------------------------------- K1': slow XOF path
// General byte-stream implementation with rejection sampling at any position. Runs only
// for reports flagged FLAG_SLOW (a sampled chunk was >= p; ~1e-14 per SumVec report).

struct ByteXof {
  uint32_t s[50];
  uint32_t pos;
};
__device__ uint32_t bx_byte(ByteXof& x) {
  if (x.pos == 168) {
    keccak_p12(x.s);
    x.pos = 0;
  }
  uint32_t v = (x.s[x.pos >> 2] >> (8 * (x.pos & 3))) & 0xffu;
  x.pos++;
  return v;
}
__device__ f128 bx_elem128(ByteXof& x) {
  uint32_t w[4];
  for (int i = 0; i < 4; i++) {
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) v |= bx_byte(x) << (8 * k);
    w[i] = v;
  }
  return w4_to_f(w[0], w[1], w[2], w[3]);
}
__device__ f128 bx_sample128(ByteXof& x) {
  for (;;) {
    f128 v = bx_elem128(x);
    if (!ge_p128(v)) return v;
  }
}
struct ByteAbs {
  uint32_t s[50];
  uint32_t pos;
};
__device__ void ba_byte(ByteAbs& a, uint32_t v) {
  a.s[a.pos >> 2] ^= (v & 0xffu) << (8 * (a.pos & 3));
  a.pos++;
  if (a.pos == 168) {
    keccak_p12(a.s);
    a.pos = 0;
  }
}
__device__ void ba_word(ByteAbs& a, uint32_t v) {
  for (int k = 0; k < 4; k++) ba_byte(a, v >> (8 * k));
}

__global__ __launch_bounds__(64) void xof_slow_kernel(Cfg c, Bufs b) {
  const uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r0 >= b.n) return;
  if (!(b.flags[r0] & FLAG_SLOW)) return;
  const uint64_t r = r0, blk = r0 / 64;
  const uint32_t lane = r0 % 64;
  uint32_t nonce[4], kmeas[4], kproof[4], kblind[4];
  load16(b.nonces + 16 * r, nonce);
  const uint8_t* hs = b.his + (uint64_t)c.his_bytes * r;
  load16(hs, kmeas);
  load16(hs + 16, kproof);
  load16(hs + 32, kblind);
  uint32_t flags = 0;
  ByteXof X;
  ByteAbs A;
  {
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 1, kmeas);
    blk_put_byte(m, pos, 1);
    blk_pad(m, pos + 1);
    sponge_oneblock(X.s, m);
    X.pos = 0;
  }
  for (int w = 0; w < 50; w++) A.s[w] = 0;
  A.pos = 0;
  {
    Block h;
    blk_zero(h);
    int pos = blk_xof_prefix(h, c.dst_id, 7, kblind);
    blk_put_byte(h, pos, 1);
    for (int i = 0; i < 4; i++) blk_put_word(h, pos + 1 + 4 * i, nonce[i]);
    for (int i = 0; i < 42; i++) ba_byte(A, h.w[i >> 2] >> (8 * (i & 3)));
  }
  Trunc tr;
  acc_zero(tr.a);
  tr.j = 0;
  tr.i = 0;
  for (uint32_t e = 0; e < c.meas_len; e++) {
    f128 x = bx_sample128(X);
    st_il(b.meas, blk, c.meas_len, e, lane, x);
    ba_word(A, lo32(x.lo));
    ba_word(A, hi32(x.lo));
    ba_word(A, lo32(x.hi));
    ba_word(A, hi32(x.hi));
    if (!c.out_is_meas && e < c.trunc_len) {
      trunc_add(tr.a, x, tr.j);
      if (++tr.j == c.bits) {
        st_il(b.outs, blk, c.out_len, tr.i, lane, acc_reduce(tr.a));
        acc_zero(tr.a);
        tr.j = 0;
        tr.i++;
      }
    }
  }
  A.s[A.pos >> 2] ^= 1u << (8 * (A.pos & 3));
  A.s[41] ^= 0x80000000u;
  keccak_p12(A.s);
  uint32_t part_h[4] = {A.s[0], A.s[1], A.s[2], A.s[3]};
  {
    Block m;
    blk_zero(m);
    int pos = blk_xof_prefix(m, c.dst_id, 2, kproof);
    blk_put_byte(m, pos, 1);
    blk_put_byte(m, pos + 1, 1);
    blk_pad(m, pos + 2);
    sponge_oneblock(X.s, m);
    X.pos = 0;
  }
  for (uint32_t e = 0; e < c.proof_len; e++) st_il(b.proof, blk, c.proof_len, e, lane, bx_sample128(X));
  uint32_t part_l[4], lead_part[4];
  load16(b.ps + (uint64_t)c.ps_bytes * r, part_l);
  load16(b.lps + (uint64_t)c.lps_bytes * r + c.lps_bytes - 16, lead_part);
  flags = xof_tail(c, b, blk, lane, r, true, nonce, part_l, lead_part, part_h, flags, true);
  b.flags[r0] = flags & ~FLAG_SLOW;
}

// ---------------------------------------------------------------------------- K3: FLP query + decide

__device__ __forceinline__ f128 ld_lead(const Bufs& b, const Cfg& c, uint64_t r, uint32_t idx, bool& dfail) {
  uint4 v = *reinterpret_cast<const uint4*>(b.lps + (uint64_t)c.lps_bytes * r + 16u * idx);
  f128 x = u4_to_f(v);
  dfail |= ge_p128(x);
  return x;
}

// Prio3Sum: gadget PolyEval(x^2 - x), arity 1, `bits` calls; one report per lane.
// LEADER: writes the leader's verifier share [v, W0, G(t)] as its prep share.
template <bool LEADER>
__global__ __launch_bounds__(256) void flp_sum_kernel(Cfg c, Bufs b) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t blk = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint64_t r0 = blk * 64 + lane;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint32_t NC = c.ncoef, C = c.calls;
  const uint4* omega = b.consts + c.c_omega;
  f128 LR = ld_il(b.coef, blk, NC, COEF_L, lane), c0R = ld_il(b.coef, blk, NC, COEF_C0, lane);
  f128 tR = ld_il(b.coef, blk, NC, COEF_T, lane), rR = ld_il(b.coef, blk, NC, COEF_R, lane);
  acc192 ao;
  acc_zero(ao);
  const MeasView mv = meas_view(c, b, blk, lane);
  for (uint32_t k = 1; k <= C; k++) {
    f128 x = u4_to_f(mv[k - 1]);
    uint64_t lo, hi;
    uint32_t top;
    mont128_lazy(x, ld_il(b.coef, blk, NC, COEF_K + k - 1, lane), lo, hi, top);
    acc_add(ao, lo, hi, top);
  }
  f128 s0 = ld_il(b.proof, blk, c.proof_len, 0, lane);
  f128 W0 = mont128(add128(mont128(s0, c0R), acc_reduce(ao)), LR);
  // v = sum_{k=1..C} r^k g(w^k). The spec evaluates the gadget polynomial g (GL = 2P - 1
  // coefficients) at every w^k by Horner: C * GL products and proof-share reads. Since w^P = 1,
  // g(w^k) = sum_{j<P} g'_j w^{kj} with g'_j = g_j + g_{j+P}, so
  //   v = sum_{j<P} g'_j S_j,   S_j = sum_{k=1..C} q_j^k,   q_j = r w^j.
  // w^{P/2} = -1 gives q_{j+P/2} = -q_j, so with E_j / O_j the even / odd-power parts of S_j,
  // S_j = E + O and S_{j+P/2} = E - O. With Q = q^2 and s = sum_{m=1..n} Q^m, n = floor(C/2):
  // E = s, O = q (1 + s - [C even] Q^n); s and Q^n come from the bits of n by doubling
  // (s_2n = s_n + Q^n s_n, Q^2n = (Q^n)^2; s_n+1 = s_n + Q^n+1). ~2 log2(C) products per pair of
  // j (identity checked in Python for C = 1..91), every proof coefficient read once.
  const uint32_t GL = c.gpoly_len, P = c.P, H = c.P / 2, n = C / 2;
  const f128 R1 = make128(R1_128_LO, R1_128_HI);
  f128 v = make128(0, 0);
  const f128 w1 = u4_to_f(omega[1 % P]);
  f128 wj = u4_to_f(omega[0]);  // w^j R
  for (uint32_t j = 0; j < H; j++) {
    f128 ga = ld_il(b.proof, blk, c.proof_len, 1 + j, lane);
    if (j + P < GL) ga = add128(ga, ld_il(b.proof, blk, c.proof_len, 1 + j + P, lane));
    f128 gb = ld_il(b.proof, blk, c.proof_len, 1 + j + H, lane);
    if (j + H + P < GL) gb = add128(gb, ld_il(b.proof, blk, c.proof_len, 1 + j + H + P, lane));
    const f128 q = mont128(rR, wj);  // r w^j, Montgomery form
    f128 sq = make128(0, 0), pq = R1;  // s_n, Q^n
    if (n > 0) {
      const f128 Q = mont128(q, q);
      sq = Q;
      pq = Q;
      const uint32_t top = 31u - (uint32_t)__builtin_clz(n);
      for (int bit = (int)top - 1; bit >= 0; bit--) {
        sq = add128(sq, mont128(pq, sq));
        pq = mont128(pq, pq);
        if ((n >> bit) & 1u) {
          pq = mont128(pq, Q);
          sq = add128(sq, pq);
        }
      }
    }
    const f128 O = mont128(q, add128(R1, (C & 1u) ? sq : sub128(sq, pq)));
    v = add128(v, mont128(ga, add128(sq, O)));
    v = add128(v, mont128(gb, sub128(sq, O)));
    wj = mont128(wj, w1);
  }
  f128 G = make128(0, 0);
  for (uint32_t m = GL; m-- > 0;) G = add128(mont128(G, tR), ld_il(b.proof, blk, c.proof_len, 1 + m, lane));
  if (LEADER) {
    if (r0 < b.n) {
      uint4* o = reinterpret_cast<uint4*>(b.lps_out + (uint64_t)c.lps_bytes * r);
      o[0] = f_to_u4(v);
      o[1] = f_to_u4(W0);
      o[2] = f_to_u4(G);
      b.verdicts[r0] = (b.flags[r] & (FLAG_INIT_FAIL | FLAG_INPUT_FAIL)) ? 1 : 0;
    }
    return;
  }
  bool dfail = false;
  f128 lv = ld_lead(b, c, r, 0, dfail), lw = ld_lead(b, c, r, 1, dfail), lg = ld_lead(b, c, r, 2, dfail);
  const uint32_t flags = b.flags[r];
  uint32_t verdict = 0;
  if (flags & FLAG_INIT_FAIL)
    verdict = 1;
  else if (dfail)
    verdict = 2;
  else {
    f128 V0 = add128(v, lv), V1 = add128(W0, lw), VG = add128(G, lg);
    // (V1^2 - V1) == VG, compared in the R^-1 scaled domain
    f128 lhs = sub128(mont128(V1, V1), mont128(V1, make128(1, 0)));
    if (!is_zero128(V0) || !eq128(lhs, mont128(VG, make128(1, 0))))
      verdict = 3;
    else if (flags & FLAG_NEXT_FAIL)
      verdict = 4;
  }
  if (r0 < b.n) b.verdicts[r0] = (uint8_t)verdict;
}

// The part kernels' common end: the calls kf+1..C (the ragged last call, or every call of a padded
// group) with guarded direct loads, then the wires at t, the leader's verifier share and the gadget
// polynomial's share of v and G(t) for group g of block blk.
template <int PPW, bool HIST, bool LEADER>
__device__ __forceinline__ void psum_group_finish(const Cfg& c, const Bufs& b, uint64_t blk, uint32_t g, uint32_t lane,
                                                  const f128* E, const f128* O, f128 sxr);
template <int PPW, bool HIST, bool LEADER>
__device__ __forceinline__ void psum_part_finish(const Cfg& c, const Bufs& b, uint64_t blk, uint32_t g, uint32_t lane,
                                                 uint32_t kf, wacc26* ae, wacc26* ao, acc192& sx) {
  const uint32_t NG = c.ngroups;
  const uint64_t r0 = blk * 64 + lane;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint32_t NC = c.ncoef, C = c.calls, chunk = c.chunk, M = c.meas_len, A = 2 * chunk;
  const uint32_t j0 = g * PPW;
  const uint4* coefb = b.coef + il_idx(blk, NC, 0, lane);
  const MeasView measb = meas_view(c, b, blk, lane);
#pragma unroll 1
  for (uint32_t k = kf + 1; k <= C; k++) {  // the ragged last call(s), or every call of a padded group
    const limbs26 ck = to_limbs26(u4_to_f(coefb[(COEF_K + 2 * (k - 1)) * IL]));
    const limbs26 dk = to_limbs26(u4_to_f(coefb[(COEF_K + 2 * (k - 1) + 1) * IL]));
    const uint32_t nb = (k - 1) * chunk + j0;
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      if (j0 + i < chunk && nb + i < M) {
        const f128 x = u4_to_f(measb[nb + i]);
        const limbs26 xl = to_limbs26(x);
        wacc_mac(ae[i], xl, dk);
        wacc_mac(ao[i], xl, ck);
        if (HIST) acc_add128(sx, x);
      }
    }
    if (((k - kf) & 511u) == 0) {
#pragma unroll
      for (int i = 0; i < PPW; i++) {
        wacc_normalize(ae[i]);
        wacc_normalize(ao[i]);
      }
    }
  }
  f128 E[PPW], O[PPW];
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    E[i] = wacc_reduce(ae[i]);
    O[i] = wacc_reduce(ao[i]);
  }
  psum_group_finish<PPW, HIST, LEADER>(c, b, blk, g, lane, E, O, HIST ? acc_reduce(sx) : make128(0, 0));
}

// The group finish from the reduced wire sums E_i = (sum_k d_k x_{k,i}) R, O_i = (sum_k c_k x_{k,i}) R of
// its PPW slots: wires at t (plus the leader's verifier share), this group's share of v and G(t), written
// as the four partial sums of the group (Histogram: sxr = its sum of x).
template <int PPW, bool HIST, bool LEADER>
__device__ __forceinline__ void psum_group_finish(const Cfg& c, const Bufs& b, uint64_t blk, uint32_t g, uint32_t lane,
                                                  const f128* E, const f128* O, f128 sxr) {
  const uint32_t NG = c.ngroups;
  const uint64_t r0 = blk * 64 + lane;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint32_t NC = c.ncoef, chunk = c.chunk, A = 2 * chunk;
  const uint32_t j0 = g * PPW;
  const uint4* coefb = b.coef + il_idx(blk, NC, 0, lane);
  // ---- wires at t for this group's slots, plus the leader's verifier share. K1 scaled the constants by
  // L (xof_tail): Lc = L canonical, c0LR = c_0 L R, hsL = L (sum c_k)/2, rpowL_j = L r^(j+1), so
  //   wire_even(t) = L (c_0 se + r^(j+1) sum_k d_k x) = mont(se, c0LR) + mont(E, rpowL_j)
  //   wire_odd(t)  = L (c_0 so + sum_k c_k x - (sum c_k)/2) = mont(so, c0LR) + mont(O, Lc) - hsL
  // (E, O are R-scaled: c_k, d_k are stored in Montgomery form).
  const f128 Lc = u4_to_f(coefb[COEF_L * IL]), c0LR = u4_to_f(coefb[COEF_C0 * IL]);
  const f128 hsL = u4_to_f(coefb[COEF_HALFSUM * IL]);
  bool dfail = false;
  f128 prod = make128(0, 0);
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    const uint32_t j = j0 + i;
    if (j < chunk) {
      f128 se = ld_il(b.proof, blk, c.proof_len, 2 * j, lane);
      f128 so = ld_il(b.proof, blk, c.proof_len, 2 * j + 1, lane);
      const f128 rpowL = u4_to_f(coefb[(c.c_rpow + j) * IL]);
      const f128 We = add128(mont128(se, c0LR), mont128(E[i], rpowL));
      const f128 Wo = sub128(add128(mont128(so, c0LR), mont128(O[i], Lc)), hsL);
      if (LEADER) {  // the leader's verifier share: wire values at t
        if (r0 < b.n) {
          uint4* o = reinterpret_cast<uint4*>(b.lps_out + (uint64_t)c.lps_bytes * r);
          o[1 + 2 * j] = f_to_u4(We);
          o[2 + 2 * j] = f_to_u4(Wo);
        }
      } else {
        f128 Ve = add128(We, ld_lead(b, c, r, 1 + 2 * j, dfail));
        f128 Vo = add128(Wo, ld_lead(b, c, r, 2 + 2 * j, dfail));
        prod = add128(prod, mont128(Ve, Vo));
      }
    }
  }
  // ---- gadget polynomial: v-part = sum_m g_m * S_m and the G(t) part over this group's m-range
  const uint32_t GL = c.gpoly_len;
  const uint32_t per = (GL + NG - 1) / NG;
  const uint32_t m0 = g * per, m1 = min(GL, m0 + per);
  const uint4* Sm = b.consts + c.c_S;
  f128 vpart = make128(0, 0), gpart = make128(0, 0);
  if (m0 < m1) {
    const f128 tR = u4_to_f(coefb[COEF_T * IL]);
    for (uint32_t m = m1; m-- > m0;) {
      f128 gm = ld_il(b.proof, blk, c.proof_len, A + m, lane);
      vpart = add128(vpart, mont128(gm, u4_to_f(Sm[m])));
      gpart = add128(mont128(gpart, tR), gm);
    }
    gpart = mont128(gpart, u4_to_f(coefb[(c.c_tpow + g) * IL]));  // t^m0 R (K1's table)
  }
  uint4* pp = b.part + ((blk * c.ngt + g) * 4) * IL + lane;
  pp[0] = f_to_u4(prod);
  pp[IL] = f_to_u4(vpart);
  pp[2 * IL] = f_to_u4(gpart);
  if (HIST) pp[3 * IL] = f_to_u4(sxr);
  if (dfail && r0 < b.n) atomicOr(&b.flags[r0], FLAG_DFAIL);
}

// Prio3SumVec / Prio3Histogram: gadget ParallelSum(Mul, chunk), arity 2*chunk.
//
// Phase 1 (flp_psum_part_kernel): one wave per (64-report block, slot group). Lanes are
// reports (the interleaved staging makes every load a coalesced 1 KiB). Group g owns the
// chunk slots [g*PPW, (g+1)*PPW) -- 2*PPW lazy wire accumulators per lane, small enough to
// stay in registers at >= 3 waves/SIMD -- and the gadget-polynomial coefficients
// [g*per, (g+1)*per). It writes four partial sums per report: sum_i Ve_i*Vo_i over its
// slots, its share of v (sum_m g_m S_m), its share of G(t), and (Histogram) sum of x.
// Phase 2 (flp_psum_final_kernel): one report per lane; adds the partials, the leader's
// v and G(t), and decides.
// PF: calls whose loads are in flight ahead of the one being multiplied (1: deeper register
// prefetch measured no faster). Used for PPW = 1; PPW = 2 takes the LDS-DMA ring kernel below.
template <int PPW, bool HIST, bool LEADER, int PF = 1>
__global__ __launch_bounds__(64, 4) void flp_psum_part_kernel(Cfg c, Bufs b) {
  const uint32_t NG = c.ngroups;
  // Workgroup ids are dispatched round-robin over the 8 XCDs; map them so that the NG
  // groups of one block run back to back on one XCD and share its L2 (coefficients,
  // leader share).
  const uint32_t bid = blockIdx.x;
  const uint32_t xcd = bid & 7u, q = bid >> 3;
  const uint32_t g = q % NG;
  const uint64_t blk = (uint64_t)(q / NG) * 8 + xcd;
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t NC = c.ncoef, C = c.calls, chunk = c.chunk, M = c.meas_len;
  const uint32_t j0 = g * PPW;

  // wire sums over the calls: ae[i] = sum_k d_k x_{k,i} * R, ao[i] = sum_k c_k x_{k,i} * R
  // (c_k, d_k are stored in Montgomery form), as unreduced 26-bit-limb column sums.
  wacc26 ae[PPW], ao[PPW];
  acc192 sx;
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    wacc_zero(ae[i]);
    wacc_zero(ao[i]);
  }
  acc_zero(sx);
  const uint4* coefb = b.coef + il_idx(blk, NC, 0, lane);
  const MeasView measb = meas_view(c, b, blk, lane);
  // calls whose PPW slots of this group are all real measurement elements run branch-free;
  // the rest (the ragged last chunk, slots beyond chunk) take the guarded tail loop
  uint32_t kf = 0;
  if (j0 + PPW <= chunk && M >= j0 + PPW) kf = min(C, (M - j0 - PPW) / chunk + 1);
  for (uint32_t k0 = 1; k0 <= kf; k0 += 512) {  // <= 5 * 512 limb products (< 2^52) per column
    const uint32_t k1 = min(kf, k0 + 511);
    // software pipeline: the loads of calls k+1 .. k+PF are in flight while call k multiplies
    uint4 cr[PF], dr[PF], xr[PF][PPW];
#pragma unroll
    for (int u = 0; u < PF; u++) {
      const uint32_t k = k0 + u;
      if (k <= k1) {
        cr[u] = coefb[(COEF_K + 2 * (k - 1)) * IL];
        dr[u] = coefb[(COEF_K + 2 * (k - 1) + 1) * IL];
#pragma unroll
        for (int i = 0; i < PPW; i++) xr[u][i] = measb[(uint64_t)((k - 1) * chunk + j0 + i)];
      }
    }
#pragma unroll 1
    for (uint32_t kb = k0; kb <= k1; kb += PF) {
#pragma unroll
      for (int u = 0; u < PF; u++) {
        const uint32_t k = kb + u;
        if (k <= k1) {
          const limbs26 ck = to_limbs26(u4_to_f(cr[u]));
          const limbs26 dk = to_limbs26(u4_to_f(dr[u]));
          f128 x[PPW];
#pragma unroll
          for (int i = 0; i < PPW; i++) x[i] = u4_to_f(xr[u][i]);
          const uint32_t kn = k + PF;
          if (kn <= k1) {
            cr[u] = coefb[(COEF_K + 2 * (kn - 1)) * IL];
            dr[u] = coefb[(COEF_K + 2 * (kn - 1) + 1) * IL];
#pragma unroll
            for (int i = 0; i < PPW; i++) xr[u][i] = measb[(uint64_t)((kn - 1) * chunk + j0 + i)];
          }
#pragma unroll
          for (int i = 0; i < PPW; i++) {
            const limbs26 xl = to_limbs26(x[i]);
            wacc_mac(ae[i], xl, dk);
            wacc_mac(ao[i], xl, ck);
            if (HIST) acc_add128(sx, x[i]);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      wacc_normalize(ae[i]);
      wacc_normalize(ao[i]);
    }
  }
  psum_part_finish<PPW, HIST, LEADER>(c, b, blk, g, lane, kf, ae, ao, sx);
}

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt left unconstrained)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt(0x3f70 | (N & 15) | ((N >> 4) << 14));
}
__device__ __forceinline__ void glds16(const uint4* src, uint4* lds_row) {
  __builtin_amdgcn_global_load_lds((const void*)src, (void*)lds_row, 16, 0, 0);
}

// K3 with an LDS-DMA ring of depth D (4). A workgroup is K3W waves = K3W consecutive slot
// groups of one 64-report block. Per call k, wave 0 streams c_k and wave 1 d_k (one
// global_load_lds_dwordx4 each: 1 KiB, the block's 64 reports) into ring slot (k-1) % D, and every
// wave its own PPW measurement elements; the coefficients are fetched once per K3W groups instead of
// once per group, and D-1 calls stay in flight without holding VGPRs. One s_barrier per call: after it,
// every wave's loads of call k have landed (each waited for its own with vmcnt) and every wave has
// finished reading call k-1's slot, which the next issue overwrites. Every call runs in the ring: an
// element past the share (the ragged last call) or of a padded slot is loaded from a zero constant, so
// it adds nothing, and a padding group's wave only keeps the barriers.
constexpr uint32_t K3W = 4;
// LDS address of a __shared__ object
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)p;
}
// Four 16-byte LDS reads and one wait, in asm: the compiler's LDS-DMA wait tracking cannot tell which
// ring slot a read touches and would otherwise drain every outstanding global_load_lds (vmcnt(0))
// before each read, serialising the ring; the explicit wait_vmcnt + s_barrier order the reads here.
__device__ __forceinline__ void lds_read4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint4& v0, uint4& v1,
                                          uint4& v2, uint4& v3) {
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %5\n\t"
      "ds_read_b128 %2, %6\n\t"
      "ds_read_b128 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3)
      : "memory");
}
// W: waves (slot groups) per workgroup
// RING_ONLY (a measurement variant, instantiated only by tools/kernel_probe.hip): the ring, then a hash of
// the column sums instead of the group finish (results wrong by design), to time the finish by difference.
template <int PPW, bool HIST, bool LEADER, int D, int W = K3W, bool RING_ONLY = false>
__global__ __launch_bounds__(64 * W, 4) void flp_psum_part_glds_kernel(Cfg c, Bufs b) {
  static_assert(PPW == 2, "lds_read4 reads c, d and two measurement rows");
  constexpr int ROWS = 2 + W * PPW;  // c_k, d_k, then x[wave][i]
  __shared__ uint4 ring[D][ROWS][64];
  const uint32_t NG = c.ngroups, NW = (NG + W - 1) / W;
  const uint32_t bid = blockIdx.x, xcd = bid & 7u, q = bid >> 3;
  const uint32_t wg = q % NW;
  const uint64_t blk = (uint64_t)(q / NW) * 8 + xcd;
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;  // uniform over the workgroup
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t g = wg * W + wave;
  const uint32_t C = c.calls, chunk = c.chunk, M = c.meas_len;
  const uint32_t j0 = g * PPW;
  const uint4* coefb = b.coef + il_idx(blk, c.ncoef, 0, lane);
  const MeasView measb = meas_view(c, b, blk, lane);
  const uint4* zero = b.consts + c.c_misc + MISC_ZERO;
  const uint32_t kfw = C;  // every call (see above)
  bool real[PPW];          // slot j0 + i exists (a padding group's wave has none)
#pragma unroll
  for (int i = 0; i < PPW; i++) real[i] = g < NG && j0 + i < chunk;

  wacc26 ae[PPW], ao[PPW];
  acc192 sx;
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    wacc_zero(ae[i]);
    wacc_zero(ao[i]);
  }
  acc_zero(sx);
  // The leader reads its explicit measurement share in place (report-major rows, Bufs::meas_rs): per call
  // the workgroup needs the W*PPW = 8 consecutive elements (128 bytes) of its slots from each of the 64
  // rows. Loaded per lane as the staged layout is (one 16-byte element of 64 rows per instruction) every
  // instruction touches 64 lines for 16 bytes each, and the other waves' parts of those lines come back
  // from HBM once L1/L2 have dropped them (4.0 MB of traffic per FixedPoint 16 x 10000 report against
  // 2.67 MB for the helper's staged stream). Here instruction q (wave q / PPW) reads rows 8q..8q+7 whole:
  // lane l = 8 pp + a takes row 8q + a, part p = pp ^ (q & 1), so eight lanes cover one row's 128 bytes.
  // The part swap on odd q puts rows r and r + 8 in opposite halves of a 256-byte LDS bank window, so the
  // consumers' ds_read_b128 (16 lanes per pass, lane = row) stay conflict-free.
  const bool inpl = LEADER && !HIST && b.meas_rs != 0;
  // loads of call k into ring slot (k - 1) % D
  auto issue = [&](uint32_t k) {
    const uint32_t sl = (k - 1) % D;
    if (wave < 2) glds16(coefb + (uint64_t)(COEF_K + 2 * (k - 1) + wave) * IL, &ring[sl][wave][0]);
    if (inpl) {
      static_assert(W * PPW == 8, "one 128-byte row segment per report per call");
#pragma unroll
      for (int u = 0; u < PPW; u++) {
        const uint32_t q = wave * PPW + u, a = lane & 7u, p = (lane >> 3) ^ (q & 1u);
        const uint32_t slot = wg * (W * PPW) + p, e = (k - 1) * chunk + slot;
        const uint64_t r0 = blk * 64 + 8 * q + a, r = r0 < b.n ? r0 : b.n - 1;
        const uint4* src = slot < chunk && e < M ? reinterpret_cast<const uint4*>(b.meas_src + r * b.meas_rs) + e : zero;
        glds16(src, &ring[sl][2 + q][0]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < PPW; i++) {
        const uint32_t e = (k - 1) * chunk + j0 + i;
        glds16(real[i] && e < M ? &measb[e] : zero, &ring[sl][2 + wave * PPW + i][0]);
      }
    }
  };
  // loads a wave issues per call: 1 (coefficient, waves 0/1) + PPW (measurement)
  auto wait_call = [&](bool tail) {
    if (tail) {
      wait_vmcnt<0>();
    } else if (wave < 2) {
      wait_vmcnt<(D - 2) * (PPW + 1)>();
    } else {
      wait_vmcnt<(D - 2) * PPW>();
    }
  };
  for (uint32_t k = 1; k < D && k <= kfw; k++) issue(k);
  const uint32_t ring_base = lds_addr(&ring[0][0][lane]);
  constexpr uint32_t SLOT_BYTES = ROWS * 64 * 16, ROW_BYTES = 64 * 16;
  // this lane's measurement elements in a ring slot (relative to ring_base)
  uint32_t xoff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    const uint32_t q = lane >> 3, p = wave * PPW + i;
    xoff[i] = inpl ? (2 + q) * ROW_BYTES + ((8 * (p ^ (q & 1u)) + (lane & 7u)) * 16) - lane * 16
                   : (2 + wave * PPW + i) * ROW_BYTES;
  }
#pragma unroll 1
  for (uint32_t k = 1; k <= kfw; k++) {
    wait_call(k + D - 2 > kfw);  // near the end fewer calls are in flight: wait for all
    __builtin_amdgcn_s_barrier();
    if (k + D - 1 <= kfw) issue(k + D - 1);
    if (g < NG) {
      const uint32_t a = ring_base + ((k - 1) % D) * SLOT_BYTES;
      uint4 cv, dv, xv[PPW];
      lds_read4(a, a + ROW_BYTES, a + xoff[0], a + xoff[1], cv, dv, xv[0], xv[1]);
      const limbs26 ck = to_limbs26(u4_to_f(cv));
      const limbs26 dk = to_limbs26(u4_to_f(dv));
#pragma unroll
      for (int i = 0; i < PPW; i++) {
        const f128 x = u4_to_f(xv[i]);
        const limbs26 xl = to_limbs26(x);
        wacc_mac(ae[i], xl, dk);
        wacc_mac(ao[i], xl, ck);
        if (HIST) acc_add128(sx, x);
      }
      if ((k & 511u) == 0) {  // <= 5 * 512 limb products (< 2^52) per column
#pragma unroll
        for (int i = 0; i < PPW; i++) {
          wacc_normalize(ae[i]);
          wacc_normalize(ao[i]);
        }
      }
    }
  }
  if (g >= NG) return;
  if constexpr (RING_ONLY) {
    uint64_t h = 0;
#pragma unroll
    for (int i = 0; i < PPW; i++)
#pragma unroll
      for (int q = 0; q < 9; q++) h ^= ae[i].col[q] ^ ao[i].col[q];
    b.part[((blk * c.ngt + g) * 4) * IL + lane] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), 0, 0);
    return;
  }
  psum_part_finish<PPW, HIST, LEADER>(c, b, blk, g, lane, C, ae, ao, sx);
}

template <bool HIST, bool LEADER>
__global__ __launch_bounds__(256) void flp_psum_final_kernel(Cfg c, Bufs b) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= b.n) return;
  const uint64_t blk = r / 64;
  const uint32_t lane = r % 64, NG = c.ngroups, A = 2 * c.chunk;
  f128 P = make128(0, 0), V = make128(0, 0), G = make128(0, 0), SX = make128(0, 0);
  const uint4* pp = b.part + (blk * c.ngt * 4) * IL + lane;
  for (uint32_t g = 0; g < NG; g++, pp += 4 * IL) {
    P = add128(P, u4_to_f(pp[0]));
    V = add128(V, u4_to_f(pp[IL]));
    G = add128(G, u4_to_f(pp[2 * IL]));
    if (HIST) SX = add128(SX, u4_to_f(pp[3 * IL]));
  }
  f128 vh = V;
  if (HIST) {
    // v = jr1 * range_check + jr1^2 * (sum(x) - 1/2)
    const f128 r2R = ld_il(b.coef, blk, c.ncoef, COEF_R2, lane);
    const f128 half = u4_to_f(b.consts[c.c_misc + 1]);
    f128 sc = sub128(SX, half);
    vh = add128(mont128(V, r2R), mont128(sc, mont128(r2R, r2R)));
  }
  const uint32_t flags = b.flags[r];
  if (LEADER) {  // verifier share [v, wires(t)..., G(t)]; wires were written by the part kernel
    uint4* o = reinterpret_cast<uint4*>(b.lps_out + (uint64_t)c.lps_bytes * r);
    o[0] = f_to_u4(vh);
    o[A + 1] = f_to_u4(G);
    b.verdicts[r] = (flags & (FLAG_INIT_FAIL | FLAG_INPUT_FAIL)) ? 1 : 0;
    return;
  }
  bool df = (flags & FLAG_DFAIL) != 0;
  f128 lv = ld_lead(b, c, r, 0, df), lg = ld_lead(b, c, r, A + 1, df);
  uint32_t verdict = 0;
  if (flags & FLAG_INIT_FAIL)
    verdict = 1;
  else if (df)
    verdict = 2;
  else {
    f128 V0 = add128(vh, lv), VG = add128(G, lg);
    if (!is_zero128(V0) || !eq128(P, mont128(VG, make128(1, 0))))
      verdict = 3;
    else if (flags & FLAG_NEXT_FAIL)
      verdict = 4;
  }
  b.verdicts[r] = (uint8_t)verdict;
}

// Prio3FixedPointBoundedL2VecSum, gadget 1: ParallelSum(PolyEval(p), chunk1) over the decoded entries
// y (= the output share, already truncated by K1), p(y) = 2^(2n-2) - 2^n y + y^2. One wave per
// (64-report block, group of PPW slots). Wire j at t1 is the barycentric sum
//   W_j = L1 (c'_0 s_j + sum_k c'_k y_{(k-1) chunk1 + j} + [short last chunk] c'_last 2^(n-2)),
// the padding value 2^(n-2) being the share of the encoded 0.0 (2^(n-1) / num_shares). The group
// also writes its share of v's gadget-1 part (sum_m g_m S1_m) and of G1(t1), and (helper) the sum of
// p(V_j) over its slots, V_j = own + leader wire, in the R^-1 domain of the decide compare.
template <int PPW, bool LEADER>
__global__ __launch_bounds__(64, 4) void flp_norm_part_kernel(Cfg c, Bufs b) {
  const uint32_t NG = c.ngroups1;
  const uint32_t bid = blockIdx.x;
  const uint32_t xcd = bid & 7u, q = bid >> 3;
  const uint32_t g = q % NG;
  const uint64_t blk = (uint64_t)(q / NG) * 8 + xcd;
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint32_t lane = threadIdx.x;
  const uint64_t r0 = blk * 64 + lane;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint32_t NC = c.ncoef, C = c.calls1, ch = c.chunk1, E = c.out_len, B = c.coef1;
  const uint32_t j0 = g * PPW;
  const uint4* coefb = b.coef + il_idx(blk, NC, 0, lane);
  const uint4* outb = b.outs + il_idx(blk, E, 0, lane);
  wacc26 ao[PPW];
#pragma unroll
  for (int i = 0; i < PPW; i++) wacc_zero(ao[i]);
#pragma unroll 1
  for (uint32_t k = 1; k <= C; k++) {
    const limbs26 ck = to_limbs26(u4_to_f(coefb[(B + G1_K + k - 1) * IL]));
    const uint32_t nb = (k - 1) * ch + j0;
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      if (j0 + i < ch && nb + i < E) wacc_mac(ao[i], to_limbs26(u4_to_f(outb[(uint64_t)(nb + i) * IL])), ck);
    }
    if ((k & 511u) == 0) {
#pragma unroll
      for (int i = 0; i < PPW; i++) wacc_normalize(ao[i]);
    }
  }
  const uint4* misc = b.consts + c.c_misc;
  const f128 LR = u4_to_f(coefb[(B + G1_L) * IL]), c0R = u4_to_f(coefb[(B + G1_C0) * IL]);
  const f128 tR = u4_to_f(coefb[(B + G1_T) * IL]);
  const f128 cl = u4_to_f(coefb[(B + G1_K + C - 1) * IL]);  // c'_calls1 (the possibly short last call)
  const f128 pad = mont128(u4_to_f(misc[6]), cl);          // 2^(n-2) c'_last, canonical
  const f128 twon = u4_to_f(misc[4]), K = u4_to_f(misc[5]);
  const uint32_t A0 = 2 * c.chunk;  // gadget 0's arity: gadget 1's wires follow it in the verifier
  bool dfail = false;
  f128 prod = make128(0, 0);
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    const uint32_t j = j0 + i;
    if (j < ch) {
      const f128 s = ld_il(b.proof, blk, c.proof_len, c.proof1_off + j, lane);
      f128 O = mont128(wacc_reduce(ao[i]), make128(1, 0));  // sum_k c'_k y (canonical)
      if ((C - 1) * ch + j >= E) O = add128(O, pad);
      const f128 W = mont128(add128(mont128(s, c0R), O), LR);
      if (LEADER) {
        if (r0 < b.n) reinterpret_cast<uint4*>(b.lps_out + (uint64_t)c.lps_bytes * r)[A0 + 2 + j] = f_to_u4(W);
      } else {
        const f128 V = add128(W, ld_lead(b, c, r, A0 + 2 + j, dfail));
        // p(V) R^-1 = V^2 R^-1 - 2^n V R^-1 + 2^(2n-2) R^-1
        prod = add128(prod, add128(sub128(mont128(V, V), mont128(V, twon)), K));
      }
    }
  }
  const uint32_t GL = c.gpoly1_len;
  const uint32_t per = (GL + NG - 1) / NG;
  const uint32_t m0 = g * per, m1 = min(GL, m0 + per);
  const uint4* Sm = b.consts + c.c_S1;
  const uint32_t goff = c.proof1_off + ch;
  f128 vpart = make128(0, 0), gpart = make128(0, 0);
  if (m0 < m1) {
    for (uint32_t m = m1; m-- > m0;) {
      f128 gm = ld_il(b.proof, blk, c.proof_len, goff + m, lane);
      vpart = add128(vpart, mont128(gm, u4_to_f(Sm[m])));
      gpart = add128(mont128(gpart, tR), gm);
    }
    gpart = mont128(gpart, mpow(tR, m0));
  }
  uint4* pp = b.part + ((blk * c.ngt + c.ngroups + g) * 4) * IL + lane;
  pp[0] = f_to_u4(prod);
  pp[IL] = f_to_u4(vpart);
  pp[2 * IL] = f_to_u4(gpart);
  if (dfail && r0 < b.n) atomicOr(&b.flags[r0], FLAG_DFAIL);
}

// FixedPoint decide: v = jr1 * range_check + jr1^2 * (computed_norm - claimed_norm) where range_check
// = sum_m g0_m S0_m and computed_norm = sum_m g1_m S1_m (the circuit's gadget outputs, as shares) and
// claimed_norm = sum_b 2^b x[entries*n + b]; then both gadgets' G(wires(t_g)) == gadget_poly_g(t_g).
template <bool LEADER>
__global__ __launch_bounds__(256) void flp_fp_final_kernel(Cfg c, Bufs b) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= b.n) return;
  const uint64_t blk = r / 64;
  const uint32_t lane = r % 64, NG0 = c.ngroups, NG1 = c.ngroups1, A0 = 2 * c.chunk, A1 = c.chunk1;
  f128 P0 = make128(0, 0), V0 = P0, G0 = P0, P1 = P0, V1 = P0, G1 = P0;
  const uint4* pp = b.part + (blk * c.ngt * 4) * IL + lane;
  for (uint32_t g = 0; g < NG0; g++, pp += 4 * IL) {
    P0 = add128(P0, u4_to_f(pp[0]));
    V0 = add128(V0, u4_to_f(pp[IL]));
    G0 = add128(G0, u4_to_f(pp[2 * IL]));
  }
  for (uint32_t g = 0; g < NG1; g++, pp += 4 * IL) {
    P1 = add128(P1, u4_to_f(pp[0]));
    V1 = add128(V1, u4_to_f(pp[IL]));
    G1 = add128(G1, u4_to_f(pp[2 * IL]));
  }
  // claimed squared norm: the trailing norm_bits measurement elements, LE bits
  acc192 cn;
  acc_zero(cn);
  const uint32_t nb0 = c.trunc_len;
  const MeasView mv = meas_view(c, b, blk, lane);
  for (uint32_t i = 0; i < c.norm_bits; i++) trunc_add(cn, u4_to_f(mv[nb0 + i]), i);
  const f128 claimed = acc_reduce(cn);
  const f128 r2R = ld_il(b.coef, blk, c.ncoef, COEF_R2, lane);
  const f128 vh = add128(mont128(V0, r2R), mont128(sub128(V1, claimed), mont128(r2R, r2R)));
  const uint32_t flags = b.flags[r];
  if (LEADER) {
    uint4* o = reinterpret_cast<uint4*>(b.lps_out + (uint64_t)c.lps_bytes * r);
    o[0] = f_to_u4(vh);
    o[A0 + 1] = f_to_u4(G0);
    o[A0 + 2 + A1] = f_to_u4(G1);
    b.verdicts[r] = (flags & (FLAG_INIT_FAIL | FLAG_INPUT_FAIL)) ? 1 : 0;
    return;
  }
  bool df = (flags & FLAG_DFAIL) != 0;
  const f128 lv = ld_lead(b, c, r, 0, df), lg0 = ld_lead(b, c, r, A0 + 1, df), lg1 = ld_lead(b, c, r, A0 + 2 + A1, df);
  uint32_t verdict = 0;
  if (flags & FLAG_INIT_FAIL)
    verdict = 1;
  else if (df)
    verdict = 2;
  else {
    const f128 one = make128(1, 0);
    if (!is_zero128(add128(vh, lv)) || !eq128(P0, mont128(add128(G0, lg0), one)) ||
        !eq128(P1, mont128(add128(G1, lg1), one)))
      verdict = 3;
    else if (flags & FLAG_NEXT_FAIL)
      verdict = 4;
  }
  b.verdicts[r] = (uint8_t)verdict;
}

// ---------------------------------------------------------------------------- leader prepare_next
// leader_continued on PingPongMessage::Finish{prep_msg} (aggregation_job_driver.rs:588-602):
// prio prepare_next fails unless prep_msg equals the corrected joint-rand seed of the state.
// peer (nullable): the helper's verdicts; a report the helper rejected (PrepareStepResult::Reject)
// fails on the leader too (helper_step_failure, aggregation_job_driver.rs:646-660).
__global__ __launch_bounds__(256) void leader_finish_kernel(Cfg c, Bufs b, const uint8_t* prep_msgs,
                                                            const uint8_t* peer) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= b.n) return;
  if (b.verdicts[r] != 0) return;
  if (peer && peer[r] != 0) {
    b.verdicts[r] = 5;  // JX_HELPER_STEP_FAILURE
    return;
  }
  if (c.jr_len == 0) return;
  for (uint32_t o = 0; o < c.seed; o += 16) {
    const uint4 m = *reinterpret_cast<const uint4*>(prep_msgs + c.seed * r + o);
    const uint4 k = *reinterpret_cast<const uint4*>(b.msgs + c.seed * r + o);
    if (m.x != k.x || m.y != k.y || m.z != k.z || m.w != k.w) b.verdicts[r] = 4;
  }
}

// ---------------------------------------------------------------------------- K4: accumulate

// selection + count + checksum. Grid-stride over reports (grid capped at SELECT_WGS
// workgroups): each thread folds its reports' SHA-256(id) and selections in registers, the
// workgroup reduces through LDS, and only one set of atomics per workgroup reaches L2 (one
// set per wave serialised ~15k atomics on the same 40 bytes for 1M Count reports).
__global__ __launch_bounds__(256) void select_kernel(AccArgs a, uint8_t* sel) {
  const uint64_t padded = ((a.n + 63) / 64) * 64;
  uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t cnt = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < padded; r += (uint64_t)gridDim.x * blockDim.x) {
    bool s = false;
    if (r < a.n) s = a.verdicts[r] == 0 && (!a.mask || a.mask[r]) && (!a.seg || a.seg[r] == a.seg_id);
    sel[r] = s;
    if (s) {
      uint32_t id[4], h[8];
      load16(a.nonces + 16 * r, id);
      sha256_16(id, h);
#pragma unroll
      for (int k = 0; k < 8; k++) d[k] ^= h[k];
      cnt++;
    }
  }
  // wave XOR / sum reduce, then across the 4 waves of the workgroup in LDS
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t v = d[k];
    for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
    d[k] = v;
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  __shared__ uint32_t red[4][9];
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) red[w][k] = d[k];
    red[w][8] = cnt;
  }
  __syncthreads();
  if (threadIdx.x < 9) {
    const uint32_t k = threadIdx.x;
    uint32_t v = 0;
    for (uint32_t q = 0; q < blockDim.x / 64; q++) v = k < 8 ? (v ^ red[q][k]) : (v + red[q][k]);
    if (v) {
      if (k < 8)
        atomicXor(&a.checksum[k], v);
      else
        atomicAdd(a.count, (unsigned long long)v);
    }
  }
}

__global__ __launch_bounds__(256) void accumulate_kernel(AccArgs a, const uint8_t* sel) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= a.out_len) return;
  const uint64_t nblk = (a.n + 63) / 64;
  const uint64_t b0 = (uint64_t)blockIdx.y * a.blocks_per_chunk;
  const uint64_t b1 = (b0 + a.blocks_per_chunk < nblk) ? b0 + a.blocks_per_chunk : nblk;
  acc192 acc;
  acc_zero(acc);
  // four blocks' loads in flight per iteration (one dependent load per trip left HBM idle)
  uint64_t bk = b0;
  for (; bk + 4 <= b1; bk += 4) {
    uint4 v[4];
    uint8_t s4[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      s4[u] = sel[(bk + u) * 64 + lane];
      v[u] = a.outs[il_idx(bk + u, a.out_len, i, lane)];
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (s4[u]) acc_add128(acc, u4_to_f(v[u]));
  }
  for (; bk < b1; bk++) {
    if (sel[bk * 64 + lane]) acc_add128(acc, u4_to_f(a.outs[il_idx(bk, a.out_len, i, lane)]));
  }
  // wave reduction of the 192-bit accumulators
  for (int off = 32; off > 0; off >>= 1) {
    uint64_t o0 = ((uint64_t)__shfl_xor((uint32_t)(acc.w0 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w0, off);
    uint64_t o1 = ((uint64_t)__shfl_xor((uint32_t)(acc.w1 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w1, off);
    uint64_t o2 = ((uint64_t)__shfl_xor((uint32_t)(acc.w2 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w2, off);
    uint32_t cc = 0;
    acc.w0 = addc64(acc.w0, o0, cc);
    acc.w1 = addc64(acc.w1, o1, cc);
    acc.w2 = acc.w2 + o2 + cc;
  }
  if (lane == 0) {
    uint64_t* p = a.partials + ((uint64_t)blockIdx.y * a.out_len + i) * 3;
    p[0] = acc.w0;
    p[1] = acc.w1;
    p[2] = acc.w2;
  }
}


// one wave per output element: lanes stride over the report chunks' partial sums, then a
// shuffle reduction (Count / Sum use up to 4096 chunks of a single element)
__global__ __launch_bounds__(256) void reduce_partials_kernel(Cfg c, const uint64_t* partials, uint32_t nchunks,
                                                              uint4* agg) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= c.out_len) return;
  acc192 acc;
  acc_zero(acc);
  for (uint32_t q = lane; q < nchunks; q += 64) {
    const uint64_t* p = partials + ((uint64_t)q * c.out_len + i) * 3;
    uint32_t cc = 0;
    acc.w0 = addc64(acc.w0, p[0], cc);
    acc.w1 = addc64(acc.w1, p[1], cc);
    acc.w2 = acc.w2 + p[2] + cc;
  }
  for (int off = 32; off > 0; off >>= 1) {
    uint64_t o0 = ((uint64_t)__shfl_xor((uint32_t)(acc.w0 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w0, off);
    uint64_t o1 = ((uint64_t)__shfl_xor((uint32_t)(acc.w1 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w1, off);
    uint64_t o2 = ((uint64_t)__shfl_xor((uint32_t)(acc.w2 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w2, off);
    uint32_t cc = 0;
    acc.w0 = addc64(acc.w0, o0, cc);
    acc.w1 = addc64(acc.w1, o1, cc);
    acc.w2 = acc.w2 + o2 + cc;
  }
  if (lane != 0) return;
  acc_add128(acc, u4_to_f(agg[i]));
  if (c.fb == 8) {
    uint64_t v = reduce192_p64(acc.w0, acc.w1, acc.w2);
    agg[i] = make_uint4(lo32(v), hi32(v), 0, 0);
  } else {
    agg[i] = f_to_u4(acc_reduce(acc));
  }
}

// K4 for a small batch (<= ACC_SMALL reports, e.g. one Janus aggregation job): one kernel instead of select +
// accumulate + reduce_partials, nothing staged. Wave w of the grid sums output element w over the selected
// reports and adds it into the aggregation; every thread also folds a grid-stride share of the selected
// reports' SHA-256(id) and count, reduced per workgroup into one set of atomics (as select_kernel).
__device__ __forceinline__ bool acc_selected(const AccArgs& a, uint64_t r) {
  return a.verdicts[r] == 0 && (!a.mask || a.mask[r]) && (!a.seg || a.seg[r] == a.seg_id);
}
__global__ __launch_bounds__(256) void accumulate_small_kernel(Cfg c, AccArgs a, uint4* agg) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i < a.out_len) {
    acc192 acc;
    acc_zero(acc);
    const uint64_t nblk = (a.n + 63) / 64;
    for (uint64_t bk = 0; bk < nblk; bk++) {
      const uint64_t r = bk * 64 + lane;
      if (r < a.n && acc_selected(a, r)) acc_add128(acc, u4_to_f(a.outs[il_idx(bk, a.out_len, i, lane)]));
    }
    for (int off = 32; off > 0; off >>= 1) {
      uint64_t o0 = ((uint64_t)__shfl_xor((uint32_t)(acc.w0 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w0, off);
      uint64_t o1 = ((uint64_t)__shfl_xor((uint32_t)(acc.w1 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w1, off);
      uint64_t o2 = ((uint64_t)__shfl_xor((uint32_t)(acc.w2 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w2, off);
      uint32_t cc = 0;
      acc.w0 = addc64(acc.w0, o0, cc);
      acc.w1 = addc64(acc.w1, o1, cc);
      acc.w2 = acc.w2 + o2 + cc;
    }
    if (lane == 0) {
      acc_add128(acc, u4_to_f(agg[i]));
      if (c.fb == 8) {
        const uint64_t v = reduce192_p64(acc.w0, acc.w1, acc.w2);
        agg[i] = make_uint4(lo32(v), hi32(v), 0, 0);
      } else {
        agg[i] = f_to_u4(acc_reduce(acc));
      }
    }
  }
  uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t cnt = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += (uint64_t)gridDim.x * blockDim.x) {
    if (acc_selected(a, r)) {
      uint32_t id[4], h[8];
      load16(a.nonces + 16 * r, id);
      sha256_16(id, h);
#pragma unroll
      for (int k = 0; k < 8; k++) d[k] ^= h[k];
      cnt++;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t v = d[k];
    for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
    d[k] = v;
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  __shared__ uint32_t red[4][9];
  const uint32_t w = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) red[w][k] = d[k];
    red[w][8] = cnt;
  }
  __syncthreads();
  if (threadIdx.x < 9) {
    const uint32_t k = threadIdx.x;
    uint32_t v = 0;
    for (uint32_t q = 0; q < 4; q++) v = k < 8 ? (v ^ red[q][k]) : (v + red[q][k]);
    if (v) {
      if (k < 8)
        atomicXor(&a.checksum[k], v);
      else
        atomicAdd(a.count, (unsigned long long)v);
    }
  }
}

// K4 for up to ACC_MULTI_MAX small batches into one aggregation (the engine's deferred jx_accumulate calls,
// flushed together: one launch instead of one per aggregation job). Workgroup i < out_len sums output element
// i over every batch's finished reports, its wave w taking batches w, w + 4, ... (each 64-report block read
// as one coalesced 1 KiB row), the four waves' 192-bit sums reduced through LDS and added into the
// aggregation. Each workgroup past out_len folds one batch into the count and the ReportIdChecksum.
__global__ __launch_bounds__(256) void accumulate_multi_kernel(Cfg c, AccMultiArgs a) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (blockIdx.x < c.out_len) {
    const uint32_t i = blockIdx.x;
    acc192 acc;
    acc_zero(acc);
    for (uint32_t k = w; k < a.nb; k += 4) {
      const AccDesc d = a.d[k];
      const uint64_t nblk = (d.n + 63) / 64;
      for (uint64_t bk = 0; bk < nblk; bk++) {
        const uint64_t r = bk * 64 + lane;
        if (r < d.n && d.verdicts[r] == 0) acc_add128(acc, u4_to_f(d.outs[il_idx(bk, c.out_len, i, lane)]));
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      uint64_t o0 = ((uint64_t)__shfl_xor((uint32_t)(acc.w0 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w0, off);
      uint64_t o1 = ((uint64_t)__shfl_xor((uint32_t)(acc.w1 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w1, off);
      uint64_t o2 = ((uint64_t)__shfl_xor((uint32_t)(acc.w2 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w2, off);
      uint32_t cc = 0;
      acc.w0 = addc64(acc.w0, o0, cc);
      acc.w1 = addc64(acc.w1, o1, cc);
      acc.w2 = acc.w2 + o2 + cc;
    }
    __shared__ uint64_t red[4][3];
    if (lane == 0) {
      red[w][0] = acc.w0;
      red[w][1] = acc.w1;
      red[w][2] = acc.w2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int q = 1; q < 4; q++) {
        uint32_t cc = 0;
        acc.w0 = addc64(acc.w0, red[q][0], cc);
        acc.w1 = addc64(acc.w1, red[q][1], cc);
        acc.w2 = acc.w2 + red[q][2] + cc;
      }
      acc_add128(acc, u4_to_f(a.agg[i]));
      if (c.fb == 8) {
        const uint64_t v = reduce192_p64(acc.w0, acc.w1, acc.w2);
        a.agg[i] = make_uint4(lo32(v), hi32(v), 0, 0);
      } else {
        a.agg[i] = f_to_u4(acc_reduce(acc));
      }
    }
    return;
  }
  const AccDesc d = a.d[blockIdx.x - c.out_len];
  uint32_t h8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t cnt = 0;
  for (uint64_t r = threadIdx.x; r < d.n; r += 256) {
    if (d.verdicts[r] == 0) {
      uint32_t id[4], h[8];
      load16(d.nonces + 16 * r, id);
      sha256_16(id, h);
#pragma unroll
      for (int k = 0; k < 8; k++) h8[k] ^= h[k];
      cnt++;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t v = h8[k];
    for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
    h8[k] = v;
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  __shared__ uint32_t redc[4][9];
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) redc[w][k] = h8[k];
    redc[w][8] = cnt;
  }
  __syncthreads();
  if (threadIdx.x < 9) {
    const uint32_t k = threadIdx.x;
    uint32_t v = 0;
    for (uint32_t q = 0; q < 4; q++) v = k < 8 ? (v ^ redc[q][k]) : (v + redc[q][k]);
    if (v) {
      if (k < 8)
        atomicXor(&a.checksum[k], v);
      else
        atomicAdd(a.count, (unsigned long long)v);
    }
  }
}

// ---------------------------------------------------------------------------- K4 segmented
// One pass for any number of batch aggregations: a device counting sort of the selected reports by
// segment (LDS histograms, one global atomic per (workgroup, segment)), work items of <= L sorted
// positions that never straddle a segment, per-item 192-bit partial sums, then one reduction per
// (segment, element). The gathered loads are coalesced whenever a segment's reports are contiguous
// (the usual case: Janus jobs group reports by batch), and cost 64-byte sectors per lane otherwise.
__device__ __forceinline__ bool seg_sel(const SegArgs& a, uint64_t r, uint32_t& d) {
  if (r >= a.n || a.verdicts[r] != 0 || (a.mask && !a.mask[r])) return false;
  d = a.seg[r] - a.s0;
  return d < a.ns;
}

__global__ __launch_bounds__(256) void seg_count_kernel(SegArgs a) {
  __shared__ uint32_t h[SEG_MAX];
  for (uint32_t t = threadIdx.x; t < a.ns; t += blockDim.x) h[t] = 0;
  __syncthreads();
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t d;
    if (seg_sel(a, r, d)) atomicAdd(&h[d], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < a.ns; t += blockDim.x)
    if (h[t]) atomicAdd(&a.cnt[t], h[t]);
}

// one workgroup: segment offsets, scatter cursors and the work-item table
__global__ __launch_bounds__(1024) void seg_plan_kernel(SegArgs a) {
  __shared__ uint32_t items_base;
  if (threadIdx.x == 0) {
    uint32_t pos = 0, w = 0;
    for (uint32_t s = 0; s < a.ns; s++) {
      const uint32_t c = a.cnt[s];
      a.off[s] = pos;
      a.cursor[s] = pos;
      a.ioff[s] = w;
      pos += c;
      w += (c + a.L - 1) / a.L;
    }
    a.ioff[a.ns] = w;
    a.nitems[0] = w;
    a.nitems[1] = pos;  // selected reports = sorted positions in use
    items_base = w;
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < a.ns; s += blockDim.x) {
    const uint32_t c = a.cnt[s], p0 = a.off[s];
    uint32_t w = a.ioff[s];
    for (uint32_t q = 0; q < c; q += a.L, w++) a.items[w] = make_uint4(s, p0 + q, p0 + min(c, q + a.L), 0);
  }
}

__global__ __launch_bounds__(256) void seg_scatter_kernel(SegArgs a) {
  __shared__ uint32_t h[SEG_MAX];
  for (uint32_t t = threadIdx.x; t < a.ns; t += blockDim.x) h[t] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t r_first = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t r = r_first; r < a.n; r += stride) {
    uint32_t d;
    if (seg_sel(a, r, d)) atomicAdd(&h[d], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < a.ns; t += blockDim.x)
    if (h[t]) h[t] = atomicAdd(&a.cursor[t], h[t]);  // this workgroup's range of segment t
  __syncthreads();
  for (uint64_t r = r_first; r < a.n; r += stride) {
    uint32_t d;
    if (seg_sel(a, r, d)) a.perm[atomicAdd(&h[d], 1u)] = (uint32_t)r;
  }
}

__device__ __forceinline__ void acc192_wave_reduce(acc192& acc) {
  for (int off = 32; off > 0; off >>= 1) {
    uint64_t o0 = ((uint64_t)__shfl_xor((uint32_t)(acc.w0 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w0, off);
    uint64_t o1 = ((uint64_t)__shfl_xor((uint32_t)(acc.w1 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w1, off);
    uint64_t o2 = ((uint64_t)__shfl_xor((uint32_t)(acc.w2 >> 32), off) << 32) | __shfl_xor((uint32_t)acc.w2, off);
    uint32_t cc = 0;
    acc.w0 = addc64(acc.w0, o0, cc);
    acc.w1 = addc64(acc.w1, o1, cc);
    acc.w2 = acc.w2 + o2 + cc;
  }
}

// wave per (output element, work item): lanes walk the item's sorted positions
__global__ __launch_bounds__(256) void seg_accumulate_kernel(SegArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t w = blockIdx.y;
  if (i >= a.out_len || w >= *a.nitems) return;
  const uint4 it = a.items[w];
  acc192 acc;
  acc_zero(acc);
  uint32_t p = it.y + lane;
  for (; p + 192 < it.z; p += 256) {  // four gathers in flight
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t r = a.perm[p + 64 * u];
      v[u] = a.outs[il_idx(r >> 6, a.out_len, i, r & 63)];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc_add128(acc, u4_to_f(v[u]));
  }
  for (; p < it.z; p += 64) {
    const uint32_t r = a.perm[p];
    acc_add128(acc, u4_to_f(a.outs[il_idx(r >> 6, a.out_len, i, r & 63)]));
  }
  acc192_wave_reduce(acc);
  if (lane == 0) {
    uint64_t* q = a.partials + ((uint64_t)w * a.out_len + i) * 3;
    q[0] = acc.w0;
    q[1] = acc.w1;
    q[2] = acc.w2;
  }
}

// ReportIdChecksum per segment: thread per sorted position; a wave whose 64 positions share a
// segment (all but the boundary waves) folds them and issues one set of atomics
__global__ __launch_bounds__(256) void seg_checksum_kernel(SegArgs a) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t total = a.nitems[1];
  uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t d = 0xFFFFFFFFu;
  if (p < total) {
    const uint32_t r = a.perm[p];
    uint32_t id[4];
    load16(a.nonces + 16ull * r, id);
    sha256_16(id, h);
    d = a.seg[r] - a.s0;
  }
  const uint32_t d0 = __shfl(d, 0);
  const bool uniform = __all(d == d0);
  if (uniform) {
    if (d0 == 0xFFFFFFFFu) return;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t v = h[k];
      for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
      h[k] = v;
    }
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int k = 0; k < 8; k++) atomicXor(&a.checksums[d0][k], h[k]);
  } else if (d != 0xFFFFFFFFu) {
#pragma unroll
    for (int k = 0; k < 8; k++) atomicXor(&a.checksums[d][k], h[k]);
  }
}

// wave per (output element, segment): sum the segment's work-item partials into its aggregate
__global__ __launch_bounds__(256) void seg_reduce_kernel(SegArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t s = blockIdx.y;
  if (i >= a.out_len || s >= a.ns) return;
  acc192 acc;
  acc_zero(acc);
  for (uint32_t w = a.ioff[s] + lane; w < a.ioff[s + 1]; w += 64) {
    const uint64_t* q = a.partials + ((uint64_t)w * a.out_len + i) * 3;
    uint32_t cc = 0;
    acc.w0 = addc64(acc.w0, q[0], cc);
    acc.w1 = addc64(acc.w1, q[1], cc);
    acc.w2 = acc.w2 + q[2] + cc;
  }
  acc192_wave_reduce(acc);
  if (lane != 0) return;
  uint4* agg = a.aggs[s];
  acc_add128(acc, u4_to_f(agg[i]));
  if (a.fb == 8) {
    const uint64_t v = reduce192_p64(acc.w0, acc.w1, acc.w2);
    agg[i] = make_uint4(lo32(v), hi32(v), 0, 0);
  } else {
    agg[i] = f_to_u4(acc_reduce(acc));
  }
  if (i == 0) *a.counts[s] += a.cnt[s];
}

// multi-GPU combine: sum nparts encoded aggregate shares (LE bytes) mod p
// err: set to 1 if an input element is not canonical (>= p): the host merge rejects such a share
// (Field decode, janus_amd/distributed.py merge_aggregate_shares); the engine reports it on sync.
__global__ void combine_kernel(Cfg c, const uint8_t* parts, uint32_t nparts, uint8_t* out, uint32_t* err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.out_len) return;
  const uint32_t fb = c.fb;
  const uint64_t stride = (uint64_t)c.out_len * fb;
  if (fb == 8) {
    uint64_t s = 0;
    for (uint32_t q = 0; q < nparts; q++) {
      const uint8_t* p = parts + q * stride + (uint64_t)i * 8;
      uint64_t v = 0;
      for (int k = 7; k >= 0; k--) v = (v << 8) | p[k];
      if (v >= P64) {
        atomicOr(err, 1u);
        v -= P64;
      }
      s = add64(s, v);
    }
    for (int k = 0; k < 8; k++) out[(uint64_t)i * 8 + k] = (uint8_t)(s >> (8 * k));
  } else {
    f128 s = make128(0, 0);
    for (uint32_t q = 0; q < nparts; q++) {
      const uint8_t* p = parts + q * stride + (uint64_t)i * 16;
      uint64_t lo = 0, hi = 0;
      for (int k = 7; k >= 0; k--) lo = (lo << 8) | p[k];
      for (int k = 15; k >= 8; k--) hi = (hi << 8) | p[k];
      f128 v = make128(lo, hi);
      if (ge_p128(v)) {
        atomicOr(err, 1u);
        v = sub128(v, make128(P128_LO, P128_HI));
      }
      s = add128(s, v);
    }
    for (int k = 0; k < 8; k++) out[(uint64_t)i * 16 + k] = (uint8_t)(s.lo >> (8 * k));
    for (int k = 0; k < 8; k++) out[(uint64_t)i * 16 + 8 + k] = (uint8_t)(s.hi >> (8 * k));
  }
}

// shard record = encoded aggregate share || count (u64 LE) || checksum (32 B), see
// janus_amd/distributed.py. Thread i < out_len writes element i; thread out_len the tail.
// blockIdx.y = record: ns records from contiguous segment state (agg [ns][out_len], count [ns],
// checksum [ns][8]) to ns back-to-back records
__global__ void record_export_kernel(Cfg c, const uint4* agg, const unsigned long long* count,
                                     const uint32_t* checksum, uint8_t* dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t fb = c.fb, y = blockIdx.y;
  agg += (uint64_t)y * c.out_len;
  count += y;
  checksum += 8 * y;
  dst += (uint64_t)y * (c.out_len * fb + 40u);
  if (i < c.out_len) {
    uint4 v = agg[i];
    for (uint32_t k = 0; k < fb; k++) {
      uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
      dst[(uint64_t)i * fb + k] = (uint8_t)(w >> (8 * (k & 3)));
    }
  } else if (i == c.out_len) {
    uint8_t* t = dst + (uint64_t)c.out_len * fb;
    const unsigned long long n = *count;
    for (int k = 0; k < 8; k++) t[k] = (uint8_t)(n >> (8 * k));
    for (int k = 0; k < 32; k++) t[8 + k] = (uint8_t)(checksum[k >> 2] >> (8 * (k & 3)));
  }
}

// merge nparts shard records (compute_aggregate_share, aggregate_share.rs:87-95):
// mod-p sum of the aggregate shares, sum of the counts, XOR of the checksums.
__global__ void record_combine_kernel(Cfg c, const uint8_t* parts, uint32_t nparts, uint8_t* out, uint32_t* err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t fb = c.fb;
  const uint64_t stride = (uint64_t)c.out_len * fb + 40;
  if (i < c.out_len) {
    if (fb == 8) {
      uint64_t s = 0;
      for (uint32_t q = 0; q < nparts; q++) {
        const uint8_t* p = parts + q * stride + (uint64_t)i * 8;
        uint64_t v = 0;
        for (int k = 7; k >= 0; k--) v = (v << 8) | p[k];
        if (v >= P64) {
          atomicOr(err, 1u);
          v -= P64;
        }
        s = add64(s, v);
      }
      for (int k = 0; k < 8; k++) out[(uint64_t)i * 8 + k] = (uint8_t)(s >> (8 * k));
    } else {
      f128 s = make128(0, 0);
      for (uint32_t q = 0; q < nparts; q++) {
        const uint8_t* p = parts + q * stride + (uint64_t)i * 16;
        uint64_t lo = 0, hi = 0;
        for (int k = 7; k >= 0; k--) lo = (lo << 8) | p[k];
        for (int k = 15; k >= 8; k--) hi = (hi << 8) | p[k];
        f128 v = make128(lo, hi);
        if (ge_p128(v)) {
          atomicOr(err, 1u);
          v = sub128(v, make128(P128_LO, P128_HI));
        }
        s = add128(s, v);
      }
      for (int k = 0; k < 8; k++) out[(uint64_t)i * 16 + k] = (uint8_t)(s.lo >> (8 * k));
      for (int k = 0; k < 8; k++) out[(uint64_t)i * 16 + 8 + k] = (uint8_t)(s.hi >> (8 * k));
    }
  } else if (i == c.out_len) {
    const uint64_t tail = (uint64_t)c.out_len * fb;
    uint64_t n = 0;
    uint8_t cs[32];
    for (int k = 0; k < 32; k++) cs[k] = 0;
    for (uint32_t q = 0; q < nparts; q++) {
      const uint8_t* p = parts + q * stride + tail;
      uint64_t v = 0;
      for (int k = 7; k >= 0; k--) v = (v << 8) | p[k];
      n += v;
      for (int k = 0; k < 32; k++) cs[k] ^= p[8 + k];
    }
    for (int k = 0; k < 8; k++) out[tail + k] = (uint8_t)(n >> (8 * k));
    for (int k = 0; k < 32; k++) out[tail + 8 + k] = cs[k];
  }
}

// interleaved output shares -> [r][i] LE bytes
__global__ void transpose_out_kernel(Cfg c, const uint4* outs, uint64_t n, uint8_t* dst) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t r = t / c.out_len;
  const uint32_t i = t % c.out_len;
  if (r >= n) return;
  uint4 v = outs[il_idx(r / 64, c.out_len, i, r % 64)];
  if (c.fb == 8) {
    *reinterpret_cast<uint2*>(dst + t * 8) = make_uint2(v.x, v.y);
  } else {
    *reinterpret_cast<uint4*>(dst + t * 16) = v;
  }
}

// Coalesced launches (jx_coalesce.cpp): copy job j's slice [first, first + n) of the launch's staging into
// the job's own resident batch, so every job keeps an independent batch (interleaved output shares
// re-based to lane 0, verdicts, prep messages / leader seeds, report ids). blockIdx.y = job; the threads of
// a job stride over its destination elements (coalesced writes, reads shifted by first % 64).
__global__ __launch_bounds__(256) void scatter_jobs_kernel(Cfg c, const JobSlice* jobs, const uint4* outs,
                                                           const uint8_t* verdicts, const uint8_t* msgs,
                                                           const uint8_t* nonces) {
  const JobSlice j = jobs[blockIdx.y];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nblk = (j.n + 63) / 64;
  const uint64_t total = nblk * c.out_len * 64;
  for (uint64_t t = t0; t < total; t += stride) {
    const uint64_t blk = t / ((uint64_t)c.out_len * 64);
    const uint32_t rem = (uint32_t)(t % ((uint64_t)c.out_len * 64));
    const uint32_t e = rem / 64, l = rem % 64;
    const uint64_t i = blk * 64 + l;
    if (i >= j.n) continue;
    const uint64_t r = j.first + i;
    j.outs[t] = outs[il_idx(r / 64, c.out_len, e, r % 64)];
  }
  const uint32_t mb = c.seed;  // prep message / seed bytes: 16 or 32
  for (uint64_t i = t0; i < j.n; i += stride) {
    const uint64_t r = j.first + i;
    j.verdicts[i] = verdicts[r];
    const uint4* sm = reinterpret_cast<const uint4*>(msgs + r * mb);
    uint4* dm = reinterpret_cast<uint4*>(j.msgs + i * mb);
    dm[0] = sm[0];
    if (mb == 32) dm[1] = sm[1];
    reinterpret_cast<uint4*>(j.nonces)[i] = reinterpret_cast<const uint4*>(nonces)[r];
  }
}

__global__ void agg_encode_kernel(Cfg c, const uint4* agg, uint8_t* dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.out_len) return;
  uint4 v = agg[i];
  if (c.fb == 8)
    *reinterpret_cast<uint2*>(dst + (uint64_t)i * 8) = make_uint2(v.x, v.y);
  else
    *reinterpret_cast<uint4*>(dst + (uint64_t)i * 16) = v;
}

// ---------------------------------------------------------------------------- launchers

static inline uint32_t nblk_of(uint64_t n) { return (uint32_t)((n + 63) / 64); }

hipError_t launch_count(const Cfg& c, const Bufs& b, hipStream_t s) {
  uint32_t nb = nblk_of(b.n);
  if (b.leader)
    hipLaunchKernelGGL(count_kernel<true>, dim3((nb * 64 + 255) / 256), dim3(256), 0, s, c, b);
  else
    hipLaunchKernelGGL(count_kernel<false>, dim3((nb * 64 + 255) / 256), dim3(256), 0, s, c, b);
  return hipGetLastError();
}
hipError_t launch_xof(const Cfg& c, const Bufs& b, hipStream_t s) {
  uint32_t nb = nblk_of(b.n);
  const dim3 grid((nb + K1_WAVES - 1) / K1_WAVES), block(64 * K1_WAVES);
  const bool wide = c.bits > 32 && (c.algo == ALGO_SUM || c.algo == ALGO_SUMVEC);
  if (b.leader && wide && b.meas_rs)
    hipLaunchKernelGGL((xof_leader_kernel<true, true>), grid, block, 0, s, c, b);
  else if (b.leader && wide)
    hipLaunchKernelGGL((xof_leader_kernel<true, false>), grid, block, 0, s, c, b);
  else if (b.leader && b.meas_rs)
    hipLaunchKernelGGL((xof_leader_kernel<false, true>), grid, block, 0, s, c, b);
  else if (b.leader)
    hipLaunchKernelGGL((xof_leader_kernel<false, false>), grid, block, 0, s, c, b);
  else if (b.k1_split == 7 && !wide) {  // a word per lane: one report per wave, then the truncation
    hipLaunchKernelGGL(xof_words_kernel, dim3((uint32_t)((b.n + KW_WAVES - 1) / KW_WAVES)), dim3(64 * KW_WAVES), 0, s, c, b);
    const uint32_t nout = c.out_is_meas ? 0u : (c.trunc_len < c.meas_len ? c.trunc_len : c.meas_len) / c.bits;
    if (nout) {
      const uint64_t threads = (uint64_t)nblk_of(b.n) * 64 * nout;
      hipLaunchKernelGGL(trunc_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, c, b, nout);
    }
  } else if (b.k1_split == 8 && !wide)  // lane pairs, unrolled rounds (<= one pair-wave per SIMD)
    hipLaunchKernelGGL(xof_pairs_kernel<true>, dim3((4 * nb + K1_WAVES - 1) / K1_WAVES), block, b.k1_pairs_lds, s, c, b);
  else if (b.k1_split == 6 && !wide)  // lane pairs: 16 reports per wave
    hipLaunchKernelGGL(xof_pairs_kernel<false>, dim3((4 * nb + K1_WAVES - 1) / K1_WAVES), block, b.k1_pairs_lds, s, c,
                       b);
  else if (b.k1_split == 3) {  // lane-split: 32 reports per wave
    const dim3 g2((2 * nb + K1_WAVES - 1) / K1_WAVES);
    if (wide)
      hipLaunchKernelGGL((xof_lanes_kernel<true>), g2, block, b.k1_lds, s, c, b);
    else
      hipLaunchKernelGGL((xof_lanes_kernel<false>), g2, block, b.k1_lds, s, c, b);
  } else if (wide)
    hipLaunchKernelGGL((xof_kernel<true>), grid, block, 0, s, c, b);
  else
    hipLaunchKernelGGL((xof_kernel<false>), grid, block, 0, s, c, b);
  return hipGetLastError();
}
Bufs bufs_tail(const Cfg& c, const Bufs& b, uint64_t S) {
  Bufs t = b;
  const uint64_t blk = S / 64;
  t.n = b.n - S;
  t.nonces += S * 16;
  t.ps += S * c.ps_bytes;
  t.his += S * c.his_bytes;
  t.lps += S * c.lps_bytes;
  t.meas += blk * c.meas_len * IL;
  t.proof += blk * c.proof_len * IL;
  t.outs += blk * c.out_len * IL;
  t.coef += blk * c.ncoef * IL;
  t.flags += S;
  t.verdicts += S;
  t.msgs += S * 16;
  // per-report rows that a coalesced launch carries: the verify keys (16 B, or the 64-B HMAC pads of the
  // multiproof instance) and, for a leader launch, its explicit input shares and outbound prep shares
  if (t.vkeys) t.vkeys += S * (c.algo == ALGO_SUMVEC_F64_MULTIPROOF ? 64u : 16u);
  if (t.lis) t.lis += S * b.lis_rs;
  if (t.meas_src) t.meas_src += S * b.meas_rs;
  if (t.lps_out) t.lps_out += S * c.lps_bytes;
  return t;
}

// Dynamic LDS that caps the lane-split kernel at `wgs_per_cu` workgroups per CU (0: no cap).
uint32_t lanes_lds_bytes(uint32_t wgs_per_cu) {
  if (wgs_per_cu == 0) return 0;
  constexpr uint32_t LDS_PER_CU = 160u << 10;
  return (LDS_PER_CU / (wgs_per_cu + 1) + 1024u) / 1024u * 1024u;
}

// Reports that occupy every K1 wave slot of the device exactly once: CUs x resident
// workgroups per CU (from the kernel's register/LDS footprint) x 64 reports per wave. K1 waves
// all run the same length, so a launch runs in ceil(reports / this) equal "rounds"; the
// engine sizes its launches in whole rounds so only the last launch has a partial one.
uint64_t k1_round_reports(const Cfg& c, int device, uint32_t k1_split) {
  if (c.algo == ALGO_SUMVEC_F64_MULTIPROOF) return mp_k1_round_reports(device);
  int cus = 0, wgs = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) return 0;
  const uint32_t threads = c.algo == ALGO_COUNT ? 256u : 64u * K1_WAVES;
  hipError_t st;
  uint32_t per_wg = threads;  // reports per workgroup
  if (c.algo == ALGO_COUNT) {
    st = hipOccupancyMaxActiveBlocksPerMultiprocessor(&wgs, count_kernel<false>, threads, 0);
  } else if (k1_split == 3) {
    st = hipOccupancyMaxActiveBlocksPerMultiprocessor(&wgs, xof_lanes_kernel<false>, threads, lanes_lds_bytes(2));
    per_wg = threads / 2;
  } else if (k1_split == 6) {
    st = hipOccupancyMaxActiveBlocksPerMultiprocessor(&wgs, xof_pairs_kernel<false>, threads, 0);
    per_wg = threads / 4;
  } else {
    st = hipOccupancyMaxActiveBlocksPerMultiprocessor(&wgs, xof_kernel<false>, threads, 0);
  }
  if (st != hipSuccess || wgs <= 0) return 0;
  return (uint64_t)cus * (uint64_t)wgs * per_wg;
}
hipError_t launch_leader_finish(const Cfg& c, const Bufs& b, const uint8_t* prep_msgs, const uint8_t* peer,
                                hipStream_t s) {
  hipLaunchKernelGGL(leader_finish_kernel, dim3((uint32_t)((b.n + 255) / 256)), dim3(256), 0, s, c, b, prep_msgs,
                     peer);
  return hipGetLastError();
}
hipError_t launch_xof_slow(const Cfg& c, const Bufs& b, hipStream_t s) {
  hipLaunchKernelGGL(xof_slow_kernel, dim3((uint32_t)((b.n + 63) / 64)), dim3(64), 0, s, c, b);
  return hipGetLastError();
}

// Slots per FLP group. Each slot holds two 9-column wide accumulators (36 VGPRs); PPW = 2
// (152 VGPRs, 3 waves/SIMD) measured fastest on MI355X for SumVec(8x1000/88): K3 11.8 ms vs
// 13.6 (PPW 1) and 12.5 (PPW 4, spills) per 312,500 reports. PPW = 1 only when it wastes
// fewer padded slot-lanes (chunk_length 1). (4 and 8 slots per wave spill, 0.3-4 KB/lane: removed.)
int psum_ppw(uint32_t chunk) {
  const int cands[] = {2, 1};
  int best = 2, best_cost = 1 << 30;
  for (int p : cands) {
    int ng = (int)((chunk + p - 1) / p);
    int cost = ng * p + 3 * ng;
    if (cost < best_cost) {
      best = p;
      best_cost = cost;
    }
  }
  return best;
}

// K3 phase 1: the depth-4 LDS-DMA ring (K3W slot groups per workgroup) for PPW = 2; the per-wave
// register-prefetch kernel for PPW = 1 (chunk_length 1). Measured and removed:
// 2 / 3 calls of register prefetch, 3-waves/SIMD builds, a depth-3 ring, 8 groups per workgroup.
template <int PPW, bool HIST, bool LEADER>
static void launch_psum_part(const Cfg& c, const Bufs& b, hipStream_t s, uint32_t grid) {
  if constexpr (PPW == 2) {
    const uint32_t g2 = grid / c.ngroups * ((c.ngroups + K3W - 1) / K3W);
    hipLaunchKernelGGL((flp_psum_part_glds_kernel<PPW, HIST, LEADER, 4>), dim3(g2), dim3(64 * K3W), 0, s, c, b);
  } else {
    hipLaunchKernelGGL((flp_psum_part_kernel<PPW, HIST, LEADER>), dim3(grid), dim3(64), 0, s, c, b);
  }
}
template <int PPW, bool HIST, bool LEADER>
static void launch_psum_r(const Cfg& c, const Bufs& b, hipStream_t s) {
  const uint32_t nb = nblk_of(b.n);
  launch_psum_part<PPW, HIST, LEADER>(c, b, s, ((nb + 7) / 8) * 8 * c.ngroups);
  hipLaunchKernelGGL((flp_psum_final_kernel<HIST, LEADER>), dim3((uint32_t)((b.n + 255) / 256)), dim3(256), 0, s,
                     c, b);
}
template <int PPW>
static hipError_t launch_psum_t(const Cfg& c, const Bufs& b, hipStream_t s) {
  const bool hist = c.algo == ALGO_HISTOGRAM;
  if (hist && b.leader)
    launch_psum_r<PPW, true, true>(c, b, s);
  else if (hist)
    launch_psum_r<PPW, true, false>(c, b, s);
  else if (b.leader)
    launch_psum_r<PPW, false, true>(c, b, s);
  else
    launch_psum_r<PPW, false, false>(c, b, s);
  return hipGetLastError();
}

template <int PPW, bool LEADER>
static void launch_fp_r(const Cfg& c, const Bufs& b, hipStream_t s) {
  const uint32_t nb = nblk_of(b.n);
  launch_psum_part<PPW, false, LEADER>(c, b, s, ((nb + 7) / 8) * 8 * c.ngroups);
  hipLaunchKernelGGL((flp_norm_part_kernel<2, LEADER>), dim3(((nb + 7) / 8) * 8 * c.ngroups1), dim3(64), 0, s, c,
                     b);
  hipLaunchKernelGGL((flp_fp_final_kernel<LEADER>), dim3((uint32_t)((b.n + 255) / 256)), dim3(256), 0, s, c, b);
}

hipError_t launch_flp(const Cfg& c, const Bufs& b, hipStream_t s) {
  if (c.algo == ALGO_FIXEDPOINT_L2) {
    if (c.ppw == 2) {
      if (b.leader)
        launch_fp_r<2, true>(c, b, s);
      else
        launch_fp_r<2, false>(c, b, s);
    } else if (c.ppw == 1) {
      if (b.leader)
        launch_fp_r<1, true>(c, b, s);
      else
        launch_fp_r<1, false>(c, b, s);
    } else {
      return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (c.algo == ALGO_SUM) {
    uint32_t nb = nblk_of(b.n);
    if (b.leader)
      hipLaunchKernelGGL(flp_sum_kernel<true>, dim3((nb + 3) / 4), dim3(256), 0, s, c, b);
    else
      hipLaunchKernelGGL(flp_sum_kernel<false>, dim3((nb + 3) / 4), dim3(256), 0, s, c, b);
    return hipGetLastError();
  }
  switch (c.ppw) {
    case 2:
      return launch_psum_t<2>(c, b, s);
    case 1:
      return launch_psum_t<1>(c, b, s);
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_accumulate(const Cfg& c, const AccArgs& a, uint4* agg, hipStream_t s) {
  // sel lives at the tail of the partials allocation (see engine)
  uint8_t* sel = reinterpret_cast<uint8_t*>(a.partials + (size_t)a.nchunks * c.out_len * 3);
  uint64_t nthreads = ((a.n + 63) / 64) * 64;
  uint64_t swg = (nthreads + 255) / 256;
  if (swg > SELECT_WGS) swg = SELECT_WGS;
  hipLaunchKernelGGL(select_kernel, dim3((uint32_t)swg), dim3(256), 0, s, a, sel);
  hipLaunchKernelGGL(accumulate_kernel, dim3((c.out_len + 3) / 4, a.nchunks), dim3(256), 0, s, a,
                     (const uint8_t*)sel);
  hipLaunchKernelGGL(reduce_partials_kernel, dim3((c.out_len + 3) / 4), dim3(256), 0, s, c,
                     (const uint64_t*)a.partials, a.nchunks, agg);
  return hipGetLastError();
}

hipError_t launch_accumulate_small(const Cfg& c, const AccArgs& a, uint4* agg, hipStream_t s) {
  hipLaunchKernelGGL(accumulate_small_kernel, dim3((c.out_len + 3) / 4), dim3(256), 0, s, c, a, agg);
  return hipGetLastError();
}

__global__ __launch_bounds__(64) void host_signal_kernel(uint32_t* flag, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag + threadIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
hipError_t launch_host_signal(uint32_t* flag, uint32_t seq, hipStream_t s) {
  hipLaunchKernelGGL(host_signal_kernel, dim3(1), dim3(64), 0, s, flag, seq);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void copy_regions_kernel(CopyArgs a) {
  const CopyRegion g = a.r[blockIdx.y];
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = ((g.width | g.dst_stride | g.src_stride | (uint64_t)(uintptr_t)g.dst | (uint64_t)(uintptr_t)g.src) & 15) == 0;
  if (vec) {
    const uint64_t cpr = g.width / 16, total = cpr * g.rows;
    for (uint64_t t = t0; t < total; t += step) {
      const uint64_t row = t / cpr, ch = t - row * cpr;
      *reinterpret_cast<uint4*>(g.dst + row * g.dst_stride + 16 * ch) =
          *reinterpret_cast<const uint4*>(g.src + row * g.src_stride + 16 * ch);
    }
  } else if (g.rows == 1 && (((uint64_t)(uintptr_t)g.dst | (uint64_t)(uintptr_t)g.src) & 15) == 0) {
    // one flat run of a length that is not a multiple of 16 (a launch's verdicts, open statuses): 16-byte vectors
    // and a byte tail, not one PCIe write per byte
    const uint64_t nv = g.width / 16;
    for (uint64_t t = t0; t < nv; t += step)
      reinterpret_cast<uint4*>(g.dst)[t] = reinterpret_cast<const uint4*>(g.src)[t];
    if (t0 < g.width - 16 * nv) g.dst[16 * nv + t0] = g.src[16 * nv + t0];
  } else {
    const uint64_t total = g.width * g.rows;
    for (uint64_t t = t0; t < total; t += step) {
      const uint64_t row = t / g.width, bt = t - row * g.width;
      g.dst[row * g.dst_stride + bt] = g.src[row * g.src_stride + bt];
    }
  }
}
hipError_t launch_copy_regions(const CopyArgs& a, hipStream_t s) {
  if (a.nr == 0) return hipSuccess;
  if (a.nr > COPY_MAX_REGIONS) return hipErrorInvalidValue;
  uint64_t most = 0;
  for (uint32_t k = 0; k < a.nr; k++) {
    const CopyRegion& g = a.r[k];
    const bool vec = ((g.width | g.dst_stride | g.src_stride | (uint64_t)(uintptr_t)g.dst | (uint64_t)(uintptr_t)g.src) & 15) == 0;
    const bool flat16 = g.rows == 1 && (((uint64_t)(uintptr_t)g.dst | (uint64_t)(uintptr_t)g.src) & 15) == 0;
    const uint64_t items = vec ? g.width / 16 * g.rows : flat16 ? g.width / 16 + 16 : g.width * g.rows;
    if (items > most) most = items;
  }
  // PCIe-bound: a few hundred waves keep enough reads in flight, and a big launch's K1 keeps the rest of the
  // SIMDs (JX_COPY_WGS overrides the cap for measurement)
  static const uint64_t cap = [] {
    const char* e = getenv("JX_COPY_WGS");
    const long v = e ? atol(e) : 0;
    return v >= 1 && v <= 4096 ? (uint64_t)v : (uint64_t)64;
  }();
  uint64_t gx = (most + 255) / 256;
  if (gx > cap) gx = cap;
  if (gx == 0) gx = 1;
  hipLaunchKernelGGL(copy_regions_kernel, dim3((uint32_t)gx, a.nr), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_accumulate_multi(const Cfg& c, const AccMultiArgs& a, hipStream_t s) {
  if (a.nb == 0) return hipSuccess;
  if (a.nb > ACC_MULTI_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(accumulate_multi_kernel, dim3(c.out_len + a.nb), dim3(256), 0, s, c, a);
  return hipGetLastError();
}

// grid: workgroups of the count/scatter passes (the same for both: each workgroup re-walks its reports)
hipError_t launch_accumulate_segmented(const Cfg& c, const SegArgs& a, uint32_t grid, hipStream_t s) {
  (void)c;
  hipLaunchKernelGGL(seg_count_kernel, dim3(grid), dim3(256), 0, s, a);
  hipLaunchKernelGGL(seg_plan_kernel, dim3(1), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(seg_scatter_kernel, dim3(grid), dim3(256), 0, s, a);
  hipLaunchKernelGGL(seg_accumulate_kernel, dim3((a.out_len + 3) / 4, a.wmax), dim3(256), 0, s, a);
  // one thread per possible sorted position (n bounds the selected count); the rest return at once
  hipLaunchKernelGGL(seg_checksum_kernel, dim3((uint32_t)((a.n + 255) / 256)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(seg_reduce_kernel, dim3((a.out_len + 3) / 4, a.ns), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_combine(const Cfg& c, const uint8_t* parts, uint32_t nparts, uint8_t* out, uint32_t* err,
                          hipStream_t s) {
  hipLaunchKernelGGL(combine_kernel, dim3((c.out_len + 255) / 256), dim3(256), 0, s, c, parts, nparts, out, err);
  return hipGetLastError();
}
hipError_t launch_record_export(const Cfg& c, const uint4* agg, const unsigned long long* count,
                                const uint32_t* checksum, uint8_t* dst, hipStream_t s, uint32_t ns) {
  hipLaunchKernelGGL(record_export_kernel, dim3((c.out_len + 1 + 255) / 256, ns), dim3(256), 0, s, c, agg, count,
                     checksum, dst);
  return hipGetLastError();
}
hipError_t launch_record_combine(const Cfg& c, const uint8_t* parts, uint32_t nparts, uint8_t* out, uint32_t* err,
                                 hipStream_t s) {
  hipLaunchKernelGGL(record_combine_kernel, dim3((c.out_len + 1 + 255) / 256), dim3(256), 0, s, c, parts, nparts,
                     out, err);
  return hipGetLastError();
}
hipError_t launch_transpose_out(const Cfg& c, const uint4* outs, uint64_t n, uint8_t* dst, hipStream_t s) {
  uint64_t t = n * c.out_len;
  hipLaunchKernelGGL(transpose_out_kernel, dim3((uint32_t)((t + 255) / 256)), dim3(256), 0, s, c, outs, n, dst);
  return hipGetLastError();
}
hipError_t launch_scatter_jobs(const Cfg& c, const JobSlice* d_jobs, uint32_t njobs, uint64_t max_job_reports,
                               const uint4* outs, const uint8_t* verdicts, const uint8_t* msgs, const uint8_t* nonces,
                               hipStream_t s) {
  if (njobs == 0) return hipSuccess;
  const uint64_t elems = (max_job_reports + 63) / 64 * 64 * c.out_len;
  uint64_t gx = (elems + 255) / 256;
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(scatter_jobs_kernel, dim3((uint32_t)gx, njobs), dim3(256), 0, s, c, d_jobs, outs, verdicts, msgs,
                     nonces);
  return hipGetLastError();
}
hipError_t launch_agg_encode(const Cfg& c, const uint4* agg, uint8_t* dst, hipStream_t s) {
  hipLaunchKernelGGL(agg_encode_kernel, dim3((c.out_len + 255) / 256), dim3(256), 0, s, c, agg, dst);
  return hipGetLastError();
}

}  // namespace jx
