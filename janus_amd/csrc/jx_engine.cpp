// jx_engine.cpp — host side of the C ABI in include/jx_prio3.h.
//
// Owns device staging, constant tables, resident prepared batches and per-segment batch
// aggregations; sequences the K1 (XOF) -> K1' (slow path) -> K3 (FLP) -> K4 (accumulate) launches
// on one HIP stream per engine. Every entry point takes the engine mutex for the duration of the
// call only, so concurrent aggregation jobs can share an engine (each holds a batch handle). There
// is no CPU compute path: if the device or the kernels are unavailable every entry point fails with
// an error status.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "jx_engine_internal.h"
#include "jx_field.h"
#include "jx_sha_aes.h"

using namespace jx;
using namespace jxi;

// The message of the last failing call, per calling thread: an engine serves several host threads,
// and each reads the error of its own call (jx_last_error), never another thread's.
static thread_local std::string t_err;

namespace jxi {
std::string& thread_error() { return t_err; }
int32_t fail(jx_engine* e, int32_t code, const std::string& msg) {
  (void)e;
  t_err = msg;
  return code;
}
}  // namespace jxi

// every entry point: the engine mutex for the call, and a fresh per-thread error message
#define LOCK(e)                                   \
  std::lock_guard<jxi::FairMutex> _lk((e)->mu);   \
  t_err.clear()


// ---------------------------------------------------------------------------- host field helpers

static f128 h_mpow(f128 aR, uint64_t e) {
  f128 r = make128(R1_128_LO, R1_128_HI);
  while (e) {
    if (e & 1) r = mont128(r, aR);
    aR = mont128(aR, aR);
    e >>= 1;
  }
  return r;
}
static f128 h_minv(f128 aR) {
  // exponent p - 2 = 0xFFFFFFFFFFFFFFE3_FFFFFFFFFFFFFFFF, square-and-multiply from the top bit
  const uint64_t ehi = 0xFFFFFFFFFFFFFFE3ull, elo = 0xFFFFFFFFFFFFFFFFull;
  f128 r = make128(R1_128_LO, R1_128_HI);
  for (int i = 127; i >= 0; i--) {
    r = mont128(r, r);
    uint64_t bit = i >= 64 ? (ehi >> (i - 64)) & 1 : (elo >> i) & 1;
    if (bit) r = mont128(r, aR);
  }
  return r;
}
static uint4 h_u4(f128 a) {
  uint4 v;
  v.x = lo32(a.lo);
  v.y = hi32(a.lo);
  v.z = lo32(a.hi);
  v.w = hi32(a.hi);
  return v;
}
static f128 h_from_u64(uint64_t v) { return make128(v, 0); }

static int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}
static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) l++;
  return l;
}
static uint32_t isqrt_floor(uint32_t v) {
  uint32_t r = 0;
  while ((uint64_t)(r + 1) * (r + 1) <= v) r++;
  return r < 1 ? 1 : r;
}

namespace jx {
int psum_ppw(uint32_t chunk);
}

// ---------------------------------------------------------------------------- configuration

// HMAC-SHA256 states after the key block for a 32-byte key (little-endian memory words)
static void host_hmac_pads(const uint8_t key[32], uint32_t ist[8], uint32_t ost[8]) {
  uint32_t kbe[8];
  for (int i = 0; i < 8; i++)
    kbe[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) | ((uint32_t)key[4 * i + 2] << 8) |
             key[4 * i + 3];
  hmac_pads(kbe, ist, ost);
}

static int32_t make_cfg(const jx_prio3_params* p, const uint8_t* vk, uint32_t vk_len, Cfg& c, std::string& why) {
  memset(&c, 0, sizeof c);
  const bool mp = p->algo_id == ALGO_SUMVEC_F64_MULTIPROOF;
  if (mp ? (p->num_proofs < 2 || p->num_proofs > MP_MAX_PROOFS) : p->num_proofs != 1) {
    why = mp ? "num_proofs must be in [2, 8]" : "num_proofs must be 1";
    return JX_E_UNSUPPORTED;
  }
  if (vk_len != (mp ? 32u : 16u)) {
    why = "verify key length must be 16 (32 for Prio3SumVecField64MultiproofHmacSha256Aes128)";
    return JX_E_INVALID;
  }
  c.algo = p->algo_id;
  c.np = p->num_proofs;
  c.seed = mp ? 32 : 16;
  c.dst_id = mp ? 0xFFFF1003u : p->algo_id;  // core/src/vdaf.rs:18-20
  c.bits = p->bits;
  c.length = p->length;
  c.chunk = p->chunk_length;
  uint32_t arity = 0;
  switch (p->algo_id) {
    case ALGO_COUNT:
      c.meas_len = 1;
      c.out_len = 1;
      c.jr_len = 0;
      c.calls = 1;
      arity = 2;
      break;
    case ALGO_SUM:
      if (p->bits < 1 || p->bits > 64) {
        why = "Prio3Sum bits must be in [1, 64]";
        return JX_E_UNSUPPORTED;
      }
      c.meas_len = p->bits;
      c.out_len = 1;
      c.jr_len = 1;
      c.calls = p->bits;
      arity = 1;
      break;
    case ALGO_SUMVEC:
    case ALGO_SUMVEC_F64_MULTIPROOF:
      if (p->bits < 1 || p->bits > (mp ? 32u : 64u) || p->length < 1 || p->chunk_length < 1) {
        why = mp ? "Prio3SumVecField64Multiproof needs 1 <= bits <= 32, length >= 1, chunk_length >= 1"
                 : "Prio3SumVec needs 1 <= bits <= 64, length >= 1, chunk_length >= 1";
        return JX_E_UNSUPPORTED;
      }
      c.meas_len = p->bits * p->length;
      c.out_len = p->length;
      c.jr_len = 1;
      c.calls = (c.meas_len + p->chunk_length - 1) / p->chunk_length;
      arity = 2 * p->chunk_length;
      break;
    case ALGO_HISTOGRAM:
      if (p->length < 1 || p->chunk_length < 1) {
        why = "Prio3Histogram needs length >= 1, chunk_length >= 1";
        return JX_E_UNSUPPORTED;
      }
      c.meas_len = p->length;
      c.out_len = p->length;
      c.jr_len = 2;
      c.calls = (p->length + p->chunk_length - 1) / p->chunk_length;
      arity = 2 * p->chunk_length;
      c.out_is_meas = 1;
      break;
    case ALGO_FIXEDPOINT_L2: {
      // FixedPointBoundedL2VecSum::new(entries) as prio 0.16.1 sizes it (restated in
      // oracle/prio3_oracle.c cfg_make): n-bit entries (n = 16 | 32, BitSize16 / BitSize32,
      // core/src/vdaf.rs:26-33), 2n-2 norm bits, chunk0 = floor(sqrt(n*entries + 2n-2)),
      // chunk1 = floor(sqrt(entries)); chunk_length is not a parameter of this VDAF.
      if ((p->bits != 16 && p->bits != 32) || p->length < 1 || p->length > (1u << 24)) {
        why = "Prio3FixedPointBoundedL2VecSum needs bits (bitsize) 16 or 32 and 1 <= length <= 2^24";
        return JX_E_UNSUPPORTED;
      }
      c.dst_id = 0xFFFF0000u;
      c.norm_bits = 2 * p->bits - 2;
      c.meas_len = p->bits * p->length + c.norm_bits;
      c.out_len = p->length;
      c.jr_len = 2;
      c.chunk = isqrt_floor(c.meas_len);
      c.calls = (c.meas_len + c.chunk - 1) / c.chunk;
      arity = 2 * c.chunk;
      c.chunk1 = isqrt_floor(p->length);
      c.calls1 = (p->length + c.chunk1 - 1) / c.chunk1;
      c.P1 = next_pow2(1 + c.calls1);
      c.logP1 = ilog2(c.P1);
      c.gpoly1_len = 2 * (c.P1 - 1) + 1;
      c.ppw1 = 2;
      c.ngroups1 = (c.chunk1 + c.ppw1 - 1) / c.ppw1;
      break;
    }
    default:
      why = "unknown algo_id";
      return JX_E_INVALID;
  }
  const bool fp = c.algo == ALGO_FIXEDPOINT_L2;
  if (c.algo == ALGO_SUMVEC || c.algo == ALGO_HISTOGRAM || mp || fp) {
    c.ppw = psum_ppw(c.chunk);
    c.ngroups = (c.chunk + c.ppw - 1) / c.ppw;
  }
  c.ngt = c.ngroups + c.ngroups1;
  c.qr_len = fp ? 2 : 1;
  c.trunc_len = fp ? p->bits * p->length : c.out_len * c.bits;
  c.P = next_pow2(1 + c.calls);
  if (mp && c.P > (1u << 30)) {
    why = "too many gadget calls for Field64";
    return JX_E_UNSUPPORTED;
  }
  c.logP = ilog2(c.P);
  c.gpoly_len = 2 * (c.P - 1) + 1;
  c.proof_len = arity + c.gpoly_len;
  c.ver_len = arity + 2;
  if (fp) {  // gadget 1's sub-proof [seeds || gadget poly] and verifier part [wires || G1(t1)]
    c.proof1_off = c.proof_len;
    c.proof_len += c.chunk1 + c.gpoly1_len;
    c.ver_len += c.chunk1 + 1;
  }
  const uint32_t fb = (c.algo == ALGO_COUNT || mp) ? 8 : 16;
  c.fb = fb;
  const bool jr = c.jr_len > 0;
  const uint32_t S = c.seed;
  c.ps_bytes = jr ? 2 * S : 0;
  c.his_bytes = jr ? 3 * S : 2 * S;
  c.lps_bytes = c.np * c.ver_len * fb + (jr ? S : 0);
  c.lis_bytes = (c.meas_len + c.np * c.proof_len) * fb + (jr ? S : 0);
  if (mp) {
    c.nco = MCOEF_K + 2 * c.calls;
    c.ncoef = 0;
    host_hmac_pads(vk, c.vk_ist, c.vk_ost);
    const uint8_t zero[32] = {0};
    host_hmac_pads(zero, c.zero_ist, c.zero_ost);
  } else if (c.algo == ALGO_COUNT)
    c.ncoef = 0;
  else if (c.algo == ALGO_SUM)
    c.ncoef = COEF_K + c.calls;
  else
    c.ncoef = COEF_K + 2 * c.calls;
  if (c.algo == ALGO_SUMVEC || c.algo == ALGO_HISTOGRAM || fp) {  // gadget 0's power tables (jx_kernels.h)
    c.c_rpow = c.ncoef;
    c.ncoef += c.chunk;
    c.c_tpow = c.ncoef;
    c.ncoef += c.ngroups;
  }
  if (fp) {
    c.coef1 = c.ncoef;
    c.ncoef += G1_K + c.calls1;
  }
  for (int i = 0; i < 4; i++)
    c.vk[i] = (uint32_t)vk[4 * i] | ((uint32_t)vk[4 * i + 1] << 8) | ((uint32_t)vk[4 * i + 2] << 16) |
              ((uint32_t)vk[4 * i + 3] << 24);
  c.c_omega = 0;
  c.c_S = c.P;
  c.c_misc = c.P + c.gpoly_len;
  c.c_omega1 = c.c_misc + NMISC;
  c.c_S1 = c.c_omega1 + c.P1;
  return JX_OK;
}

// constant tables: w^k R (k < P), S_m R = (sum_{k=1..calls} w^{km}) R (m < gpoly_len), misc
static uint4 h_u4_64(uint64_t v) {
  uint4 r;
  r.x = lo32(v);
  r.y = hi32(v);
  r.z = r.w = 0;
  return r;
}

// w1^k R (k < P1) and S1_m R for gadget 1 of FixedPointBoundedL2VecSum
static void root_tables(f128 gen, uint32_t P, uint32_t logP, uint32_t calls, uint32_t glen, uint4* omega, uint4* S) {
  f128 w = gen;
  for (int i = 0; i < 66 - (int)logP; i++) w = mont128(w, w);
  f128 wk = make128(R1_128_LO, R1_128_HI);
  std::vector<f128> pw(P);
  for (uint32_t k = 0; k < P; k++) {
    pw[k] = wk;
    omega[k] = h_u4(wk);
    wk = mont128(wk, w);
  }
  for (uint32_t m = 0; m < glen; m++) {
    f128 s = make128(0, 0);
    for (uint32_t k = 1; k <= calls; k++) s = add128(s, pw[(uint64_t)(k * m) % P]);
    S[m] = h_u4(s);
  }
}

static std::vector<uint4> make_consts(const Cfg& c) {
  std::vector<uint4> t(c.P + c.gpoly_len + NMISC + c.P1 + c.gpoly1_len);
  if (c.algo == ALGO_COUNT) return t;
  if (c.algo == ALGO_SUMVEC_F64_MULTIPROOF) {
    // Field64: GEN = 7^((p-1)/2^32) (order 2^32), w = GEN^(2^(32 - logP)); canonical values
    uint64_t w = pow64_h(pow64_h(7, (P64 - 1) >> 32), 1ull << (32 - c.logP));
    std::vector<uint64_t> pw(c.P);
    uint64_t wk = 1;
    for (uint32_t k = 0; k < c.P; k++) {
      pw[k] = wk;
      t[c.c_omega + k] = h_u4_64(wk);
      wk = mul64(wk, w);
    }
    for (uint32_t m = 0; m < c.gpoly_len; m++) {
      uint64_t s = 0;
      for (uint32_t k = 1; k <= c.calls; k++) s = add64(s, pw[(uint64_t)(k * m) % c.P]);
      t[c.c_S + m] = h_u4_64(s);
    }
    t[c.c_misc + 0] = h_u4_64(pow64_h(c.P, P64 - 2));  // 1/P
    t[c.c_misc + 1] = h_u4_64(pow64_h(2, P64 - 2));    // 1/2
    return t;
  }
  // GEN = 7^((p-1)/2^66), order 2^66; w = GEN^(2^(66 - logP))
  f128 gen = h_mpow(to_mont128(h_from_u64(7)), 4611686018427387897ull);
  root_tables(gen, c.P, c.logP, c.calls, c.gpoly_len, &t[c.c_omega], &t[c.c_S]);
  f128 invP = h_minv(to_mont128(h_from_u64(c.P)));
  f128 half_m = h_minv(to_mont128(h_from_u64(2)));
  t[c.c_misc + 0] = h_u4(invP);                     // (1/P) R
  t[c.c_misc + 1] = h_u4(from_mont128(half_m));     // 1/2 canonical
  t[c.c_misc + 2] = h_u4(make128(R1_128_LO, R1_128_HI));
  t[c.c_misc + 3] = h_u4(half_m);                   // (1/2) R
  if (c.algo == ALGO_FIXEDPOINT_L2) {
    const uint32_t n = c.bits;
    t[c.c_misc + 4] = h_u4(make128(n < 64 ? 1ull << n : 0, n >= 64 ? 1ull << (n - 64) : 0));  // 2^n
    const uint32_t e2 = 2 * n - 2;                                                           // 2^(2n-2) R^-1
    t[c.c_misc + 5] = h_u4(from_mont128(make128(e2 < 64 ? 1ull << e2 : 0, e2 >= 64 ? 1ull << (e2 - 64) : 0)));
    t[c.c_misc + 6] = h_u4(make128(1ull << (n - 2), 0));                                      // 2^(n-2)
    t[c.c_misc + 7] = h_u4(h_minv(to_mont128(h_from_u64(c.P1))));                            // (1/P1) R
    root_tables(gen, c.P1, c.logP1, c.calls1, c.gpoly1_len, &t[c.c_omega1], &t[c.c_S1]);
  }
  return t;
}

// ---------------------------------------------------------------------------- staging (per call, from the arena)

// staging element bytes: the multiproof Field64 kernels use 8-byte elements (outputs stay uint4)
static uint32_t stage_eb(const Cfg& c) { return c.algo == ALGO_SUMVEC_F64_MULTIPROOF ? 8u : 16u; }
static uint64_t coef_elems(const Cfg& c) { return c.algo == ALGO_SUMVEC_F64_MULTIPROOF ? (uint64_t)c.np * c.nco : c.ncoef; }
static uint64_t part_bytes(const Cfg& c) {
  return c.algo == ALGO_SUMVEC_F64_MULTIPROOF ? 24ull * c.np * c.ngroups : 64ull * c.ngt;
}
// the output shares alias the measurement-share staging (Histogram: output = measurement share)
static bool outs_alias_meas(const Cfg& c) { return c.out_is_meas && c.algo != ALGO_COUNT; }
// The leader's FLP kernels read its explicit measurement share in place (Bufs::meas_rs) instead of a
// staged copy: every TurboSHAKE instance whose output is not the measurement share itself.
static bool leader_inplace(const Cfg& c) {
  return c.algo == ALGO_SUM || c.algo == ALGO_SUMVEC || c.algo == ALGO_FIXEDPOINT_L2;
}

namespace jxi {
size_t align256(size_t v) { return (v + 255) / 256 * 256; }
uint32_t vk_row_bytes(const Cfg& c) { return c.algo == ALGO_SUMVEC_F64_MULTIPROOF ? 64u : 16u; }
void vk_row(const Cfg& c, uint8_t* dst) {
  if (c.algo == ALGO_SUMVEC_F64_MULTIPROOF) {  // the HMAC-SHA256 pads of the 32-byte key: ist[8] || ost[8]
    memcpy(dst, c.vk_ist, 32);
    memcpy(dst + 32, c.vk_ost, 32);
  } else {
    memcpy(dst, c.vk, 16);
  }
}
}  // namespace jxi

// Staging bytes of one report for a fused helper launch (the launch-size budget, jx_engine_create_ex).
static uint64_t per_report_bytes(const Cfg& c, bool with_meas = true) {
  uint64_t b = (uint64_t)stage_eb(c) * ((with_meas ? c.meas_len : 0) + (uint64_t)c.np * c.proof_len + coef_elems(c));
  b += 16ull * (c.out_is_meas ? 0 : c.out_len);
  b += 16 + c.ps_bytes + c.his_bytes + c.lps_bytes + 4 + 1 + c.seed + 1 + 4 + 1;
  b += part_bytes(c);  // FLP partial sums
  return b;
}

// Report chunks of accumulate_kernel: one wave per (output element, chunk), so short outputs
// (Count, Sum: 1 element) need many chunks to fill the device; >= 16384 waves in total.
static uint32_t acc_nchunks(const jx_engine* e) {
  if (e->acc_chunks) return e->acc_chunks;
  const uint32_t want = (16384u + e->cfg.out_len - 1) / e->cfg.out_len;
  return want < 16u ? 16u : (want > 4096u ? 4096u : want);
}

// Lay the regions named by `fl` for `cap` reports out from `base` (nullptr: only size them).
static size_t stage_layout(jx_engine* e, uint64_t cap, uint32_t fl, uint8_t* base) {
  const Cfg& c = e->cfg;
  const uint64_t eb = stage_eb(c);
  size_t off = 0;
  auto take = [&](auto*& p, size_t bytes) {
    using T = std::remove_reference_t<decltype(p)>;
    if (base) p = reinterpret_cast<T>(base + off);
    off += align256(bytes ? bytes : 1);
  };
  if (fl & SG_IN) {
    take(e->d_nonces, cap * 16);
    take(e->d_ps, cap * c.ps_bytes);
  }
  if (fl & SG_HIN) {
    take(e->d_his, cap * c.his_bytes);
    take(e->d_lps, cap * c.lps_bytes);
  }
  if (fl & SG_MEAS) take(e->d_meas, cap * c.meas_len * eb);
  if (fl & SG_PREP) {
    take(e->d_proof, cap * c.np * c.proof_len * eb);
    if (!outs_alias_meas(c)) take(e->d_outs, cap * c.out_len * 16);
    take(e->d_coef, cap * coef_elems(c) * eb);
    take(e->d_flags, cap * 4);
    take(e->d_part, cap * part_bytes(c));
  }
  if (fl & SG_RES) {
    take(e->d_verdicts, cap);
    take(e->d_msgs, cap * c.seed);
  }
  if (fl & SG_ACC) {
    take(e->d_mask, cap);
    take(e->d_seg, cap * 4);
    take(e->d_partials, (size_t)acc_nchunks(e) * c.out_len * 3 * sizeof(uint64_t) + cap);
  }
  if (fl & SG_LEAD) {
    take(e->d_lis, cap * e->lis_stride);
    take(e->d_lps_out, cap * c.lps_bytes);
  }
  if (fl & SG_LMSG) take(e->d_in_msgs, cap * c.seed);
  if (fl & SG_VK) take(e->d_vkeys, cap * vk_row_bytes(c));
  if (fl & SG_JOBS) take(e->d_jobs, (size_t)MAX_JOBS_PER_LAUNCH * sizeof(JobSlice));
  if (fl & SG_ENC) {
    take(e->d_encrows, cap * sizeof(EncRow));
    take(e->d_ct, e->enc_ct_bytes);
    take(e->d_pt, e->enc_ct_bytes);
    take(e->d_keys, (size_t)ENC_MAX_KEYS * sizeof(HpkeKeyRow));
    take(e->d_status, cap);
  }
  return off;
}

static void stage_clear(jx_engine* e) {
  e->d_nonces = e->d_ps = e->d_his = e->d_lps = nullptr;
  e->d_meas = e->d_proof = e->d_outs = e->d_coef = nullptr;
  e->d_flags = nullptr;
  e->d_part = nullptr;
  e->d_verdicts = e->d_msgs = nullptr;
  e->d_partials = nullptr;
  e->d_mask = nullptr;
  e->d_seg = nullptr;
  e->d_lis = e->d_lps_out = e->d_in_msgs = nullptr;
  e->d_vkeys = nullptr;
  e->d_jobs = nullptr;
  e->d_encrows = nullptr;
  e->d_ct = e->d_pt = e->d_status = nullptr;
  e->d_keys = nullptr;
  e->cap = 0;
  e->stage_flags = 0;
}

namespace jxi {
size_t stage_bytes(const jx_engine* e, uint64_t cap, uint32_t flags) {
  return stage_layout(const_cast<jx_engine*>(e), (cap + 63) / 64 * 64, flags, nullptr);
}

// JX_E_NOMEM naming what holds the device memory (resident batches are the caller's to release).
static int32_t nomem(jx_engine* e, const char* what, size_t bytes) {
  uint64_t held = 0;
  for (auto& kv : e->batches) held += kv.second.slab.bytes;
  Arena* A = e->arena;
  return fail(e, JX_E_NOMEM,
              std::string(what) + ": out of device memory allocating " + std::to_string(bytes) + " B; " +
                  std::to_string(e->batches.size()) + " resident batches of this engine hold " + std::to_string(held) +
                  " B; the device arena holds " + std::to_string(A->allocated) + " of its " + std::to_string(A->budget) +
                  " B budget (release finished or abandoned jobs with jx_batch_release)");
}

int32_t stage_acquire(jx_engine* e, uint64_t n, uint32_t fl, Stage& st, bool may_wait) {
  st.release();
  const uint64_t cap = (n + 63) / 64 * 64;
  const size_t bytes = stage_layout(e, cap, fl, nullptr);
  hipError_t rc = arena_get(e->arena, bytes, e->stream, true, may_wait, st.slab);
  if (rc == hipErrorOutOfMemory) return nomem(e, "staging", bytes);
  HIPCHK(e, rc);
  st.e = e;
  stage_layout(e, cap, fl, (uint8_t*)st.slab.p);
  e->cap = cap;
  e->stage_flags = fl;
  return JX_OK;
}

void Stage::release() {
  if (!e) return;
  arena_put(e->arena, slab, e->stream);
  stage_clear(e);
  e = nullptr;
}
}  // namespace jxi

// the fused paths' output shares (engine staging)
uint4* jxi::staging_outs(jx_engine* e) { return outs_alias_meas(e->cfg) ? e->d_meas : e->d_outs; }

// Per-call device scratch from the arena, handed back stream-ordered on the engine stream when it goes out of
// scope: no hipMalloc / hipFree / stream synchronize on a call path (hipFree waits for the device, and every
// engine's launches on it).
namespace {
struct Scratch {
  jx_engine* e = nullptr;
  Slab s;
  Scratch() = default;
  Scratch(const Scratch&) = delete;
  Scratch& operator=(const Scratch&) = delete;
  ~Scratch() {
    if (s.p) arena_put(e->arena, s, e->stream);
  }
  uint8_t* p() const { return (uint8_t*)s.p; }
};
}  // namespace

// may_wait: the caller holds no other staging (arena_get's rule)
static int32_t scratch_get(jx_engine* e, size_t bytes, Scratch& out, bool may_wait = false) {
  out.e = e;
  const hipError_t st = arena_get(e->arena, bytes, e->stream, true, may_wait, out.s);
  if (st == hipErrorOutOfMemory) return nomem(e, "scratch", bytes);
  HIPCHK(e, st);
  return JX_OK;
}

// Running aggregations: segment states (aggregate share | checksum | count) carved from arena slabs of
// kSegsPerSlab states, so a new batch-aggregation id costs no device allocation on the call path (one slab per
// kSegsPerSlab ids, held until the engine is destroyed).
constexpr uint32_t kSegsPerSlab = 64;
static size_t seg_state_bytes(const Cfg& c) { return align256((size_t)c.out_len * 16 + 32 + 8); }

static int32_t get_segment(jx_engine* e, uint32_t id, Segment** out) {
  auto it = e->segs.find(id);
  if (it == e->segs.end()) {
    const size_t sb = seg_state_bytes(e->cfg);
    if (e->seg_slabs.empty() || e->seg_next == kSegsPerSlab) {
      Slab sl;
      const hipError_t st = arena_get(e->arena, sb * kSegsPerSlab, e->stream, false, false, sl);
      if (st == hipErrorOutOfMemory) return nomem(e, "batch aggregations", sb * kSegsPerSlab);
      HIPCHK(e, st);
      e->seg_slabs.push_back(sl);
      e->seg_next = 0;
    }
    uint8_t* m = (uint8_t*)e->seg_slabs.back().p + sb * e->seg_next++;
    Segment s;
    s.agg = (uint4*)m;
    s.checksum = (uint32_t*)(m + (size_t)e->cfg.out_len * 16);
    s.count = (unsigned long long*)(m + (size_t)e->cfg.out_len * 16 + 32);
    HIPCHK(e, hipMemsetAsync(m, 0, sb, e->stream));
    it = e->segs.emplace(id, s).first;
  }
  *out = &it->second;
  return JX_OK;
}

// ---------------------------------------------------------------------------- resident batches

// A new resident batch of n reports (handle in *id), one arena allocation. Slabs handed back by released
// batches (of any engine on the device) are reused stream-ordered.
int32_t jxi::batch_new(jx_engine* e, uint64_t n, bool leader, uint64_t* id, Batch** out) {
  const Cfg& c = e->cfg;
  const uint64_t cap = (n + 63) / 64 * 64;
  const size_t o_outs = 0, o_ver = align256((size_t)cap * c.out_len * 16), o_msg = o_ver + align256(cap),
               o_non = o_msg + align256((size_t)cap * c.seed), bytes = o_non + align256(cap * 16);
  Batch b;
  b.n = n;
  b.leader = leader;
  // a slab a deferred-accumulate flush has read (the same job size comes back every time): no arena round trip;
  // its users wait on that flush (e->stream is in order after it already)
  auto rit = e->recycle.lower_bound(bytes);
  if (rit != e->recycle.end() && rit->first <= bytes + bytes / 4) {
    b.slab = rit->second;
    b.wait_ev = e->ev_flush;
    e->recycle_bytes -= rit->first;
    e->recycle.erase(rit);
  } else {
    hipError_t st = arena_get(e->arena, bytes, e->stream, false, false, b.slab);
    if (st == hipErrorOutOfMemory) return nomem(e, "new batch", bytes);
    HIPCHK(e, st);
  }
  uint8_t* m = (uint8_t*)b.slab.p;
  b.outs = (uint4*)(m + o_outs);
  b.verdicts = m + o_ver;
  b.msgs = m + o_msg;
  b.nonces = m + o_non;
  *id = ++e->batch_gen;
  e->last_batch = *id;
  *out = &e->batches.emplace(*id, b).first->second;
  return JX_OK;
}

void jxi::batch_free(jx_engine* e, std::map<uint64_t, Batch>::iterator it) {
  arena_put(e->arena, it->second.slab, e->stream);  // reused after the work queued on the engine stream
  if (e->last_batch == it->first) e->last_batch = 0;
  e->batches.erase(it);
}

static int32_t find_batch(jx_engine* e, uint64_t id, uint64_t n, const char* what, Batch** out) {
  auto it = e->batches.find(id);
  if (id == 0 || it == e->batches.end() || __atomic_load_n(&it->second.pending, __ATOMIC_ACQUIRE))
    return fail(e, JX_E_STATE, std::string(what) + ": batch id names no resident prepared batch (released or never made)");
  if (it->second.n != n)
    return fail(e, JX_E_INVALID, std::string(what) + ": report count differs from the batch's");
  *out = &it->second;
  return JX_OK;
}

static AccSrc batch_src(const Batch& b) { return AccSrc{b.n, b.outs, b.verdicts, b.nonces}; }

// ---------------------------------------------------------------------------- timing

static hipError_t stage_begin(jx_engine* e, hipEvent_t* ev) {
  if (!e->timing) return hipSuccess;
  hipError_t st = hipEventCreate(ev);
  if (st != hipSuccess) return st;
  return hipEventRecord(*ev, e->stream);
}
static hipError_t stage_end(jx_engine* e, int stage, hipEvent_t ev0) {
  e->launches[stage]++;
  if (!e->timing) return hipSuccess;
  hipEvent_t ev1;
  hipError_t st = hipEventCreate(&ev1);
  if (st != hipSuccess) return st;
  st = hipEventRecord(ev1, e->stream);
  e->pending.push_back({stage, {ev0, ev1}});
  return st;
}
int32_t jxi::drain_timing(jx_engine* e) {
  if (e->pending.empty()) return JX_OK;
  HIPCHK(e, hipStreamSynchronize(e->stream));
  for (auto& p : e->pending) {
    float t = 0;
    HIPCHK(e, hipEventElapsedTime(&t, p.second.first, p.second.second));
    e->ms[p.first] += t;
    (void)hipEventDestroy(p.second.first);
    (void)hipEventDestroy(p.second.second);
  }
  e->pending.clear();
  return JX_OK;
}

static bool use_inplace(const jx_engine* e) { return leader_inplace(e->cfg); }

// ---------------------------------------------------------------------------- core sequencing

// Prepare n <= cap reports whose inputs are at the given device pointers; the output shares go to
// outs (a batch's buffer, or the staging of the fused paths), verdicts and prep messages / leader
// seeds to verdicts / msgs.
int32_t jxi::prep_core(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* his,
                       const uint8_t* lps, uint8_t* verdicts, uint8_t* msgs, uint4* outs, const uint8_t* lis,
                       uint8_t* lps_out, uint64_t lis_rs, const uint8_t* vkeys, hipEvent_t before_flp,
                       const std::function<int32_t()>* after_k1) {
  const Cfg& c = e->cfg;
  const bool leader = lis != nullptr;
  Bufs b{};
  b.n = n;
  b.nonces = nonces;
  b.ps = ps;
  b.his = his;
  b.lps = lps;
  b.lis = lis;
  b.lis_rs = lis_rs ? lis_rs : c.lis_bytes;
  b.vkeys = vkeys;
  b.lps_out = lps_out;
  b.leader = leader ? 1u : 0u;
  b.meas = outs_alias_meas(c) ? outs : e->d_meas;
  if (leader && use_inplace(e)) {
    b.meas_src = lis;
    b.meas_rs = b.lis_rs;
  }
  b.proof = e->d_proof;
  b.outs = outs;
  b.coef = e->d_coef;
  b.flags = e->d_flags;
  b.part = e->d_part;
  b.verdicts = verdicts;
  b.msgs = msgs;
  b.consts = e->d_consts;
  b.force_slow = e->force_slow;
  b.k1_split = e->k1_split;
  b.k1_lds = lanes_lds_bytes(e->lanes_wg_cap);
  // A helper launch that would give the fused two-sponge K1 less than one wave per SIMD is bound by
  // the per-report sponge latency, not by issue: the lane-split kernel runs it in twice the waves
  // (FixedPointBoundedL2VecSum 16 x 10000, 24,576 reports: 153 -> 92 ms on MI355X), below one
  // lane-split wave per SIMD the lane-pair kernel splits every sponge over two lanes, and up to one
  // report-wave per SIMD the word-per-lane kernel spreads it over 25 (round_reports: the fused kernel's
  // two waves per SIMD, 4 x that many lane-split or 8 x lane-pair lanes; profiles/r05_words_sweep.jsonl).
  const bool wide = c.bits > 32 && (c.algo == ALGO_SUM || c.algo == ALGO_SUMVEC);
  if (e->k1_split == 0 && !leader && !wide && e->round_reports) {
    if (128 * n <= e->round_reports)  // a report per wave, <= one wave per SIMD (1,024 on MI355X): 2.6 vs 3.6 ms
      b.k1_split = 7;
    else if (4 * n <= e->round_reports)
      b.k1_split = 6;
    else if (2 * n <= e->round_reports)
      b.k1_split = 3;
  }
  // the lane pairs with unrolled rounds while each pair-wave has a SIMD to itself (<= 16,384 reports on MI355X)
  if (b.k1_split == 6 && 8 * n <= e->round_reports) b.k1_split = 8;
  // A lane-pair launch of at most half the CUs' workgroups (<= 8,192 reports on MI355X: the coalescer's launches
  // of Janus-sized jobs, two in flight) reserves LDS for one workgroup per CU, so a second such launch lands on
  // other CUs instead of doubling up SIMDs with the first (profiles/r06_jobs_*: K1 3.6 ms alone, 4.5 ms beside
  // another launch on shared CUs).
  if ((b.k1_split == 8 || b.k1_split == 6) && e->k1_split == 0 && 16 * n <= e->round_reports)
    b.k1_pairs_lds = lanes_lds_bytes(1);
  // A lane-split launch past one wave per SIMD puts two of its long chains on some SIMDs and the launch waits
  // for those. Instead the first round_reports / 4 reports (a lane-split wave per SIMD) run lane-split and the
  // rest as lane pairs beside them on the side stream: FixedPointBoundedL2VecSum 16 x 10000, 40,960 reports,
  // 148.4 -> 123.5 ms (tools/kernel_probe fpmix, profiles/r05_fp_mixed_k1.jsonl). Only while no other engine
  // on the device has a large K1 launch in flight: beside the leader's 640 K1 waves (configs[4] with two jobs in
  // flight) the 1,536 mixed waves pack worse than 1,280 lane-split ones (helper K1 154 -> 161 ms, every split
  // point tried; profiles/r05_fp_mixed_k1.jsonl).
  const uint64_t split_at = e->round_reports / 4 / 64 * 64;
  const bool big = split_at && n > split_at;
  const bool mixed = e->k1_split == 0 && b.k1_split == 3 && !wide && big && c.algo != ALGO_COUNT &&
                     c.algo != ALGO_SUMVEC_F64_MULTIPROOF && !arena_big_busy(e->arena, e);
  hipEvent_t ev = nullptr;
  if (c.algo == ALGO_COUNT) {
    HIPCHK(e, stage_begin(e, &ev));
    HIPCHK(e, launch_count(c, b, e->stream));
    HIPCHK(e, stage_end(e, ST_XOF, ev));
  } else if (c.algo == ALGO_SUMVEC_F64_MULTIPROOF) {
    HIPCHK(e, stage_begin(e, &ev));
    HIPCHK(e, launch_mp_xof(c, b, e->stream));
    HIPCHK(e, stage_end(e, ST_XOF, ev));
    if (!leader) {
      HIPCHK(e, stage_begin(e, &ev));
      HIPCHK(e, launch_mp_slow(c, b, e->stream));
      HIPCHK(e, stage_end(e, ST_SLOW, ev));
    }
    HIPCHK(e, stage_begin(e, &ev));
    HIPCHK(e, launch_mp_flp(c, b, e->stream));
    HIPCHK(e, stage_end(e, ST_FLP, ev));
  } else {
    HIPCHK(e, stage_begin(e, &ev));
    if (mixed) {
      if (!e->side) HIPCHK(e, hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking));
      if (!e->ev_fork) HIPCHK(e, hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
      if (!e->ev_side) HIPCHK(e, hipEventCreateWithFlags(&e->ev_side, hipEventDisableTiming));
      Bufs head = b, tail = bufs_tail(c, b, split_at);
      head.n = split_at;
      tail.k1_split = 8 * tail.n <= e->round_reports ? 8u : 6u;
      tail.k1_pairs_lds = 0;
      HIPCHK(e, hipEventRecord(e->ev_fork, e->stream));
      HIPCHK(e, hipStreamWaitEvent(e->side, e->ev_fork, 0));
      HIPCHK(e, launch_xof(c, head, e->stream));
      HIPCHK(e, launch_xof(c, tail, e->side));
      HIPCHK(e, hipEventRecord(e->ev_side, e->side));
      HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev_side, 0));
    } else {
      HIPCHK(e, launch_xof(c, b, e->stream));
    }
    if (big) HIPCHK(e, arena_big_record(e->arena, e, e->stream));
    HIPCHK(e, stage_end(e, ST_XOF, ev));
    if (after_k1) {
      const int32_t rc = (*after_k1)();
      if (rc) return rc;
    }
    if (!leader) {  // the leader's shares are explicit: no rejection-sampled streams to redo
      HIPCHK(e, stage_begin(e, &ev));
      HIPCHK(e, launch_xof_slow(c, b, e->stream));
      HIPCHK(e, stage_end(e, ST_SLOW, ev));
    }
    // the caller's upload of the rest of the leader prep shares (K1 reads only their joint-rand parts)
    if (before_flp) HIPCHK(e, hipStreamWaitEvent(e->stream, before_flp, 0));
    HIPCHK(e, stage_begin(e, &ev));
    HIPCHK(e, launch_flp(c, b, e->stream));
    HIPCHK(e, stage_end(e, ST_FLP, ev));
  }
  return JX_OK;
}

// Accumulate the finished (and, with d_mask, accepted) reports of src into one aggregation. With
// d_dense (dense per-report indices), only reports whose index is 0 are taken.
static int32_t accumulate_one(jx_engine* e, const AccSrc& src, const uint8_t* d_mask, const uint32_t* d_dense,
                              const Segment& t) {
  const Cfg& c = e->cfg;
  AccArgs a{};
  a.n = src.n;
  a.outs = src.outs;
  a.out_len = c.out_len;
  a.verdicts = src.verdicts;
  a.mask = d_mask;
  a.seg = d_dense;
  a.seg_id = 0;
  a.partials = e->d_partials;
  a.nchunks = acc_nchunks(e);
  uint64_t nblk = (src.n + 63) / 64;
  a.blocks_per_chunk = (uint32_t)((nblk + a.nchunks - 1) / a.nchunks);
  if (a.blocks_per_chunk == 0) a.blocks_per_chunk = 1;
  a.nonces = src.nonces;
  a.checksum = t.checksum;
  a.count = t.count;
  hipEvent_t ev = nullptr;
  HIPCHK(e, stage_begin(e, &ev));
  if (src.n <= ACC_SMALL)
    HIPCHK(e, launch_accumulate_small(c, a, t.agg, e->stream));
  else
    HIPCHK(e, launch_accumulate(c, a, t.agg, e->stream));
  HIPCHK(e, stage_end(e, ST_ACC, ev));
  return JX_OK;
}

// Run the deferred accumulations (jx_accumulate): per aggregation, up to ACC_MULTI_MAX batches per
// accumulate_multi launch; their slabs go back to the arena stream-ordered after the launches. One launch per
// aggregation instead of one per job takes the per-job kernel launch off the engine mutex (a coalesced 100-report
// job's callers return together, and each one's accumulate launch serialised them).
constexpr uint64_t kAccQReports = 16384;  // a flush once this many reports wait (their batches hold HBM)
constexpr size_t kRecycleBytes = 512ull << 20;  // batch slabs an engine keeps from its flushes
static int32_t flush_acc(jx_engine* e) {
  if (e->accq.empty()) return JX_OK;
  std::vector<std::pair<Batch, uint32_t>> q;
  q.swap(e->accq);
  e->accq_reports = 0;
  e->acc_flushes++;
  std::map<uint32_t, std::vector<size_t>> by;
  for (size_t k = 0; k < q.size(); k++) by[q[k].second].push_back(k);
  auto run = [&]() -> int32_t {
    HIPCHK(e, hipSetDevice(e->device));
    for (auto& kv : by) {
      Segment* s = nullptr;
      int32_t rc = get_segment(e, kv.first, &s);
      if (rc) return rc;
      const std::vector<size_t>& ix = kv.second;
      for (size_t o = 0; o < ix.size(); o += ACC_MULTI_MAX) {
        AccMultiArgs a{};
        a.agg = s->agg;
        a.count = s->count;
        a.checksum = s->checksum;
        for (size_t j = o; j < ix.size() && a.nb < ACC_MULTI_MAX; j++) {
          const Batch& b = q[ix[j]].first;
          a.d[a.nb++] = AccDesc{b.outs, b.verdicts, b.nonces, b.n};
        }
        hipEvent_t ev = nullptr;
        HIPCHK(e, stage_begin(e, &ev));
        HIPCHK(e, launch_accumulate_multi(e->cfg, a, e->stream));
        HIPCHK(e, stage_end(e, ST_ACC, ev));
      }
    }
    return JX_OK;
  };
  int32_t rc = run();
  // the slabs: kept for the engine's next batches behind one event (up to kRecycleBytes), the rest back to the
  // arena, after the launches that read them
  if (rc == JX_OK && !e->ev_flush && hipEventCreateWithFlags(&e->ev_flush, hipEventDisableTiming) != hipSuccess)
    e->ev_flush = nullptr;
  const bool keep = rc == JX_OK && e->ev_flush && hipEventRecord(e->ev_flush, e->stream) == hipSuccess;
  for (auto& p : q) {
    Slab& sl = p.first.slab;
    if (keep && e->recycle_bytes + sl.bytes <= kRecycleBytes) {
      e->recycle_bytes += sl.bytes;
      e->recycle.emplace(sl.bytes, sl);
    } else {
      arena_put(e->arena, sl, e->stream);
    }
  }
  return rc;
}
#define FLUSH_ACC(e)                 \
  do {                               \
    int32_t _fr = flush_acc(e);      \
    if (_fr) return _fr;             \
  } while (0)

// Upload the device pointer table (aggs, counts, checksums) of `targets` into per-call scratch `tbl` (e->d_ptrs
// points at it while it is held). The pinned host copy is double-buffered and reused only once the upload
// that last read it has completed, so the host never waits for the call's own kernels.
static int32_t upload_targets(jx_engine* e, const std::vector<Segment>& targets, Scratch& tbl) {
  const uint64_t S = targets.size();
  int32_t rc = scratch_get(e, 3 * S * sizeof(void*), tbl);
  if (rc) return rc;
  e->d_ptrs = (void**)tbl.p();
  const int k = e->ptrs_k;
  e->ptrs_k ^= 1;
  if (!e->ev_ptrs[k]) HIPCHK(e, hipEventCreateWithFlags(&e->ev_ptrs[k], hipEventDisableTiming));
  else HIPCHK(e, hipEventSynchronize(e->ev_ptrs[k]));
  if (e->h_ptrs_cap[k] < S) {
    if (e->h_ptrs[k]) (void)hipHostFree(e->h_ptrs[k]);
    e->h_ptrs[k] = nullptr;
    HIPCHK(e, hipHostMalloc((void**)&e->h_ptrs[k], 3 * S * sizeof(void*), hipHostMallocDefault));
    e->h_ptrs_cap[k] = S;
  }
  void** h = e->h_ptrs[k];
  for (uint64_t t = 0; t < S; t++) {
    h[t] = targets[t].agg;
    h[S + t] = targets[t].count;
    h[2 * S + t] = targets[t].checksum;
  }
  HIPCHK(e, hipMemcpyAsync(e->d_ptrs, h, 3 * S * sizeof(void*), hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipEventRecord(e->ev_ptrs[k], e->stream));
  return JX_OK;
}

// Reports per segmented-accumulate work item: enough items that out_len x items >= 16384 waves.
static uint32_t seg_items_len(const jx_engine* e, uint64_t n) {
  const uint64_t nch = acc_nchunks(e);
  uint64_t L = (n + nch - 1) / nch;
  L = (L + 63) / 64 * 64;
  return (uint32_t)(L < 64 ? 64 : L);
}

// Accumulate the finished, accepted reports of src into the aggregations named by a dense per-report
// index d_dense[r] in [0, S) (S = segments of the table uploaded by upload_targets; indices >= S are
// skipped); one pass per SEG_MAX segments.
static int32_t accumulate_many(jx_engine* e, const AccSrc& src, const uint8_t* d_mask, const uint32_t* d_dense,
                               uint64_t S) {
  const Cfg& c = e->cfg;
  const uint64_t n = src.n;
  if (S == 0 || n == 0) return JX_OK;
  // per-pass segments: SEG_MAX, or fewer when the per-item partials would exceed ~512 MiB
  const uint32_t L = seg_items_len(e, n);
  const uint64_t items_n = (n + L - 1) / L;
  const uint64_t per_item = (uint64_t)c.out_len * 24;
  uint64_t ns_max = (512ull << 20) / per_item;
  ns_max = ns_max > items_n + 64 ? ns_max - items_n : 64;
  if (ns_max > SEG_MAX) ns_max = SEG_MAX;
  const uint64_t wmax = items_n + (S < ns_max ? S : ns_max);
  // the counting-sort state, permutation, work items and partials: one per-call scratch slab (reused from the
  // arena stream-ordered; no allocation or synchronization once warm)
  const size_t o_segx = 0, o_perm = align256((4 * SEG_MAX + 3) * sizeof(uint32_t)),
               o_items = o_perm + align256(n * sizeof(uint32_t)), o_spart = o_items + align256(wmax * sizeof(uint4)),
               wbytes = o_spart + align256(wmax * per_item);
  Scratch work;
  int32_t rc = scratch_get(e, wbytes, work);
  if (rc) return rc;
  e->d_segx = (uint32_t*)(work.p() + o_segx);
  e->d_perm = (uint32_t*)(work.p() + o_perm);
  e->d_items = (uint4*)(work.p() + o_items);
  e->d_spart = (uint64_t*)(work.p() + o_spart);
  uint64_t grid = (n + 255) / 256;
  if (grid > SELECT_WGS) grid = SELECT_WGS;
  for (uint64_t s0 = 0; s0 < S; s0 += ns_max) {
    const uint32_t ns = (uint32_t)(S - s0 < ns_max ? S - s0 : ns_max);
    SegArgs a{};
    a.n = n;
    a.outs = src.outs;
    a.out_len = c.out_len;
    a.fb = c.fb;
    a.verdicts = src.verdicts;
    a.mask = d_mask;
    a.seg = d_dense;
    a.s0 = (uint32_t)s0;
    a.ns = ns;
    a.nonces = src.nonces;
    a.cnt = e->d_segx;
    a.off = e->d_segx + SEG_MAX;
    a.cursor = e->d_segx + 2 * SEG_MAX;
    a.ioff = e->d_segx + 3 * SEG_MAX;
    a.nitems = e->d_segx + 4 * SEG_MAX + 1;
    a.perm = e->d_perm;
    a.L = L;
    a.items = e->d_items;
    a.wmax = (uint32_t)(items_n + ns);
    a.partials = e->d_spart;
    a.aggs = reinterpret_cast<uint4* const*>(e->d_ptrs + s0);
    a.counts = reinterpret_cast<unsigned long long* const*>(e->d_ptrs + S + s0);
    a.checksums = reinterpret_cast<uint32_t* const*>(e->d_ptrs + 2 * S + s0);
    HIPCHK(e, hipMemsetAsync(a.cnt, 0, ns * sizeof(uint32_t), e->stream));
    hipEvent_t ev = nullptr;
    HIPCHK(e, stage_begin(e, &ev));
    HIPCHK(e, launch_accumulate_segmented(c, a, (uint32_t)grid, e->stream));
    HIPCHK(e, stage_end(e, ST_ACC, ev));
  }
  return JX_OK;
}

// Densify host segment ids: ids in first-seen order, dense index per report.
static void densify(const uint32_t* seg, uint64_t n, std::vector<uint32_t>& dense, std::vector<uint32_t>& ids) {
  std::unordered_map<uint32_t, uint32_t> m;
  dense.resize(n);
  ids.clear();
  for (uint64_t i = 0; i < n; i++) {
    auto it = m.find(seg[i]);
    if (it == m.end()) {
      it = m.emplace(seg[i], (uint32_t)ids.size()).first;
      ids.push_back(seg[i]);
    }
    dense[i] = it->second;
  }
}

// The running aggregations named by a caller's segment-id table. A repeated id would make two
// segmented-reduce rows update one aggregation without atomics: refused.
static int32_t segment_targets(jx_engine* e, const uint32_t* ids, uint64_t nids, std::vector<Segment>& out) {
  std::unordered_set<uint32_t> seen;
  out.clear();
  for (uint64_t t = 0; t < nids; t++) {
    if (!seen.insert(ids[t]).second)
      return fail(e, JX_E_INVALID, "segment_ids holds a repeated batch-aggregation id");
    Segment* s = nullptr;
    int32_t rc = get_segment(e, ids[t], &s);
    if (rc) return rc;
    out.push_back(*s);
  }
  return JX_OK;
}

// Accumulate src into targets[d_dense[r]] (d_dense nullable: all into targets[0]). One target takes the
// coalesced select/accumulate path; several upload their pointer table (unless `uploaded`).
static int32_t accumulate_into(jx_engine* e, const AccSrc& src, const uint8_t* d_mask, const uint32_t* d_dense,
                               const std::vector<Segment>& targets, bool uploaded = false) {
  if (src.n == 0 || targets.empty()) return JX_OK;
  if (targets.size() == 1 || !d_dense) return accumulate_one(e, src, d_mask, d_dense, targets[0]);
  Scratch tbl;
  if (!uploaded) {
    int32_t rc = upload_targets(e, targets, tbl);
    if (rc) return rc;
  }
  return accumulate_many(e, src, d_mask, d_dense, targets.size());
}

// Per-call delta aggregations (zeroed): ns contiguous segment states in per-call scratch `d`.
static int32_t delta_targets(jx_engine* e, uint32_t ns, std::vector<Segment>& out, Scratch& d) {
  const size_t agg_b = (size_t)ns * e->cfg.out_len * 16, bytes = agg_b + (size_t)ns * 8 + (size_t)ns * 32;
  int32_t rc = scratch_get(e, bytes, d);
  if (rc) return rc;
  uint8_t* base = d.p();
  HIPCHK(e, hipMemsetAsync(base, 0, bytes, e->stream));
  out.resize(ns);
  for (uint32_t s = 0; s < ns; s++) {
    out[s].agg = (uint4*)base + (size_t)s * e->cfg.out_len;
    out[s].count = (unsigned long long*)(base + agg_b) + s;
    out[s].checksum = (uint32_t*)(base + agg_b + (size_t)ns * 8) + 8 * s;
  }
  return JX_OK;
}

static uint32_t record_bytes(const Cfg& c) { return c.out_len * c.fb + 40u; }

// Reports per launch for an n-report fused call: the fewest launches that fit the staging
// budget (default_chunk), split evenly (multiple of 64) so every launch has the same shape.
// When the chunk is a whole number of K1 rounds (round_reports), launches are full chunks and
// only the last one carries a partial round (1.25M SumVec reports: 4 x 262,144 + 201,424
// instead of 4 x 312,500). Measured on MI355X: K1 time per report is unchanged (its waves do
// not finish in lockstep rounds), the step went 188.4 -> 184.6 ms, within run-to-run noise.
static uint64_t launch_chunk(const jx_engine* e, uint64_t n) {
  if (n <= e->default_chunk) return n;
  if (e->round_reports && e->default_chunk % e->round_reports == 0) return e->default_chunk;
  const uint64_t launches = (n + e->default_chunk - 1) / e->default_chunk;
  const uint64_t per = (n + launches - 1) / launches;
  return (per + 63) / 64 * 64;
}

// ---------------------------------------------------------------------------- pipelines
// A helper launch of the fused path runs K1 (two sponges per lane, two waves per SIMD, VALU), then K3
// (LDS-DMA ring: HBM + limb products) and K4 (HBM): one after the other, every launch's waves are in the
// same phase at the same time (the K1 waves of a round reach their FLP-coefficient tails together, K3 runs
// at a throttled clock beside an idle Keccak pipe). With P pipelines the launches of one call alternate
// over P child engines, each with its own stream and per-call staging from the arena, so different
// launches' phases overlap; only the K4s are ordered (they add into the same aggregation). Measured on
// MI355X with P independent engines (tools/multi_engine_probe.py): SumVec 8x1000/88, 1.25M reports,
// 7.28M (one) -> 7.67M (two) -> 7.79M reports/s (three). Used when a call spans >= 2 launches of one
// segment; not for Count (one tiny kernel) or the multiproof path.
// host: the host-buffer path, whose pageable copies also take turns (3 by default there: SumVec 1.25M
// reports 5.02M -> 6.44M (two) -> 7.12M (three) reports/s including the copies, tools/bench_host_path.py).
static uint32_t pipes_for(const jx_engine* e, uint64_t n, uint64_t chunk, bool many, bool host = false) {
  const Cfg& c = e->cfg;
  if (many || c.algo == ALGO_COUNT || c.algo == ALGO_SUMVEC_F64_MULTIPROOF) return 1;
  const uint64_t launches = (n + chunk - 1) / chunk;
  const uint64_t want = e->npipes ? e->npipes : (host ? 3 : 2);
  return (uint32_t)(launches < want ? launches : want);
}

jx_engine* jxi::new_child(jx_engine* parent) {
  jx_engine* q = new jx_engine();
  q->cfg = parent->cfg;
  q->device = parent->device;
  q->is_pipe = true;
  q->arena = parent->arena;
  q->d_consts = parent->d_consts;
  q->default_chunk = parent->default_chunk;
  q->auto_chunk = parent->auto_chunk;
  q->round_reports = parent->round_reports;
  q->lis_stride = parent->lis_stride;
  if (hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&q->ev_join, hipEventDisableTiming) != hipSuccess) {
    jx_engine_destroy(q);
    return nullptr;
  }
  return q;
}

constexpr uint32_t MAX_PIPES = 4;

// Staging for up to P pipelines: the first one may wait for the arena, the others take what is free
// now (so two calls never wait on each other holding half their pipelines). *got = pipelines staged.
static int32_t pipes_acquire(jx_engine* e, uint32_t P, uint64_t chunk, uint32_t flags, Stage* st, uint32_t* got) {
  *got = 0;
  while (e->pipes.size() < P) {
    jx_engine* q = new_child(e);
    if (!q) return fail(e, JX_E_HIP, "pipelines: stream creation failed");
    e->pipes.push_back(q);
  }
  if (!e->ev_pipe) HIPCHK(e, hipEventCreateWithFlags(&e->ev_pipe, hipEventDisableTiming));
  for (uint32_t k = 0; k < P; k++) {
    jx_engine* q = e->pipes[k];
    q->force_slow = e->force_slow;
    q->k1_split = e->k1_split;
    q->lanes_wg_cap = e->lanes_wg_cap;
    q->timing = e->timing;
    q->acc_chunks = e->acc_chunks;
    int32_t rc = stage_acquire(q, chunk, flags, st[k], k == 0);
    if (rc) {
      if (k == 0) return rc;
      t_err.clear();  // run with the pipelines that fit (retried on the next call)
      break;
    }
    *got = k + 1;
  }
  return JX_OK;
}

// Move the pipelines' kernel timings into the engine's.
static int32_t collect_pipe_timing(jx_engine* e) {
  for (jx_engine* q : e->pipes) {
    int32_t rc = drain_timing(q);
    if (rc) return rc;
    for (int i = 0; i < NST; i++) {
      e->ms[i] += q->ms[i];
      e->launches[i] += q->launches[i];
      q->ms[i] = 0;
      q->launches[i] = 0;
    }
  }
  return JX_OK;
}

// measurement staging for a helper prepare whose outputs go to a batch (Histogram writes its
// measurement share, which is its output share, straight into the batch)
static uint32_t helper_meas_flag(const Cfg& c) { return outs_alias_meas(c) ? 0u : SG_MEAS; }

// ---------------------------------------------------------------------------- C ABI

extern "C" {

int32_t jx_engine_create(const jx_prio3_params* params, const uint8_t verify_key[16], int32_t device,
                         jx_engine** out) {
  return jx_engine_create_ex(params, verify_key, 16, device, out);
}

int32_t jx_engine_create_ex(const jx_prio3_params* params, const uint8_t* verify_key, uint32_t verify_key_len,
                            int32_t device, jx_engine** out) {
  if (!params || !verify_key || !out) return JX_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return JX_E_NODEVICE;
  if (device < 0 || device >= ndev) return JX_E_INVALID;
  jx_engine* e = new jx_engine();
  std::string why;
  int32_t rc = make_cfg(params, verify_key, verify_key_len, e->cfg, why);
  if (rc) {
    t_err = why;
    delete e;
    return rc;
  }
  e->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return JX_E_HIP;
  }
  e->arena = arena_for(device);
  arena_engine_add(e->arena);
  // staged leader input shares (host-buffer leader path, coalesced leader launches): rows padded to 128 B for
  // the instances whose FLP kernels read the measurement share in place, so those reads take whole lines
  e->lis_stride = leader_inplace(e->cfg) ? (e->cfg.lis_bytes + 127u) / 128u * 128u : e->cfg.lis_bytes;
  std::vector<uint4> consts = make_consts(e->cfg);
  // On the engine stream, synchronized on it alone: creating an engine orders nothing with the caller's
  // streams (that is jx_engine_wait_stream's job).
  if (hipMalloc((void**)&e->d_consts, consts.size() * sizeof(uint4)) != hipSuccess ||
      hipMemcpyAsync(e->d_consts, consts.data(), consts.size() * sizeof(uint4), hipMemcpyHostToDevice, e->stream) !=
          hipSuccess ||
      hipStreamSynchronize(e->stream) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_wait, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming) != hipSuccess) {
    jx_engine_destroy(e);
    return JX_E_HIP;
  }
  // Reports per launch of the fused paths: ~48 GiB of staging, enough for several K1 occupancy rounds of
  // the small VDAFs. A VDAF whose reports need megabytes of staging (FixedPointBoundedL2VecSum at
  // length 10000: 2.8 MB) would fill only a few percent of the SIMDs at 48 GiB, and K1 is bound by
  // the per-report sponge latency (15k sequential permutations), so throughput scales with the
  // reports in flight: grow the budget toward one full K1 round, up to 1/3 of the device memory
  // (two roles, e.g. leader and helper, still fit on one MI355X). Staging is checked out of the device
  // arena per call, so this sizes launches, not what an idle engine holds. Debug option 5 overrides it.
  const uint64_t per = per_report_bytes(e->cfg);
  e->round_reports = k1_round_reports(e->cfg, device, 0);
  uint64_t budget = 48ull << 30;
  size_t mem_free = 0, mem_total = 0;
  if (hipMemGetInfo(&mem_free, &mem_total) == hipSuccess && e->round_reports && e->round_reports * per > budget) {
    const uint64_t cap = mem_total / 3;
    budget = e->round_reports * per < cap ? e->round_reports * per : cap;
    if (budget < (48ull << 30)) budget = 48ull << 30;
  }
  uint64_t chunk = budget / per;
  if (chunk > (1ull << 22)) chunk = 1ull << 22;
  chunk = chunk / 256 * 256;
  if (chunk < 256) chunk = 256;
  if (e->round_reports && chunk >= e->round_reports) chunk = chunk / e->round_reports * e->round_reports;
  e->default_chunk = e->auto_chunk = chunk;
  *out = e;
  return JX_OK;
}

void jx_engine_destroy(jx_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  if (e->coal) coalescer_release(e);
  for (jx_engine* p : e->pipes) jx_engine_destroy(p);
  e->pipes.clear();
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (auto& p : e->pending) {
    (void)hipEventDestroy(p.second.first);
    (void)hipEventDestroy(p.second.second);
  }
  e->segs.clear();
  if (e->arena) {
    for (auto& p : e->accq) arena_put(e->arena, p.first.slab, e->stream);  // deferred accumulations: unread
    e->accq.clear();
    for (auto& kv : e->recycle) arena_put(e->arena, kv.second, e->stream);
    e->recycle.clear();
    for (Slab& sl : e->seg_slabs) arena_put(e->arena, sl, e->stream);
    for (auto& kv : e->batches) arena_put(e->arena, kv.second.slab, e->stream);
  }
  e->seg_slabs.clear();
  e->batches.clear();
  if (e->d_consts && !e->is_pipe) (void)hipFree(e->d_consts);
  if (e->ev_pipe) (void)hipEventDestroy(e->ev_pipe);
  if (e->d_err) (void)hipFree(e->d_err);
  for (int k = 0; k < 2; k++) {
    if (e->h_ptrs[k]) (void)hipHostFree(e->h_ptrs[k]);
    if (e->ev_ptrs[k]) (void)hipEventDestroy(e->ev_ptrs[k]);
  }
  if (e->h_acc) (void)hipHostFree(e->h_acc);
  if (e->ev_hacc) (void)hipEventDestroy(e->ev_hacc);
  if (e->ev_flush) (void)hipEventDestroy(e->ev_flush);
  if (e->ev_wait) (void)hipEventDestroy(e->ev_wait);
  if (e->ev_join) (void)hipEventDestroy(e->ev_join);
  if (e->arena) arena_big_forget(e->arena, e);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_side) (void)hipEventDestroy(e->ev_side);
  if (e->side) (void)hipStreamDestroy(e->side);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  if (e->arena && !e->is_pipe) arena_engine_remove(e->arena);
  delete e;
}

int32_t jx_engine_sizes(const jx_engine* e, uint32_t* ps, uint32_t* his, uint32_t* lps, uint32_t* pm,
                        uint32_t* out_len, uint32_t* fb) {
  if (!e) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  if (ps) *ps = c.ps_bytes;
  if (his) *his = c.his_bytes;
  if (lps) *lps = c.lps_bytes;
  if (pm) *pm = c.jr_len ? c.seed : 0;
  if (out_len) *out_len = c.out_len;
  if (fb) *fb = c.fb;
  return JX_OK;
}

// Reserve: warm the device arena with staging for `reports` reports (checked out once, then idle in the
// arena for the next call of any engine on the device).
int32_t jx_engine_set_capacity(jx_engine* e, uint64_t reports) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  Stage st;
  return stage_acquire(e, reports, SG_IN | SG_HIN | SG_MEAS | SG_PREP | SG_RES | SG_ACC, st);
}

// Release batch `id` when a prepare call fails after creating it.
static int32_t drop_on_error(jx_engine* e, uint64_t id, int32_t rc) {
  if (rc) {
    auto it = e->batches.find(id);
    if (it != e->batches.end()) batch_free(e, it);
  }
  return rc;
}

static int32_t copy_out_shares(jx_engine* e, const uint4* outs, uint64_t n, uint8_t* dst) {
  const Cfg& c = e->cfg;
  Scratch tmp;
  int32_t rc = scratch_get(e, n * c.out_len * c.fb, tmp);
  if (rc) return rc;
  HIPCHK(e, launch_transpose_out(c, outs, n, tmp.p(), e->stream));
  HIPCHK(e, hipMemcpyAsync(dst, tmp.p(), n * c.out_len * c.fb, hipMemcpyDeviceToHost, e->stream));
  return JX_OK;
}

static int32_t helper_prep_batch_locked(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps,
                                        const uint8_t* his, const uint8_t* lps, uint8_t* out_msgs, uint8_t* out_verdicts,
                                        uint8_t* out_shares, Batch* B) {
  const Cfg& c = e->cfg;
  Stage st;
  int32_t rc = stage_acquire(e, n, SG_IN | SG_HIN | helper_meas_flag(c) | SG_PREP, st);
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(B->nonces, nonces, n * 16, hipMemcpyHostToDevice, e->stream));
  if (c.ps_bytes) HIPCHK(e, hipMemcpyAsync(e->d_ps, ps, n * c.ps_bytes, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(e->d_his, his, n * c.his_bytes, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(e->d_lps, lps, n * c.lps_bytes, hipMemcpyHostToDevice, e->stream));
  rc = prep_core(e, n, B->nonces, e->d_ps, e->d_his, e->d_lps, B->verdicts, B->msgs, B->outs);
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(out_verdicts, B->verdicts, n, hipMemcpyDeviceToHost, e->stream));
  if (out_msgs && c.jr_len)
    HIPCHK(e, hipMemcpyAsync(out_msgs, B->msgs, n * c.seed, hipMemcpyDeviceToHost, e->stream));
  if (out_shares) {
    rc = copy_out_shares(e, B->outs, n, out_shares);
    if (rc) return rc;
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return drain_timing(e);
}

// Coalesced prepares take jobs up to a quarter of a launch (larger ones fill the device by themselves) that fit
// one of the coalescer's lanes for their role (a leader's explicit input shares can be MBs per report); the
// rest take the direct path.
static bool coalescible(const jx_engine* e, uint64_t n, bool leader = false, bool encrypted = false,
                        uint64_t ct_bytes = 0) {
  return e->coalesce && n > 0 && n <= e->default_chunk / 4 && coalescer_accepts(e, leader, n, encrypted, ct_bytes);
}

int32_t jx_helper_prep_batch(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* public_shares,
                             const uint8_t* helper_input_shares, const uint8_t* leader_prep_shares,
                             uint8_t* out_prep_msgs, uint8_t* out_verdicts, uint8_t* out_output_shares,
                             uint64_t* out_batch_id) {
  if (out_batch_id) *out_batch_id = 0;
  if (!e || (n && (!nonces || !helper_input_shares || !leader_prep_shares || !out_verdicts))) return JX_E_INVALID;
  if (n && e->cfg.ps_bytes && !public_shares) return JX_E_INVALID;
  if (!out_output_shares && coalescible(e, n)) {
    t_err.clear();
    return coalesced_helper_prep(e, n, nonces, public_shares, helper_input_shares, leader_prep_shares, out_prep_msgs,
                                 out_verdicts, out_batch_id);
  }
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  uint64_t id = 0;
  Batch* B = nullptr;
  int32_t rc = batch_new(e, n, false, &id, &B);
  if (rc) return rc;
  if (n) {
    rc = helper_prep_batch_locked(e, n, nonces, public_shares, helper_input_shares, leader_prep_shares, out_prep_msgs,
                                  out_verdicts, out_output_shares, B);
    if (rc) return drop_on_error(e, id, rc);
  }
  if (out_batch_id) *out_batch_id = id;
  return JX_OK;
}

int32_t jx_helper_prep_encrypted_batch(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint64_t* times,
                                       const uint8_t* public_shares, const uint8_t task_id[32],
                                       jx_hpke* const* keypairs, uint32_t nkeypairs, const uint8_t* key_index,
                                       const uint8_t* encs, const uint8_t* payloads, const uint64_t* payload_offsets,
                                       uint32_t flags, const uint8_t* leader_prep_shares, uint8_t* out_prep_msgs,
                                       uint8_t* out_verdicts, uint8_t* out_open_status, uint64_t* out_batch_id) {
  if (out_batch_id) *out_batch_id = 0;
  if (!e || (n && (!nonces || !times || !task_id || !key_index || !encs || !payload_offsets || !leader_prep_shares ||
                   !out_verdicts)))
    return JX_E_INVALID;
  const Cfg& c = e->cfg;
  if (n && c.ps_bytes && !public_shares) return JX_E_INVALID;
  if (nkeypairs > JX_ENC_MAX_KEYPAIRS || (nkeypairs && !keypairs) || (flags & ~JX_ENC_REQUIRE_TASKPROV))
    return fail(e, JX_E_INVALID, "encrypted prepare: at most JX_ENC_MAX_KEYPAIRS keypairs, flags JX_ENC_*");
  for (uint32_t k = 0; k < nkeypairs; k++)
    if (!keypairs[k] || hpke_device(keypairs[k]) != e->device)
      return fail(e, JX_E_INVALID, "encrypted prepare: every keypair must be an HPKE context on the engine's device");
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t k0 = key_index[2 * i], k1 = key_index[2 * i + 1];
    if ((k0 >= nkeypairs && k0 != JX_KEY_NONE && k0 != JX_KEY_MALFORMED) || (k1 >= nkeypairs && k1 != JX_KEY_NONE) ||
        payload_offsets[i + 1] < payload_offsets[i] || payload_offsets[i + 1] - payload_offsets[i] > 0xFFFFFFFFull)
      return fail(e, JX_E_INVALID, "encrypted prepare: key_index out of range or payload offsets decreasing");
  }
  if (n && payload_offsets[n] > payload_offsets[0] && !payloads) return JX_E_INVALID;
  EncJob job;
  job.times = times;
  job.task_id = task_id;
  job.keypairs = keypairs;
  job.nkeys = nkeypairs;
  job.key_index = key_index;
  job.encs = encs;
  job.payloads = payloads;
  job.payload_offsets = payload_offsets;
  job.flags = flags;
  const uint64_t ct = n ? job.ct_bytes(n) : 0;
  if (coalescible(e, n, false, true, ct)) {
    t_err.clear();
    return coalesced_helper_prep(e, n, nonces, public_shares, nullptr, leader_prep_shares, out_prep_msgs, out_verdicts,
                                 out_batch_id, &job, out_open_status);
  }
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  uint64_t id = 0;
  Batch* B = nullptr;
  int32_t rc = batch_new(e, n, false, &id, &B);
  if (rc) return rc;
  if (n) {
    auto run = [&]() -> int32_t {
      // the job's rows in pageable host memory, uploaded with its inputs; the key table is the job's keypairs
      std::vector<EncRow> rows(n);
      uint8_t key_map[JX_ENC_MAX_KEYPAIRS];
      std::vector<HpkeKeyRow> keys(nkeypairs ? nkeypairs : 1);
      for (uint32_t k = 0; k < nkeypairs; k++) {
        key_map[k] = (uint8_t)k;
        hpke_key_row(keypairs[k], &keys[k]);
      }
      fill_enc_rows(job, n, rows.data(), 0, key_map);
      e->enc_ct_bytes = ct ? ct : 1;
      Stage st;
      int32_t r = stage_acquire(e, n, SG_IN | SG_HIN | SG_ENC | helper_meas_flag(c) | SG_PREP, st);
      if (r) return r;
      HIPCHK(e, hipMemcpyAsync(B->nonces, nonces, n * 16, hipMemcpyHostToDevice, e->stream));
      if (c.ps_bytes) HIPCHK(e, hipMemcpyAsync(e->d_ps, public_shares, n * c.ps_bytes, hipMemcpyHostToDevice, e->stream));
      HIPCHK(e, hipMemcpyAsync(e->d_lps, leader_prep_shares, n * c.lps_bytes, hipMemcpyHostToDevice, e->stream));
      HIPCHK(e, hipMemcpyAsync(e->d_encrows, rows.data(), n * sizeof(EncRow), hipMemcpyHostToDevice, e->stream));
      if (ct) HIPCHK(e, hipMemcpyAsync(e->d_ct, payloads + payload_offsets[0], ct, hipMemcpyHostToDevice, e->stream));
      if (nkeypairs)
        HIPCHK(e, hipMemcpyAsync(e->d_keys, keys.data(), nkeypairs * sizeof(HpkeKeyRow), hipMemcpyHostToDevice, e->stream));
      HpkeRowsArgs ha{n, e->d_encrows, e->d_ct, e->d_pt, e->d_keys, nkeypairs, B->nonces, e->d_ps, c.ps_bytes,
                      e->d_his, c.his_bytes, e->d_status};
      HIPCHK(e, launch_hpke_rows(ha, e->stream));
      r = prep_core(e, n, B->nonces, e->d_ps, e->d_his, e->d_lps, B->verdicts, B->msgs, B->outs);
      if (r) return r;
      HIPCHK(e, launch_open_mask(e->d_status, B->verdicts, n, e->stream));
      HIPCHK(e, hipMemcpyAsync(out_verdicts, B->verdicts, n, hipMemcpyDeviceToHost, e->stream));
      if (out_prep_msgs && c.jr_len)
        HIPCHK(e, hipMemcpyAsync(out_prep_msgs, B->msgs, n * c.seed, hipMemcpyDeviceToHost, e->stream));
      if (out_open_status) HIPCHK(e, hipMemcpyAsync(out_open_status, e->d_status, n, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));  // the pageable rows and the caller's outputs
      return drain_timing(e);
    };
    rc = run();
    if (rc) return drop_on_error(e, id, rc);
  }
  if (out_batch_id) *out_batch_id = id;
  return JX_OK;
}

int32_t jx_engine_batch_id(const jx_engine* e, uint64_t* batch_id) {
  if (!e || !batch_id) return JX_E_INVALID;
  LOCK(const_cast<jx_engine*>(e));
  auto it = e->batches.find(e->last_batch);
  *batch_id = it != e->batches.end() && !__atomic_load_n(&it->second.pending, __ATOMIC_ACQUIRE) ? e->last_batch.load() : 0;
  return JX_OK;
}

int32_t jx_engine_batches(const jx_engine* e, uint64_t* resident, uint64_t* device_bytes) {
  if (!e) return JX_E_INVALID;
  LOCK(const_cast<jx_engine*>(e));
  uint64_t bytes = 0;
  for (auto& kv : e->batches) bytes += kv.second.slab.bytes;
  if (resident) *resident = e->batches.size();
  if (device_bytes) *device_bytes = bytes;
  return JX_OK;
}

int32_t jx_engine_memory(const jx_engine* e, jx_memory_stats* out) {
  if (!e || !out) return JX_E_INVALID;
  memset(out, 0, sizeof *out);
  {
    LOCK(const_cast<jx_engine*>(e));
    for (auto& kv : e->batches) out->batch_bytes += kv.second.slab.bytes;
    out->resident_batches = e->batches.size();
    out->last_pipelines = e->last_pipes;
  }
  Arena* A = e->arena;
  {
    std::lock_guard<std::mutex> lk(A->mu);
    out->arena_budget = A->budget;
    out->arena_allocated = A->allocated;
    out->arena_in_use = A->in_use;
    out->arena_peak = A->peak;
    out->arena_allocs = A->allocs;
    out->arena_reuses = A->reuses;
    out->arena_waits = A->waits;
    out->arena_engines = A->engines;
  }
  uint64_t cs[16] = {0};
  coalescer_stats(e, cs);
  out->coalesce_pinned_bytes = cs[9];
  out->coalesced_helper_launches = cs[10];
  out->coalesced_helper_jobs = cs[11];
  out->coalesced_leader_launches = cs[12];
  out->coalesced_leader_jobs = cs[13];
  out->coalesced_encrypted_jobs = cs[14];
  out->coalesced_launches = cs[0];
  out->coalesced_jobs = cs[1];
  out->coalesced_reports = cs[2];
  out->coalesce_window_us = cs[3];
  out->coalesce_gather_us = cs[5];
  out->coalesce_copy_us = cs[6];
  out->coalesce_enqueue_us = cs[7];
  out->coalesce_device_us = cs[8];
  {
    std::lock_guard<std::mutex> lk(A->mu);
    out->arena_cross_stream_waits = A->cross_waits;
    out->arena_frees = A->frees;
  }
  return JX_OK;
}

int32_t jx_batch_release(jx_engine* e, uint64_t batch_id) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  auto it = e->batches.find(batch_id);
  if (batch_id == 0 || it == e->batches.end() || __atomic_load_n(&it->second.pending, __ATOMIC_ACQUIRE))
    return fail(e, JX_E_STATE, "release: batch id names no resident prepared batch");
  HIPCHK(e, hipSetDevice(e->device));
  batch_free(e, it);
  return JX_OK;
}

int32_t jx_engine_leader_sizes(const jx_engine* e, uint32_t* leader_input_share) {
  if (!e) return JX_E_INVALID;
  if (leader_input_share) *leader_input_share = e->cfg.lis_bytes;
  return JX_OK;
}

int32_t jx_leader_prep_init_batch(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* public_shares,
                                  const uint8_t* leader_input_shares, uint8_t* out_prep_shares,
                                  uint8_t* out_verdicts, uint64_t* out_batch_id) {
  if (out_batch_id) *out_batch_id = 0;
  if (!e || (n && (!nonces || !leader_input_shares || !out_prep_shares || !out_verdicts))) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  if (n && c.ps_bytes && !public_shares) return JX_E_INVALID;
  if (coalescible(e, n, true)) {
    t_err.clear();
    return coalesced_leader_init(e, n, nonces, public_shares, leader_input_shares, out_prep_shares, out_verdicts,
                                 out_batch_id);
  }
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  uint64_t id = 0;
  Batch* B = nullptr;
  int32_t rc = batch_new(e, n, true, &id, &B);
  if (rc) return rc;
  if (n) {
    auto run = [&]() -> int32_t {
      Stage st;
      int32_t r = stage_acquire(e, n, SG_IN | SG_LEAD | SG_PREP | (use_inplace(e) ? 0u : SG_MEAS), st);
      if (r) return r;
      HIPCHK(e, hipMemcpyAsync(B->nonces, nonces, n * 16, hipMemcpyHostToDevice, e->stream));
      if (c.ps_bytes)
        HIPCHK(e, hipMemcpyAsync(e->d_ps, public_shares, n * c.ps_bytes, hipMemcpyHostToDevice, e->stream));
      if (e->lis_stride == c.lis_bytes)
        HIPCHK(e, hipMemcpyAsync(e->d_lis, leader_input_shares, n * c.lis_bytes, hipMemcpyHostToDevice, e->stream));
      else  // padded rows (aligned in-place reads of the measurement share)
        HIPCHK(e, hipMemcpy2DAsync(e->d_lis, e->lis_stride, leader_input_shares, c.lis_bytes, c.lis_bytes, n,
                                   hipMemcpyHostToDevice, e->stream));
      r = prep_core(e, n, B->nonces, e->d_ps, nullptr, nullptr, B->verdicts, B->msgs, B->outs, e->d_lis, e->d_lps_out,
                    e->lis_stride);
      if (r) return r;
      HIPCHK(e, hipMemcpyAsync(out_verdicts, B->verdicts, n, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipMemcpyAsync(out_prep_shares, e->d_lps_out, n * c.lps_bytes, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
      return drain_timing(e);
    };
    rc = run();
    if (rc) return drop_on_error(e, id, rc);
  }
  if (out_batch_id) *out_batch_id = id;
  return JX_OK;
}

int32_t jx_leader_prep_init_device_ex(jx_engine* e, uint64_t n, const void* d_nonces, const void* d_public_shares,
                                      const void* d_leader_input_shares, uint64_t lis_stride, void* d_out_prep_shares,
                                      void* d_out_verdicts, uint64_t* out_batch_id) {
  if (!out_batch_id) return JX_E_INVALID;
  *out_batch_id = 0;
  if (!e || (n && (!d_nonces || !d_leader_input_shares || !d_out_prep_shares))) return JX_E_INVALID;
  LOCK(e);
  const Cfg& c = e->cfg;
  if (n && c.ps_bytes && !d_public_shares) return JX_E_INVALID;
  if (lis_stride == 0) lis_stride = c.lis_bytes;
  if (lis_stride < c.lis_bytes || (lis_stride & 15u))
    return fail(e, JX_E_INVALID, "leader init: the row stride must be >= the leader input share and a multiple of 16");
  // the in-place FLP kernels read the measurement share in 16-byte vectors (header contract)
  if (n && use_inplace(e) && (reinterpret_cast<uintptr_t>(d_leader_input_shares) & 15u))
    return fail(e, JX_E_INVALID, "leader init: d_leader_input_shares must be 16-byte aligned");
  HIPCHK(e, hipSetDevice(e->device));
  uint64_t id = 0;
  Batch* B = nullptr;
  int32_t rc = batch_new(e, n, true, &id, &B);
  if (rc) return rc;
  if (n) {
    auto run = [&]() -> int32_t {
      Stage st;
      int32_t r = stage_acquire(e, n, SG_PREP | (use_inplace(e) ? 0u : SG_MEAS), st);
      if (r) return r;
      HIPCHK(e, hipMemcpyAsync(B->nonces, d_nonces, n * 16, hipMemcpyDeviceToDevice, e->stream));
      r = prep_core(e, n, B->nonces, (const uint8_t*)d_public_shares, nullptr, nullptr, B->verdicts, B->msgs, B->outs,
                    (const uint8_t*)d_leader_input_shares, (uint8_t*)d_out_prep_shares, lis_stride);
      if (r) return r;
      if (d_out_verdicts) HIPCHK(e, hipMemcpyAsync(d_out_verdicts, B->verdicts, n, hipMemcpyDeviceToDevice, e->stream));
      return JX_OK;
    };
    rc = run();
    if (rc) return drop_on_error(e, id, rc);
  }
  *out_batch_id = id;
  return JX_OK;
}

int32_t jx_leader_prep_init_device(jx_engine* e, uint64_t n, const void* d_nonces, const void* d_public_shares,
                                   const void* d_leader_input_shares, void* d_out_prep_shares, void* d_out_verdicts,
                                   uint64_t* out_batch_id) {
  return jx_leader_prep_init_device_ex(e, n, d_nonces, d_public_shares, d_leader_input_shares, 0, d_out_prep_shares,
                                       d_out_verdicts, out_batch_id);
}

static int32_t leader_batch(jx_engine* e, uint64_t batch_id, uint64_t n, Batch** B) {
  int32_t rc = find_batch(e, batch_id, n, "leader finish", B);
  if (rc) return rc;
  if (!(*B)->leader) return fail(e, JX_E_STATE, "leader finish: the batch is a helper batch");
  if ((*B)->finished) return fail(e, JX_E_STATE, "leader finish: the batch was already finished");
  return JX_OK;
}

int32_t jx_leader_prep_finish_batch(jx_engine* e, uint64_t batch_id, uint64_t n, const uint8_t* prep_msgs,
                                    uint8_t* out_verdicts, uint8_t* out_output_shares) {
  if (!e || (n && !out_verdicts)) return JX_E_INVALID;
  LOCK(e);
  const Cfg& c = e->cfg;
  Batch* B = nullptr;
  int32_t rc = leader_batch(e, batch_id, n, &B);
  if (rc) return rc;
  if (n && c.jr_len && !prep_msgs) return JX_E_INVALID;
  if (n == 0) {
    B->finished = true;
    return JX_OK;
  }
  HIPCHK(e, hipSetDevice(e->device));
  Stage st;
  if (c.jr_len) {
    rc = stage_acquire(e, n, SG_LMSG, st);
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(e->d_in_msgs, prep_msgs, n * c.seed, hipMemcpyHostToDevice, e->stream));
    Bufs b{};
    b.n = n;
    b.verdicts = B->verdicts;
    b.msgs = B->msgs;
    HIPCHK(e, launch_leader_finish(c, b, e->d_in_msgs, nullptr, e->stream));
  }
  // finished once prepare_next is queued: a failure above leaves the batch finishable (or releasable)
  B->finished = true;
  HIPCHK(e, hipMemcpyAsync(out_verdicts, B->verdicts, n, hipMemcpyDeviceToHost, e->stream));
  if (out_output_shares) {
    rc = copy_out_shares(e, B->outs, n, out_output_shares);
    if (rc) return rc;
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return JX_OK;
}

int32_t jx_leader_prep_finish_device(jx_engine* e, uint64_t batch_id, uint64_t n, const void* d_prep_msgs,
                                     const void* d_peer_verdicts, void* d_out_verdicts) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  const Cfg& c = e->cfg;
  Batch* B = nullptr;
  int32_t rc = leader_batch(e, batch_id, n, &B);
  if (rc) return rc;
  if (n && c.jr_len && !d_prep_msgs) return JX_E_INVALID;
  if (n == 0) {
    B->finished = true;
    return JX_OK;
  }
  HIPCHK(e, hipSetDevice(e->device));
  Bufs b{};
  b.n = n;
  b.verdicts = B->verdicts;
  b.msgs = B->msgs;
  HIPCHK(e, launch_leader_finish(c, b, (const uint8_t*)d_prep_msgs, (const uint8_t*)d_peer_verdicts, e->stream));
  B->finished = true;
  if (d_out_verdicts) HIPCHK(e, hipMemcpyAsync(d_out_verdicts, B->verdicts, n, hipMemcpyDeviceToDevice, e->stream));
  return JX_OK;
}

// A batch ready to accumulate: helper batches at once, leader batches after prepare_next.
static int32_t ready_batch(jx_engine* e, uint64_t batch_id, uint64_t n, const char* what, Batch** B) {
  int32_t rc = find_batch(e, batch_id, n, what, B);
  if (rc) return rc;
  if ((*B)->leader && !(*B)->finished)
    return fail(e, JX_E_STATE, std::string(what) + ": leader batch not finished (jx_leader_prep_finish_*)");
  return JX_OK;
}

// Upload small host arrays through the engine's pinned buffer (no host wait for the call's own work: the
// buffer is rewritten only after the upload that last read it has completed).
static int32_t upload_small(jx_engine* e, const std::vector<std::pair<const void*, size_t>>& src,
                            const std::vector<void*>& dst) {
  size_t total = 0;
  for (auto& s : src) total += align256(s.second);
  if (!e->ev_hacc) HIPCHK(e, hipEventCreateWithFlags(&e->ev_hacc, hipEventDisableTiming));
  else HIPCHK(e, hipEventSynchronize(e->ev_hacc));
  if (e->h_acc_cap < total) {
    if (e->h_acc) (void)hipHostFree(e->h_acc);
    e->h_acc = nullptr;
    e->h_acc_cap = 0;
    HIPCHK(e, hipHostMalloc((void**)&e->h_acc, total, hipHostMallocDefault));
    e->h_acc_cap = total;
  }
  size_t off = 0;
  for (size_t i = 0; i < src.size(); i++) {
    memcpy(e->h_acc + off, src[i].first, src[i].second);
    HIPCHK(e, hipMemcpyAsync(dst[i], e->h_acc + off, src[i].second, hipMemcpyHostToDevice, e->stream));
    off += align256(src[i].second);
  }
  HIPCHK(e, hipEventRecord(e->ev_hacc, e->stream));
  return JX_OK;
}

int32_t jx_accumulate(jx_engine* e, uint64_t batch_id, uint64_t n, const uint8_t* accept_mask,
                      const uint32_t* segment) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  Batch* B = nullptr;
  int32_t rc = ready_batch(e, batch_id, n, "accumulate", &B);
  if (rc) return rc;
  HIPCHK(e, hipSetDevice(e->device));
  // one aggregation, every finished report, a job-sized batch: deferred (flush_acc)
  bool one_seg = true;
  for (uint64_t i = 1; segment && i < n && one_seg; i++) one_seg = segment[i] == segment[0];
  if (e->acc_defer && n > 0 && n <= ACC_SMALL && !accept_mask && one_seg) {
    const uint32_t sid = segment ? segment[0] : 0;
    Segment* s = nullptr;
    rc = get_segment(e, sid, &s);  // creates it now (its memset is queued before any later flush)
    if (rc) return rc;
    auto it = e->batches.find(batch_id);
    e->accq.emplace_back(it->second, sid);
    e->accq_reports += n;
    e->acc_deferred++;
    if (e->last_batch == it->first) e->last_batch = 0;
    e->batches.erase(it);  // a batch is accumulated at most once
    if (e->accq.size() >= ACC_MULTI_MAX || e->accq_reports >= kAccQReports) return flush_acc(e);
    return JX_OK;
  }
  auto run = [&]() -> int32_t {
    if (n == 0) return JX_OK;
    Stage st;
    // mask / index scratch and the accumulate partials (a small unmasked batch needs neither)
    int32_t r = accept_mask || segment || n > ACC_SMALL ? stage_acquire(e, n, SG_ACC, st) : JX_OK;
    if (r) return r;
    std::vector<uint32_t> ids{0};
    std::vector<std::pair<const void*, size_t>> src;
    std::vector<void*> dst;
    const uint8_t* dm = nullptr;
    const uint32_t* ds = nullptr;
    if (accept_mask) {
      src.push_back({accept_mask, n});
      dst.push_back(e->d_mask);
      dm = e->d_mask;
    }
    if (segment) {
      densify(segment, n, e->h_dense, ids);
      if (ids.size() > 1) {
        src.push_back({e->h_dense.data(), n * 4});
        dst.push_back(e->d_seg);
        ds = e->d_seg;
      }
    }
    if (!src.empty()) {
      r = upload_small(e, src, dst);
      if (r) return r;
    }
    std::vector<Segment> targets;
    r = segment_targets(e, ids.data(), ids.size(), targets);
    if (r) return r;
    r = accumulate_into(e, batch_src(*B), dm, ds, targets);
    if (r) return r;
    return drain_timing(e);
  };
  rc = run();
  if (rc) return rc;
  batch_free(e, e->batches.find(batch_id));  // a batch is accumulated at most once
  return JX_OK;
}

int32_t jx_accumulate_device(jx_engine* e, uint64_t batch_id, uint64_t n, const void* d_accept_mask,
                             const void* d_segment, const uint32_t* segment_ids, uint32_t nsegments) {
  if (!e || !segment_ids || nsegments == 0) return JX_E_INVALID;
  LOCK(e);
  Batch* B = nullptr;
  int32_t rc = ready_batch(e, batch_id, n, "accumulate", &B);
  if (rc) return rc;
  HIPCHK(e, hipSetDevice(e->device));
  if (n) {
    Stage st;
    rc = stage_acquire(e, n, SG_ACC, st);  // the accumulate partials
    if (rc) return rc;
    std::vector<Segment> targets;
    rc = segment_targets(e, segment_ids, nsegments, targets);
    if (rc) return rc;
    rc = accumulate_into(e, batch_src(*B), (const uint8_t*)d_accept_mask, (const uint32_t*)d_segment, targets);
    if (rc) return rc;
  }
  batch_free(e, e->batches.find(batch_id));
  return JX_OK;
}

// Deltas: accumulate a batch into zeroed per-call aggregations and export them as records. Pure with
// respect to engine state (the batch stays resident; the running aggregations are not touched).
static int32_t batch_records(jx_engine* e, Batch* B, const uint8_t* d_mask, const uint32_t* d_index, uint32_t ns,
                             uint8_t* d_out) {
  std::vector<Segment> targets;
  Scratch deltas;
  int32_t rc = delta_targets(e, ns, targets, deltas);
  if (rc) return rc;
  rc = accumulate_into(e, batch_src(*B), d_mask, d_index, targets);
  if (rc) return rc;
  HIPCHK(e, launch_record_export(e->cfg, targets[0].agg, targets[0].count, targets[0].checksum, d_out, e->stream, ns));
  return JX_OK;
}

int32_t jx_batch_aggregate_records(jx_engine* e, uint64_t batch_id, uint64_t n, const uint8_t* accept_mask,
                                   const uint32_t* segment_index, uint32_t nsegments, uint8_t* out_records) {
  if (!e || !out_records || nsegments == 0) return JX_E_INVALID;
  LOCK(e);
  Batch* B = nullptr;
  int32_t rc = ready_batch(e, batch_id, n, "aggregate records", &B);
  if (rc) return rc;
  HIPCHK(e, hipSetDevice(e->device));
  const uint64_t rb = record_bytes(e->cfg);
  Stage st;
  rc = stage_acquire(e, n ? n : 1, SG_ACC, st);  // mask / index scratch and the accumulate partials
  if (rc) return rc;
  const uint8_t* dm = nullptr;
  const uint32_t* di = nullptr;
  if (n && accept_mask) {
    HIPCHK(e, hipMemcpyAsync(e->d_mask, accept_mask, n, hipMemcpyHostToDevice, e->stream));
    dm = e->d_mask;
  }
  if (n && segment_index) {
    HIPCHK(e, hipMemcpyAsync(e->d_seg, segment_index, n * 4, hipMemcpyHostToDevice, e->stream));
    di = e->d_seg;
  }
  Scratch rec;
  rc = scratch_get(e, rb * nsegments, rec);
  if (rc) return rc;
  rc = batch_records(e, B, dm, di, nsegments, rec.p());
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(out_records, rec.p(), rb * nsegments, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return drain_timing(e);
}

int32_t jx_batch_aggregate_records_device(jx_engine* e, uint64_t batch_id, uint64_t n, const void* d_accept_mask,
                                          const void* d_segment_index, uint32_t nsegments, void* d_out_records) {
  if (!e || !d_out_records || nsegments == 0) return JX_E_INVALID;
  LOCK(e);
  Batch* B = nullptr;
  int32_t rc = ready_batch(e, batch_id, n, "aggregate records", &B);
  if (rc) return rc;
  HIPCHK(e, hipSetDevice(e->device));
  Stage st;
  rc = stage_acquire(e, n ? n : 1, SG_ACC, st);  // the accumulate partials
  if (rc) return rc;
  return batch_records(e, B, (const uint8_t*)d_accept_mask, (const uint32_t*)d_segment_index, nsegments,
                       (uint8_t*)d_out_records);
}

int32_t jx_helper_prep_aggregate(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* public_shares,
                                 const uint8_t* helper_input_shares, const uint8_t* leader_prep_shares,
                                 uint32_t segment, uint8_t* out_prep_msgs, uint8_t* out_verdicts) {
  if (!e || !nonces || !helper_input_shares || !leader_prep_shares) return JX_E_INVALID;
  LOCK(e);
  const Cfg& c = e->cfg;
  if (c.ps_bytes && !public_shares) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  const uint64_t chunk = launch_chunk(e, n);
  Segment* seg = nullptr;
  int32_t rc = get_segment(e, segment, &seg);
  if (rc) return rc;
  const std::vector<Segment> targets{*seg};
  const uint32_t want = pipes_for(e, n, chunk, false, true);
  Stage pst[MAX_PIPES];
  uint32_t P = 0;
  if (want > 1) {
    rc = pipes_acquire(e, want, chunk, SG_IN | SG_HIN | SG_MEAS | SG_PREP | SG_ACC, pst, &P);
    if (rc) return rc;
  }
  e->last_pipes = P > 1 ? P : 1;
  if (P > 1) {
    // the pipelines (see jx_helper_prep_aggregate_device): launch i's host-to-device copies (pageable: the
    // host thread stages them) go out while the other pipeline's kernels run; the verdicts and prep
    // messages collect in an engine buffer and come back once, after the join
    const uint64_t ob = n + (c.jr_len ? n * c.seed : 0);
    Scratch hout;  // per call, from the arena (handed back after the copies below are queued)
    rc = scratch_get(e, ob, hout);
    if (rc) return rc;
    uint8_t* dv = hout.p();
    uint8_t* dm = hout.p() + n;
    HIPCHK(e, hipEventRecord(e->ev_pipe, e->stream));
    for (uint32_t k = 0; k < P; k++) HIPCHK(e, hipStreamWaitEvent(e->pipes[k]->stream, e->ev_pipe, 0));
    auto run = [&]() -> int32_t {
      uint64_t i = 0;
      for (uint64_t off = 0; off < n; off += chunk, i++) {
        jx_engine* q = e->pipes[i % P];
        const uint64_t m = (n - off) < chunk ? (n - off) : chunk;
        HIPCHK(e, hipMemcpyAsync(q->d_nonces, nonces + off * 16, m * 16, hipMemcpyHostToDevice, q->stream));
        if (c.ps_bytes)
          HIPCHK(e, hipMemcpyAsync(q->d_ps, public_shares + off * c.ps_bytes, m * c.ps_bytes, hipMemcpyHostToDevice,
                                   q->stream));
        HIPCHK(e, hipMemcpyAsync(q->d_his, helper_input_shares + off * c.his_bytes, m * c.his_bytes,
                                 hipMemcpyHostToDevice, q->stream));
        HIPCHK(e, hipMemcpyAsync(q->d_lps, leader_prep_shares + off * c.lps_bytes, m * c.lps_bytes,
                                 hipMemcpyHostToDevice, q->stream));
        int32_t r = prep_core(q, m, q->d_nonces, q->d_ps, q->d_his, q->d_lps, dv + off, dm + off * c.seed,
                              staging_outs(q));
        if (r) return r;
        if (i > 0) HIPCHK(e, hipStreamWaitEvent(q->stream, e->ev_pipe, 0));  // the previous launch's K4
        r = accumulate_into(q, AccSrc{m, staging_outs(q), dv + off, q->d_nonces}, nullptr, nullptr, targets);
        if (r) return r;
        HIPCHK(e, hipEventRecord(e->ev_pipe, q->stream));
      }
      return JX_OK;
    };
    rc = run();
    for (uint32_t k = 0; k < P; k++) {
      HIPCHK(e, hipEventRecord(e->pipes[k]->ev_join, e->pipes[k]->stream));
      HIPCHK(e, hipStreamWaitEvent(e->stream, e->pipes[k]->ev_join, 0));
    }
    if (rc) return rc;
    if (out_verdicts) HIPCHK(e, hipMemcpyAsync(out_verdicts, dv, n, hipMemcpyDeviceToHost, e->stream));
    if (out_prep_msgs && c.jr_len)
      HIPCHK(e, hipMemcpyAsync(out_prep_msgs, dm, n * c.seed, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return JX_OK;
  }
  if (P == 1) pst[0].release();  // one pipeline's staging only: run on the engine stream
  Stage st;
  rc = stage_acquire(e, chunk, SG_IN | SG_HIN | SG_MEAS | SG_PREP | SG_RES | SG_ACC, st);
  if (rc) return rc;
  for (uint64_t off = 0; off < n; off += chunk) {
    const uint64_t m = (n - off) < chunk ? (n - off) : chunk;
    HIPCHK(e, hipMemcpyAsync(e->d_nonces, nonces + off * 16, m * 16, hipMemcpyHostToDevice, e->stream));
    if (c.ps_bytes)
      HIPCHK(e, hipMemcpyAsync(e->d_ps, public_shares + off * c.ps_bytes, m * c.ps_bytes, hipMemcpyHostToDevice,
                               e->stream));
    HIPCHK(e, hipMemcpyAsync(e->d_his, helper_input_shares + off * c.his_bytes, m * c.his_bytes,
                             hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->d_lps, leader_prep_shares + off * c.lps_bytes, m * c.lps_bytes,
                             hipMemcpyHostToDevice, e->stream));
    rc = prep_core(e, m, e->d_nonces, e->d_ps, e->d_his, e->d_lps, e->d_verdicts, e->d_msgs, staging_outs(e));
    if (rc) return rc;
    rc = accumulate_into(e, AccSrc{m, staging_outs(e), e->d_verdicts, e->d_nonces}, nullptr, nullptr, targets);
    if (rc) return rc;
    if (out_verdicts)
      HIPCHK(e, hipMemcpyAsync(out_verdicts + off, e->d_verdicts, m, hipMemcpyDeviceToHost, e->stream));
    if (out_prep_msgs && c.jr_len)
      HIPCHK(e, hipMemcpyAsync(out_prep_msgs + off * c.seed, e->d_msgs, m * c.seed, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  return drain_timing(e);
}

int32_t jx_helper_prep_aggregate_device(jx_engine* e, uint64_t n, const void* d_nonces, const void* d_ps,
                                        const void* d_his, const void* d_lps, const void* d_segment,
                                        const uint32_t* segment_ids, uint32_t nsegments, void* d_out_prep_msgs,
                                        void* d_out_verdicts) {
  if (!e || !d_nonces || !d_his || !d_lps || !segment_ids || nsegments == 0) return JX_E_INVALID;
  LOCK(e);
  const Cfg& c = e->cfg;
  if (c.ps_bytes && !d_ps) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  const uint64_t chunk = launch_chunk(e, n);
  std::vector<Segment> targets;
  int32_t rc = segment_targets(e, segment_ids, nsegments, targets);
  if (rc) return rc;
  const uint8_t *N = (const uint8_t*)d_nonces, *PS = (const uint8_t*)d_ps, *H = (const uint8_t*)d_his,
                *L = (const uint8_t*)d_lps;
  const uint32_t* SG = (const uint32_t*)d_segment;
  const bool many = SG && targets.size() > 1;
  const uint32_t want = pipes_for(e, n, chunk, many);
  Stage pst[MAX_PIPES];
  uint32_t P = 0;
  if (want > 1) {
    rc = pipes_acquire(e, want, chunk, SG_MEAS | SG_PREP | SG_RES | SG_ACC, pst, &P);
    if (rc) return rc;
  }
  e->last_pipes = P > 1 ? P : 1;
  if (P > 1) {
    // every pipeline orders after the caller's producers (jx_engine_wait_stream / _event act on the
    // engine stream) and the engine stream after every pipeline (the join), so the call keeps the
    // single-stream ordering contract
    HIPCHK(e, hipEventRecord(e->ev_pipe, e->stream));
    for (uint32_t k = 0; k < P; k++) HIPCHK(e, hipStreamWaitEvent(e->pipes[k]->stream, e->ev_pipe, 0));
    auto run = [&]() -> int32_t {
      uint64_t i = 0;
      for (uint64_t off = 0; off < n; off += chunk, i++) {
        jx_engine* q = e->pipes[i % P];
        const uint64_t m = (n - off) < chunk ? (n - off) : chunk;
        uint8_t* vout = d_out_verdicts ? (uint8_t*)d_out_verdicts + off : q->d_verdicts;
        uint8_t* mout = (d_out_prep_msgs && c.jr_len) ? (uint8_t*)d_out_prep_msgs + off * c.seed : q->d_msgs;
        int32_t r = prep_core(q, m, N + off * 16, PS ? PS + off * c.ps_bytes : nullptr, H + off * c.his_bytes,
                              L + off * c.lps_bytes, vout, mout, staging_outs(q));
        if (r) return r;
        if (i > 0) HIPCHK(e, hipStreamWaitEvent(q->stream, e->ev_pipe, 0));  // the previous launch's K4
        r = accumulate_into(q, AccSrc{m, staging_outs(q), vout, N + off * 16}, nullptr, SG ? SG + off : nullptr,
                            targets);
        if (r) return r;
        HIPCHK(e, hipEventRecord(e->ev_pipe, q->stream));
      }
      return JX_OK;
    };
    rc = run();
    // the join, also after a failed launch: whatever was queued on a pipeline stays ordered before the
    // engine stream's later work (and jx_engine_sync)
    for (uint32_t k = 0; k < P; k++) {
      HIPCHK(e, hipEventRecord(e->pipes[k]->ev_join, e->pipes[k]->stream));
      HIPCHK(e, hipStreamWaitEvent(e->stream, e->pipes[k]->ev_join, 0));
    }
    return rc;
  }
  if (P == 1) pst[0].release();
  Stage st;
  rc = stage_acquire(e, chunk, SG_MEAS | SG_PREP | SG_RES | SG_ACC, st);
  if (rc) return rc;
  // the pointer table is uploaded once for every launch of the call (no per-launch host sync)
  Scratch tbl;
  if (many) {
    rc = upload_targets(e, targets, tbl);
    if (rc) return rc;
  }
  for (uint64_t off = 0; off < n; off += chunk) {
    const uint64_t m = (n - off) < chunk ? (n - off) : chunk;
    uint8_t* vout = d_out_verdicts ? (uint8_t*)d_out_verdicts + off : e->d_verdicts;
    uint8_t* mout = (d_out_prep_msgs && c.jr_len) ? (uint8_t*)d_out_prep_msgs + off * c.seed : e->d_msgs;
    rc = prep_core(e, m, N + off * 16, PS ? PS + off * c.ps_bytes : nullptr, H + off * c.his_bytes,
                   L + off * c.lps_bytes, vout, mout, staging_outs(e));
    if (rc) return rc;
    rc = accumulate_into(e, AccSrc{m, staging_outs(e), vout, N + off * 16}, nullptr, SG ? SG + off : nullptr, targets,
                         many);
    if (rc) return rc;
  }
  return JX_OK;
}

int32_t jx_aggregate_read(jx_engine* e, uint32_t segment, uint8_t* out_agg, uint64_t* count) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  FLUSH_ACC(e);  // the deferred accumulations land first
  const Cfg& c = e->cfg;
  const uint32_t fb = c.fb;
  Segment* s = nullptr;
  int32_t rc = get_segment(e, segment, &s);
  if (rc) return rc;
  Scratch tmp;
  rc = scratch_get(e, (size_t)c.out_len * fb, tmp, true);
  if (rc) return rc;
  HIPCHK(e, launch_agg_encode(c, s->agg, tmp.p(), e->stream));
  if (out_agg) HIPCHK(e, hipMemcpyAsync(out_agg, tmp.p(), (size_t)c.out_len * fb, hipMemcpyDeviceToHost, e->stream));
  unsigned long long cnt = 0;
  HIPCHK(e, hipMemcpyAsync(&cnt, s->count, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (count) *count = cnt;
  return drain_timing(e);
}

int32_t jx_aggregate_checksum(jx_engine* e, uint32_t segment, uint8_t out_checksum[32]) {
  if (!e || !out_checksum) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  FLUSH_ACC(e);  // the deferred accumulations land first
  Segment* s = nullptr;
  int32_t rc = get_segment(e, segment, &s);
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(out_checksum, s->checksum, 32, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return JX_OK;
}

int32_t jx_aggregate_reset(jx_engine* e) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  FLUSH_ACC(e);  // the deferred accumulations land first
  for (auto& kv : e->segs) {
    HIPCHK(e, hipMemsetAsync(kv.second.agg, 0, (size_t)e->cfg.out_len * 16, e->stream));
    HIPCHK(e, hipMemsetAsync(kv.second.checksum, 0, 32, e->stream));
    HIPCHK(e, hipMemsetAsync(kv.second.count, 0, 8, e->stream));
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return JX_OK;
}

int32_t jx_aggregate_export_device(jx_engine* e, uint32_t segment, void* d_dst) {
  if (!e || !d_dst) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  FLUSH_ACC(e);  // the deferred accumulations land first
  Segment* s = nullptr;
  int32_t rc = get_segment(e, segment, &s);
  if (rc) return rc;
  HIPCHK(e, launch_agg_encode(e->cfg, s->agg, (uint8_t*)d_dst, e->stream));
  return JX_OK;
}

static int32_t ensure_err(jx_engine* e) {
  if (!e->d_err) {
    HIPCHK(e, hipMalloc((void**)&e->d_err, sizeof(uint32_t)));
    HIPCHK(e, hipMemsetAsync(e->d_err, 0, sizeof(uint32_t), e->stream));
  }
  return JX_OK;
}

int32_t jx_aggregate_combine_device(jx_engine* e, const void* d_parts, uint32_t nparts, void* d_out) {
  if (!e || !d_parts || !d_out || nparts == 0) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  int32_t rc = ensure_err(e);
  if (rc) return rc;
  HIPCHK(e, launch_combine(e->cfg, (const uint8_t*)d_parts, nparts, (uint8_t*)d_out, e->d_err, e->stream));
  return JX_OK;
}

int32_t jx_shard_record_export_device(jx_engine* e, uint32_t segment, void* d_dst) {
  if (!e || !d_dst) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  FLUSH_ACC(e);  // the deferred accumulations land first
  Segment* s = nullptr;
  int32_t rc = get_segment(e, segment, &s);
  if (rc) return rc;
  HIPCHK(e, launch_record_export(e->cfg, s->agg, s->count, s->checksum, (uint8_t*)d_dst, e->stream));
  return JX_OK;
}

int32_t jx_shard_record_combine_device(jx_engine* e, const void* d_records, uint32_t nrecords, void* d_out) {
  if (!e || !d_records || !d_out || nrecords == 0) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  int32_t rc = ensure_err(e);
  if (rc) return rc;
  HIPCHK(e, launch_record_combine(e->cfg, (const uint8_t*)d_records, nrecords, (uint8_t*)d_out, e->d_err, e->stream));
  return JX_OK;
}

int32_t jx_shard_record_bytes(const jx_engine* e, uint32_t* bytes) {
  if (!e || !bytes) return JX_E_INVALID;
  *bytes = record_bytes(e->cfg);
  return JX_OK;
}

int32_t jx_engine_sync(jx_engine* e) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  FLUSH_ACC(e);  // the deferred accumulations land first
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (e->d_err) {
    uint32_t bad = 0;
    HIPCHK(e, hipMemcpy(&bad, e->d_err, sizeof bad, hipMemcpyDeviceToHost));
    if (bad) {
      HIPCHK(e, hipMemset(e->d_err, 0, sizeof bad));
      return fail(e, JX_E_INVALID, "combine: a merged share holds a non-canonical field element (>= p)");
    }
  }
  return JX_OK;
}

int32_t jx_engine_wait_event(jx_engine* e, void* event) {
  if (!e || !event) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamWaitEvent(e->stream, (hipEvent_t)event, 0));
  return JX_OK;
}

int32_t jx_engine_record_event(jx_engine* e, void* event) {
  if (!e || !event) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  FLUSH_ACC(e);  // the deferred accumulations land first
  HIPCHK(e, hipEventRecord((hipEvent_t)event, e->stream));
  return JX_OK;
}

int32_t jx_engine_wait_stream(jx_engine* e, void* stream) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  // hipStreamWaitEvent captures the event's current record, so one reused event serves every call
  HIPCHK(e, hipEventRecord(e->ev_wait, (hipStream_t)stream));
  HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev_wait, 0));
  return JX_OK;
}

int32_t jx_engine_join_stream(jx_engine* e, void* stream) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  FLUSH_ACC(e);  // the deferred accumulations land first
  HIPCHK(e, hipEventRecord(e->ev_join, e->stream));
  HIPCHK(e, hipStreamWaitEvent((hipStream_t)stream, e->ev_join, 0));
  return JX_OK;
}

int32_t jx_engine_stream(jx_engine* e, void** stream) {
  if (!e || !stream) return JX_E_INVALID;
  LOCK(e);
  FLUSH_ACC(e);  // work the caller queues on the stream sees the deferred accumulations
  *stream = (void*)e->stream;
  return JX_OK;
}

int32_t jx_engine_timing(jx_engine* e, int32_t enable) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  int32_t rc = drain_timing(e);
  if (rc) return rc;
  rc = collect_pipe_timing(e);
  if (rc) return rc;
  for (jx_engine* q : e->pipes) q->timing = enable != 0;
  e->timing = enable != 0;
  for (int i = 0; i < NST; i++) {
    e->ms[i] = 0;
    e->launches[i] = 0;
  }
  return JX_OK;
}

int32_t jx_engine_timing_read(jx_engine* e, float ms[4], uint64_t launches[4]) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  int32_t rc = drain_timing(e);
  if (rc) return rc;
  rc = collect_pipe_timing(e);
  if (rc) return rc;
  for (int i = 0; i < NST; i++) {
    if (ms) ms[i] = (float)e->ms[i];
    if (launches) launches[i] = e->launches[i];
  }
  return JX_OK;
}

int32_t jx_engine_coalesce(jx_engine* e, int32_t enable, uint32_t window_us) {
  if (!e || e->is_pipe) return JX_E_INVALID;
  if (window_us > 1000000) return JX_E_INVALID;
  // under the engine mutex: concurrent enables create (and reference) the device coalescer once
  LOCK(e);
  HIPCHK(e, hipSetDevice(e->device));
  if (enable && !e->coal) {
    e->coal = coalescer_for(e);
    if (!e->coal) return fail(e, JX_E_HIP, "coalesce: could not start the device coalescer");
  }
  e->coalesce = enable != 0;
  if (e->coal) coalescer_set_window(e, window_us);
  return JX_OK;
}

int32_t jx_engine_debug(jx_engine* e, int32_t option, int64_t value) {
  if (!e) return JX_E_INVALID;
  LOCK(e);
  if (option == 1) {
    e->force_slow = value != 0;
    return JX_OK;
  }
  if (option == 3) {  // helper K1 kernel
    if (value != 0 && value != 3 && value != 5 && value != 6 && value != 7) return JX_E_INVALID;
    // 0: automatic (fused; lane-split below one fused wave per SIMD, lane pairs below one lane-split
    // wave per SIMD, a word per lane for the smallest launches), 3: lane-split, 5: fused, 6: lane pairs,
    // 7: a word per lane (6, 7: bits <= 32)
    e->k1_split = (uint32_t)value;
    return JX_OK;
  }
  if (option == 4) {  // pipelines of the fused device path: 0 automatic, 1 single stream, 2..4
    if (value < 0 || value > 4) return JX_E_INVALID;
    e->npipes = (uint32_t)value;
    return JX_OK;
  }
  if (option == 2) {  // accumulate chunking (tests); staging is sized per call
    if (value < 1 || value > 4096) return JX_E_INVALID;
    e->acc_chunks = (uint32_t)value;
    return JX_OK;
  }
  if (option == 6) {  // lane-split K1 workgroups per CU: 0 no cap, 1..8
    if (value < 0 || value > 8) return JX_E_INVALID;
    e->lanes_wg_cap = (uint32_t)value;
    for (jx_engine* q : e->pipes) q->lanes_wg_cap = e->lanes_wg_cap;
    return JX_OK;
  }
  if (option == 8) {  // jx_accumulate of job-sized batches: 1 deferred and flushed together (default), 0 at once
    if (value != 0 && value != 1) return JX_E_INVALID;
    if (!value) FLUSH_ACC(e);
    e->acc_defer = value != 0;
    return JX_OK;
  }
  if (option == 9) {  // tests: run the deferred accumulations now
    FLUSH_ACC(e);
    return JX_OK;
  }
  if (option == 7) {  // tests: the device coalescer's gathers wait (up to their window) for this many jobs
    if (value < 0 || value > (int64_t)MAX_JOBS_PER_LAUNCH) return JX_E_INVALID;
    if (!e->coal) return fail(e, JX_E_STATE, "debug option 7: coalescing is off");
    coalescer_set_min_jobs(e, (uint32_t)value);
    return JX_OK;
  }
  if (option == 5) {  // reports per launch of the fused paths: 0 automatic, else >= 64 (rounded down to 64)
    if (value != 0 && value < 64) return JX_E_INVALID;
    e->default_chunk = value ? (uint64_t)value / 64 * 64 : e->auto_chunk;
    for (jx_engine* q : e->pipes) q->default_chunk = e->default_chunk;
    return JX_OK;
  }
  return JX_E_INVALID;
}

const char* jx_status_str(int32_t s) {
  switch (s) {
    case JX_OK:
      return "ok";
    case JX_E_INVALID:
      return "invalid argument";
    case JX_E_UNSUPPORTED:
      return "unsupported Prio3 parameters";
    case JX_E_HIP:
      return "HIP runtime error";
    case JX_E_NOMEM:
      return "device out of memory";
    case JX_E_STATE:
      return "call out of order";
    case JX_E_NODEVICE:
      return "no HIP device";
    default:
      return "unknown status";
  }
}

const char* jx_last_error(const jx_engine* e) {
  (void)e;
  return t_err.c_str();
}

}  // extern "C"
