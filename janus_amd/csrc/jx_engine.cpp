// jx_engine.cpp — host side of the C ABI in include/jx_prio3.h.
//
// Owns device staging, constant tables and per-segment batch aggregations; sequences
// the K1 (XOF) -> K1' (slow path) -> K3 (FLP) -> K4 (accumulate) launches on one HIP
// stream per engine. There is no CPU compute path: if the device or the kernels are
// unavailable every entry point fails with an error status.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/jx_prio3.h"
#include "jx_field.h"
#include "jx_kernels.h"
#include "jx_sha_aes.h"

using namespace jx;

namespace {

struct Segment {
  uint4* agg = nullptr;                 // [out_len] canonical
  uint32_t* checksum = nullptr;         // [8]
  unsigned long long* count = nullptr;  // [1]
};

enum { ST_XOF = 0, ST_FLP = 1, ST_ACC = 2, ST_SLOW = 3, NST = 4 };

}  // namespace

struct jx_engine {
  Cfg cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t cap = 0;  // reports (multiple of 64)
  uint64_t default_chunk = 0;
  uint64_t round_reports = 0;  // reports that fill every K1 wave slot once (0: unknown)
  // inputs (engine-owned copies for host entry points)
  uint8_t *d_nonces = nullptr, *d_ps = nullptr, *d_his = nullptr, *d_lps = nullptr;
  // staging
  uint4 *d_meas = nullptr, *d_proof = nullptr, *d_outs = nullptr, *d_coef = nullptr, *d_consts = nullptr;
  uint32_t* d_flags = nullptr;
  uint4* d_part = nullptr;
  uint8_t *d_verdicts = nullptr, *d_msgs = nullptr;
  // accumulation scratch: partials + selection bytes
  uint64_t* d_partials = nullptr;
  uint32_t acc_chunks = 0;  // report chunks of the accumulate kernel (0: acc_nchunks picks)
  uint8_t* d_tmp = nullptr;  // output-share transpose / aggregate encode
  size_t tmp_bytes = 0;
  uint8_t* d_mask = nullptr;
  uint32_t* d_seg = nullptr;
  // leader role staging (allocated on first leader call): input shares, outbound prep
  // shares, inbound prep messages; the corrected seeds (prepare state) live in d_msgs
  uint8_t *d_lis = nullptr, *d_lps_out = nullptr, *d_in_msgs = nullptr;
  uint64_t leader_cap = 0;
  bool leader_batch = false;
  std::map<uint32_t, Segment> segs;
  uint64_t last_n = 0;
  bool have_batch = false;
  // every prepared batch gets a generation id; finish / accumulate name the batch they mean
  uint64_t batch_gen = 0, batch_id = 0;
  // segmented accumulation scratch (allocated on first use)
  uint32_t* d_segx = nullptr;  // cnt, off, cursor [SEG_MAX each], ioff [SEG_MAX + 1], nitems [2]
  uint32_t* d_perm = nullptr;
  uint64_t perm_cap = 0;
  uint4* d_items = nullptr;
  uint64_t* d_spart = nullptr;
  uint64_t spart_wmax = 0;
  void** d_ptrs = nullptr;  // [3][nptrs]: aggs, counts, checksums of the call's segments
  uint64_t ptrs_cap = 0;
  std::vector<void*> h_ptrs;
  std::vector<uint32_t> h_dense;
  uint32_t* d_err = nullptr;  // combine kernels: non-canonical input seen (reported by jx_engine_sync)
  // the nonces of the resident batch (device pointer; engine copy or caller's)
  const uint8_t* batch_nonces = nullptr;
  // timing
  bool timing = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  double ms[NST] = {0, 0, 0, 0};
  uint64_t launches[NST] = {0, 0, 0, 0};
  uint32_t force_slow = 0;
  uint32_t k1_split = 0;  // helper K1 as squeeze-only + absorb-only launches (JX_K1_SPLIT, debug option 3)
  uint32_t k3_pf = 21;    // K3 load pipeline variant (JX_K3_PF, debug option 4): the depth-4 LDS-DMA ring
  // Overlapped fused path (multi-launch device calls): K3 + K4 of launch i run on stream2 while K1 of
  // launch i+1 runs on stream, from a second staging set. Off by default: measured on MI355X
  // (SumVec 8x1000/88, 5 launches per step) the concurrent kernels slow each other down more than they
  // hide (K1 26.6 -> 36.1 ms, K3 8.4 -> 23.5 ms per launch; 7.00M -> 6.62M reports/s).
  // JX_OVERLAP=1 / debug option 5 = 1 turn it on.
  uint32_t overlap = 0;
  uint4 *d_meas2 = nullptr, *d_proof2 = nullptr, *d_outs2 = nullptr, *d_coef2 = nullptr;
  uint32_t* d_flags2 = nullptr;
  uint4* d_part2 = nullptr;
  uint64_t cap2 = 0;
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_k1[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr}, ev_join = nullptr;
  std::string err;
};

static int32_t fail(jx_engine* e, int32_t code, const std::string& msg) {
  if (e) e->err = msg;
  return code;
}
#define HIPCHK(e, call)                                                                                   \
  do {                                                                                                    \
    hipError_t _st = (call);                                                                              \
    if (_st != hipSuccess)                                                                                \
      return fail((e), _st == hipErrorOutOfMemory ? JX_E_NOMEM : JX_E_HIP,                                \
                  std::string(#call) + ": " + hipGetErrorString(_st));                                    \
  } while (0)

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

// ---------------------------------------------------------------------------- buffers

static void free_staging(jx_engine* e) {
  void* ptrs[] = {e->d_nonces, e->d_ps,       e->d_his,     e->d_lps,  e->d_meas, e->d_proof, e->d_outs,
                  e->d_coef,   e->d_flags,    e->d_verdicts, e->d_msgs, e->d_partials, e->d_mask, e->d_seg,
                  e->d_part};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  e->d_nonces = e->d_ps = e->d_his = e->d_lps = nullptr;
  e->d_meas = e->d_proof = e->d_outs = e->d_coef = nullptr;
  e->d_flags = nullptr;
  e->d_part = nullptr;
  e->d_verdicts = e->d_msgs = nullptr;
  e->d_partials = nullptr;
  e->d_mask = nullptr;
  e->d_seg = nullptr;
  e->cap = 0;
  void* ptrs2[] = {e->d_meas2, e->d_proof2, e->d_outs2, e->d_coef2, e->d_flags2, e->d_part2};
  for (void* p : ptrs2)
    if (p) (void)hipFree(p);
  e->d_meas2 = e->d_proof2 = e->d_outs2 = e->d_coef2 = nullptr;
  e->d_flags2 = nullptr;
  e->d_part2 = nullptr;
  e->cap2 = 0;
  e->have_batch = false;
  for (uint8_t** p : {&e->d_lis, &e->d_lps_out, &e->d_in_msgs}) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
  }
  e->leader_cap = 0;
}

// staging element bytes: the multiproof Field64 kernels use 8-byte elements (outputs stay uint4)
static uint32_t stage_eb(const Cfg& c) { return c.algo == ALGO_SUMVEC_F64_MULTIPROOF ? 8u : 16u; }
static uint64_t coef_elems(const Cfg& c) { return c.algo == ALGO_SUMVEC_F64_MULTIPROOF ? (uint64_t)c.np * c.nco : c.ncoef; }
static uint64_t part_bytes(const Cfg& c) {
  return c.algo == ALGO_SUMVEC_F64_MULTIPROOF ? 24ull * c.np * c.ngroups : 64ull * c.ngt;
}

static uint64_t per_report_bytes(const Cfg& c) {
  uint64_t b = (uint64_t)stage_eb(c) * (c.meas_len + (uint64_t)c.np * c.proof_len + coef_elems(c));
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

static int32_t ensure_capacity(jx_engine* e, uint64_t n) {
  if (n <= e->cap) return JX_OK;
  free_staging(e);
  const Cfg& c = e->cfg;
  uint64_t cap = (n + 63) / 64 * 64;
  auto A = [&](void** p, size_t bytes) -> hipError_t { return hipMalloc(p, bytes ? bytes : 16); };
  HIPCHK(e, A((void**)&e->d_nonces, cap * 16));
  HIPCHK(e, A((void**)&e->d_ps, cap * c.ps_bytes));
  HIPCHK(e, A((void**)&e->d_his, cap * c.his_bytes));
  HIPCHK(e, A((void**)&e->d_lps, cap * c.lps_bytes));
  const uint64_t eb = stage_eb(c);
  HIPCHK(e, A((void**)&e->d_meas, cap * c.meas_len * eb));
  HIPCHK(e, A((void**)&e->d_proof, cap * c.np * c.proof_len * eb));
  if (c.algo == ALGO_COUNT || !c.out_is_meas) HIPCHK(e, A((void**)&e->d_outs, cap * c.out_len * 16));
  HIPCHK(e, A((void**)&e->d_coef, cap * coef_elems(c) * eb));
  HIPCHK(e, A((void**)&e->d_flags, cap * 4));
  HIPCHK(e, A((void**)&e->d_part, cap * part_bytes(c)));
  HIPCHK(e, A((void**)&e->d_verdicts, cap));
  HIPCHK(e, A((void**)&e->d_msgs, cap * c.seed));
  HIPCHK(e, A((void**)&e->d_mask, cap));
  HIPCHK(e, A((void**)&e->d_seg, cap * 4));
  size_t pbytes = (size_t)acc_nchunks(e) * c.out_len * 3 * sizeof(uint64_t) + cap;
  HIPCHK(e, A((void**)&e->d_partials, pbytes));
  HIPCHK(e, hipMemsetAsync(e->d_flags, 0, cap * 4, e->stream));
  e->cap = cap;
  return JX_OK;
}

// The second staging set of the overlapped fused path (same shapes as the first; cap reports). Returns
// false, with nothing allocated, when the device cannot hold it: the caller then runs serially.
static bool ensure_second_set(jx_engine* e) {
  if (e->cap2 >= e->cap && e->d_meas2) return true;
  const Cfg& c = e->cfg;
  const uint64_t cap = e->cap, eb = stage_eb(c);
  auto A = [&](void** p, size_t bytes) { return hipMalloc(p, bytes ? bytes : 16) == hipSuccess; };
  bool ok = A((void**)&e->d_meas2, cap * c.meas_len * eb) && A((void**)&e->d_proof2, cap * c.np * c.proof_len * eb) &&
            ((c.algo != ALGO_COUNT && c.out_is_meas) || A((void**)&e->d_outs2, cap * c.out_len * 16)) &&
            A((void**)&e->d_coef2, cap * coef_elems(c) * eb) && A((void**)&e->d_flags2, cap * 4) &&
            A((void**)&e->d_part2, cap * part_bytes(c));
  if (ok) ok = hipMemsetAsync(e->d_flags2, 0, cap * 4, e->stream) == hipSuccess;
  if (ok && !e->stream2) ok = hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking) == hipSuccess;
  for (hipEvent_t* ev : {&e->ev_k1[0], &e->ev_k1[1], &e->ev_free[0], &e->ev_free[1], &e->ev_join})
    if (ok && !*ev) ok = hipEventCreateWithFlags(ev, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    void* ptrs2[] = {e->d_meas2, e->d_proof2, e->d_outs2, e->d_coef2, e->d_flags2, e->d_part2};
    for (void* p : ptrs2)
      if (p) (void)hipFree(p);
    e->d_meas2 = e->d_proof2 = e->d_outs2 = e->d_coef2 = nullptr;
    e->d_flags2 = nullptr;
    e->d_part2 = nullptr;
    e->cap2 = 0;
    (void)hipGetLastError();  // the failed allocation is not an engine error
    return false;
  }
  e->cap2 = cap;
  return true;
}

static int32_t get_segment(jx_engine* e, uint32_t id, Segment** out) {
  auto it = e->segs.find(id);
  if (it == e->segs.end()) {
    Segment s;
    HIPCHK(e, hipMalloc((void**)&s.agg, (size_t)e->cfg.out_len * 16));
    HIPCHK(e, hipMalloc((void**)&s.checksum, 32));
    HIPCHK(e, hipMalloc((void**)&s.count, 8));
    HIPCHK(e, hipMemsetAsync(s.agg, 0, (size_t)e->cfg.out_len * 16, e->stream));
    HIPCHK(e, hipMemsetAsync(s.checksum, 0, 32, e->stream));
    HIPCHK(e, hipMemsetAsync(s.count, 0, 8, e->stream));
    it = e->segs.emplace(id, s).first;
  }
  *out = &it->second;
  return JX_OK;
}

static int32_t ensure_tmp(jx_engine* e, size_t bytes) {
  if (bytes <= e->tmp_bytes) return JX_OK;
  if (e->d_tmp) (void)hipFree(e->d_tmp);
  e->d_tmp = nullptr;
  e->tmp_bytes = 0;
  HIPCHK(e, hipMalloc((void**)&e->d_tmp, bytes));
  e->tmp_bytes = bytes;
  return JX_OK;
}

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

// ---------------------------------------------------------------------------- timing

static hipError_t stage_begin(jx_engine* e, hipEvent_t* ev, hipStream_t s = nullptr) {
  if (!e->timing) return hipSuccess;
  hipError_t st = hipEventCreate(ev);
  if (st != hipSuccess) return st;
  return hipEventRecord(*ev, s ? s : e->stream);
}
static hipError_t stage_end(jx_engine* e, int stage, hipEvent_t ev0, hipStream_t s = nullptr) {
  e->launches[stage]++;
  if (!e->timing) return hipSuccess;
  hipEvent_t ev1;
  hipError_t st = hipEventCreate(&ev1);
  if (st != hipSuccess) return st;
  st = hipEventRecord(ev1, s ? s : e->stream);
  e->pending.push_back({stage, {ev0, ev1}});
  return st;
}
static int32_t drain_timing(jx_engine* e) {
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

// ---------------------------------------------------------------------------- core sequencing

// Prepare n <= cap reports whose inputs are at the given device pointers.
// set: staging set (1 = the overlapped path's second set); parts: 1 = the XOF stage (K1, K1') on sx,
// 2 = the FLP stage (K3) on sf, 3 = both (default streams: the engine stream).
static int32_t prep_core(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* his,
                         const uint8_t* lps, uint8_t* verdicts, uint8_t* msgs, const uint8_t* lis = nullptr,
                         uint8_t* lps_out = nullptr, int set = 0, int parts = 3, hipStream_t sx = nullptr,
                         hipStream_t sf = nullptr) {
  const Cfg& c = e->cfg;
  const bool leader = lis != nullptr;
  if (!sx) sx = e->stream;
  if (!sf) sf = e->stream;
  Bufs b{};
  b.n = n;
  b.nonces = nonces;
  b.ps = ps;
  b.his = his;
  b.lps = lps;
  b.lis = lis;
  b.lps_out = lps_out;
  b.leader = leader ? 1u : 0u;
  b.meas = set ? e->d_meas2 : e->d_meas;
  b.proof = set ? e->d_proof2 : e->d_proof;
  b.outs = (c.out_is_meas && c.algo != ALGO_COUNT) ? b.meas : (set ? e->d_outs2 : e->d_outs);
  b.coef = set ? e->d_coef2 : e->d_coef;
  b.flags = set ? e->d_flags2 : e->d_flags;
  b.part = set ? e->d_part2 : e->d_part;
  b.verdicts = verdicts;
  b.msgs = msgs;
  b.consts = e->d_consts;
  b.force_slow = e->force_slow;
  b.k1_split = e->k1_split;
  // A helper launch that would give the fused two-sponge K1 less than one wave per SIMD is bound by
  // the per-report sponge latency, not by issue: the lane-split kernel runs it in twice the waves
  // (FixedPointBoundedL2VecSum 16 x 10000, 24,576 reports: 153 -> 92 ms on MI355X).
  const bool wide = c.bits > 32 && (c.algo == ALGO_SUM || c.algo == ALGO_SUMVEC);
  if (e->k1_split == 0 && !leader && !wide && e->round_reports && 2 * n < e->round_reports) b.k1_split = 3;
  b.k3_pf = e->k3_pf;
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
    if (parts & 1) {
      HIPCHK(e, stage_begin(e, &ev, sx));
      HIPCHK(e, launch_xof(c, b, sx));
      HIPCHK(e, stage_end(e, ST_XOF, ev, sx));
      if (!leader) {  // the leader's shares are explicit: no rejection-sampled streams to redo
        HIPCHK(e, stage_begin(e, &ev, sx));
        HIPCHK(e, launch_xof_slow(c, b, sx));
        HIPCHK(e, stage_end(e, ST_SLOW, ev, sx));
      }
    }
    if (parts & 2) {
      HIPCHK(e, stage_begin(e, &ev, sf));
      HIPCHK(e, launch_flp(c, b, sf));
      HIPCHK(e, stage_end(e, ST_FLP, ev, sf));
    }
  }
  e->batch_nonces = nonces;
  e->leader_batch = leader;
  return JX_OK;
}

static int32_t ensure_leader_capacity(jx_engine* e, uint64_t n) {
  int32_t rc = ensure_capacity(e, n);
  if (rc) return rc;
  if (n <= e->leader_cap && e->d_lis) return JX_OK;
  for (uint8_t** p : {&e->d_lis, &e->d_lps_out, &e->d_in_msgs}) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
  }
  const Cfg& c = e->cfg;
  const uint64_t cap = e->cap;
  HIPCHK(e, hipMalloc((void**)&e->d_lis, cap * c.lis_bytes));
  HIPCHK(e, hipMalloc((void**)&e->d_lps_out, cap * c.lps_bytes));
  HIPCHK(e, hipMalloc((void**)&e->d_in_msgs, cap * c.seed));
  e->leader_cap = cap;
  return JX_OK;
}

// Single-segment accumulate into aggregation seg_id. With d_seg (dense indices), only reports whose
// index is 0 are taken.
// st / set / nonces: the overlapped path's stream, staging set and launch nonces (default: the engine
// stream, set 0 and the resident batch's nonces)
static int32_t accumulate_core(jx_engine* e, uint64_t n, const uint8_t* verdicts, const uint8_t* d_mask,
                               const uint32_t* d_seg, uint32_t seg_id, bool dense = false, hipStream_t st = nullptr,
                               int set = 0, const uint8_t* nonces = nullptr) {
  const Cfg& c = e->cfg;
  Segment* s = nullptr;
  int32_t rc = get_segment(e, seg_id, &s);
  if (rc) return rc;
  if (!st) st = e->stream;
  AccArgs a{};
  a.n = n;
  uint4* meas = set ? e->d_meas2 : e->d_meas;
  a.outs = (c.out_is_meas && c.algo != ALGO_COUNT) ? meas : (set ? e->d_outs2 : e->d_outs);
  a.out_len = c.out_len;
  a.verdicts = verdicts;
  a.mask = d_mask;
  a.seg = d_seg;
  a.seg_id = dense ? 0u : seg_id;
  a.partials = e->d_partials;
  a.nchunks = acc_nchunks(e);
  uint64_t nblk = (n + 63) / 64;
  a.blocks_per_chunk = (uint32_t)((nblk + a.nchunks - 1) / a.nchunks);
  if (a.blocks_per_chunk == 0) a.blocks_per_chunk = 1;
  a.nonces = nonces ? nonces : e->batch_nonces;
  a.checksum = s->checksum;
  a.count = s->count;
  hipEvent_t ev = nullptr;
  HIPCHK(e, stage_begin(e, &ev, st));
  HIPCHK(e, launch_accumulate(c, a, s->agg, st));
  HIPCHK(e, stage_end(e, ST_ACC, ev, st));
  return JX_OK;
}

// Reports per segmented-accumulate work item: enough items that out_len x items >= 16384 waves.
static uint32_t seg_items_len(const jx_engine* e, uint64_t n) {
  const uint64_t nch = acc_nchunks(e);
  uint64_t L = (n + nch - 1) / nch;
  L = (L + 63) / 64 * 64;
  return (uint32_t)(L < 64 ? 64 : L);
}

// Accumulate the finished, accepted reports of a prepared batch into the aggregations named by a
// dense per-report segment index d_dense[r] in [0, ids.size()) (segment ids[d]); one pass per
// SEG_MAX segments. The device pointer table is uploaded once per call.
static int32_t accumulate_segmented(jx_engine* e, uint64_t n, const uint8_t* verdicts, const uint8_t* d_mask,
                                    const uint32_t* d_dense, const std::vector<uint32_t>& ids) {
  const Cfg& c = e->cfg;
  const uint64_t S = ids.size();
  if (S == 0 || n == 0) return JX_OK;
  HIPCHK(e, hipStreamSynchronize(e->stream));  // h_ptrs may still feed an earlier async upload
  // per-pass segments: SEG_MAX, or fewer when the per-item partials would exceed ~512 MiB
  const uint32_t L = seg_items_len(e, n);
  const uint64_t items_n = (n + L - 1) / L;
  const uint64_t per_item = (uint64_t)c.out_len * 24;
  uint64_t ns_max = (512ull << 20) / per_item;
  ns_max = ns_max > items_n + 64 ? ns_max - items_n : 64;
  if (ns_max > SEG_MAX) ns_max = SEG_MAX;
  const uint64_t wmax = items_n + (S < ns_max ? S : ns_max);
  if (!e->d_segx) HIPCHK(e, hipMalloc((void**)&e->d_segx, (4 * SEG_MAX + 3) * sizeof(uint32_t)));
  if (e->perm_cap < n) {
    if (e->d_perm) (void)hipFree(e->d_perm);
    e->d_perm = nullptr;
    HIPCHK(e, hipMalloc((void**)&e->d_perm, n * sizeof(uint32_t)));
    e->perm_cap = n;
  }
  if (e->spart_wmax < wmax) {
    if (e->d_items) (void)hipFree(e->d_items);
    if (e->d_spart) (void)hipFree(e->d_spart);
    e->d_items = nullptr;
    e->d_spart = nullptr;
    HIPCHK(e, hipMalloc((void**)&e->d_items, wmax * sizeof(uint4)));
    HIPCHK(e, hipMalloc((void**)&e->d_spart, wmax * per_item));
    e->spart_wmax = wmax;
  }
  if (e->ptrs_cap < S) {
    if (e->d_ptrs) (void)hipFree(e->d_ptrs);
    e->d_ptrs = nullptr;
    HIPCHK(e, hipMalloc((void**)&e->d_ptrs, 3 * S * sizeof(void*)));
    e->ptrs_cap = S;
  }
  e->h_ptrs.assign(3 * S, nullptr);
  for (uint64_t t = 0; t < S; t++) {
    Segment* sg = nullptr;
    int32_t rc = get_segment(e, ids[t], &sg);
    if (rc) return rc;
    e->h_ptrs[t] = sg->agg;
    e->h_ptrs[S + t] = sg->count;
    e->h_ptrs[2 * S + t] = sg->checksum;
  }
  HIPCHK(e, hipMemcpyAsync(e->d_ptrs, e->h_ptrs.data(), 3 * S * sizeof(void*), hipMemcpyHostToDevice, e->stream));
  uint64_t grid = (n + 255) / 256;
  if (grid > SELECT_WGS) grid = SELECT_WGS;
  for (uint64_t s0 = 0; s0 < S; s0 += ns_max) {
    const uint32_t ns = (uint32_t)(S - s0 < ns_max ? S - s0 : ns_max);
    SegArgs a{};
    a.n = n;
    a.outs = (c.out_is_meas && c.algo != ALGO_COUNT) ? e->d_meas : e->d_outs;
    a.out_len = c.out_len;
    a.fb = c.fb;
    a.verdicts = verdicts;
    a.mask = d_mask;
    a.seg = d_dense;
    a.s0 = (uint32_t)s0;
    a.ns = ns;
    a.nonces = e->batch_nonces;
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

// Accumulate the resident batch into segment_ids[d_dense[r]] (d_dense nullable: all into
// segment_ids[0]). One segment takes the coalesced select/accumulate path.
static int32_t accumulate_any(jx_engine* e, uint64_t n, const uint8_t* verdicts, const uint8_t* d_mask,
                              const uint32_t* d_dense, const std::vector<uint32_t>& ids) {
  if (ids.size() == 1 || !d_dense) return accumulate_core(e, n, verdicts, d_mask, d_dense, ids[0], d_dense != nullptr);
  return accumulate_segmented(e, n, verdicts, d_mask, d_dense, ids);
}

static int32_t check_batch(jx_engine* e, uint64_t batch_id, uint64_t n, const char* what) {
  if (batch_id == 0 || batch_id != e->batch_id || !e->have_batch || n != e->last_n)
    return fail(e, JX_E_STATE, std::string(what) + ": batch id / size does not name the resident prepared batch");
  return JX_OK;
}

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
    delete e;
    return rc;
  }
  e->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return JX_E_HIP;
  }
  std::vector<uint4> consts = make_consts(e->cfg);
  if (hipMalloc((void**)&e->d_consts, consts.size() * sizeof(uint4)) != hipSuccess ||
      hipMemcpy(e->d_consts, consts.data(), consts.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess) {
    jx_engine_destroy(e);
    return JX_E_HIP;
  }
  // Default chunk for the fused path: ~48 GiB of staging, enough for several K1 occupancy rounds of
  // the small VDAFs. A VDAF whose reports need megabytes of staging (FixedPointBoundedL2VecSum at
  // length 10000: 2.8 MB) would fill only a few percent of the SIMDs at 48 GiB, and K1 is bound by
  // the per-report sponge latency (15k sequential permutations), so throughput scales with the
  // reports in flight: grow the budget toward one full K1 round, up to 1/3 of the device memory
  // (two engines, e.g. leader and helper, still fit on one MI355X). JX_STAGING_GB / JX_CHUNK_REPORTS override.
  const uint64_t per = per_report_bytes(e->cfg);
  if (const char* env = getenv("JX_K1_SPLIT")) {
    const int v = atoi(env);
    if (v >= 0 && v <= 5) e->k1_split = (uint32_t)v;
  }
  e->round_reports = k1_round_reports(e->cfg, device, e->k1_split);
  uint64_t budget = 48ull << 30;
  size_t mem_free = 0, mem_total = 0;
  if (hipMemGetInfo(&mem_free, &mem_total) == hipSuccess && e->round_reports &&
      e->round_reports * per > budget) {
    const uint64_t cap = mem_total / 3;
    budget = e->round_reports * per < cap ? e->round_reports * per : cap;
    if (budget < (48ull << 30)) budget = 48ull << 30;
  }
  if (const char* env = getenv("JX_STAGING_GB")) {
    const uint64_t gb = strtoull(env, nullptr, 10);
    if (gb >= 1) budget = gb << 30;
  }
  uint64_t chunk = budget / per;
  if (chunk > (1ull << 22)) chunk = 1ull << 22;
  chunk = chunk / 256 * 256;
  if (chunk < 256) chunk = 256;
  if (e->round_reports && chunk >= e->round_reports) chunk = chunk / e->round_reports * e->round_reports;
  if (const char* env = getenv("JX_CHUNK_REPORTS")) {
    uint64_t v = strtoull(env, nullptr, 10);
    if (v >= 64) chunk = v / 64 * 64;
  }
  e->default_chunk = chunk;
  if (const char* env = getenv("JX_OVERLAP")) e->overlap = atoi(env) != 0;
  if (const char* env = getenv("JX_K3_PF")) {
    const int v = atoi(env);
    if (v == 1 || v == 2 || v == 12 || v == 13 || (v >= 20 && v <= 26 && v != 24)) e->k3_pf = (uint32_t)v;  // 22/23/25: timing probes
  }
  *out = e;
  return JX_OK;
}

void jx_engine_destroy(jx_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  if (e->stream2) (void)hipStreamSynchronize(e->stream2);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (hipEvent_t ev : {e->ev_k1[0], e->ev_k1[1], e->ev_free[0], e->ev_free[1], e->ev_join})
    if (ev) (void)hipEventDestroy(ev);
  for (auto& p : e->pending) {
    (void)hipEventDestroy(p.second.first);
    (void)hipEventDestroy(p.second.second);
  }
  free_staging(e);
  for (auto& kv : e->segs) {
    (void)hipFree(kv.second.agg);
    (void)hipFree(kv.second.checksum);
    (void)hipFree(kv.second.count);
  }
  if (e->d_consts) (void)hipFree(e->d_consts);
  if (e->d_tmp) (void)hipFree(e->d_tmp);
  for (void* q : {(void*)e->d_segx, (void*)e->d_perm, (void*)e->d_items, (void*)e->d_spart, (void*)e->d_ptrs,
                  (void*)e->d_err})
    if (q) (void)hipFree(q);
  if (e->d_lis) (void)hipFree(e->d_lis);
  if (e->d_lps_out) (void)hipFree(e->d_lps_out);
  if (e->d_in_msgs) (void)hipFree(e->d_in_msgs);
  if (e->stream2) (void)hipStreamDestroy(e->stream2);
  if (e->stream) (void)hipStreamDestroy(e->stream);
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

int32_t jx_engine_set_capacity(jx_engine* e, uint64_t reports) {
  if (!e) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  return ensure_capacity(e, reports);
}

int32_t jx_helper_prep_batch(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* public_shares,
                             const uint8_t* helper_input_shares, const uint8_t* leader_prep_shares,
                             uint8_t* out_prep_msgs, uint8_t* out_verdicts, uint8_t* out_output_shares) {
  if (!e || !nonces || !helper_input_shares || !leader_prep_shares || !out_verdicts) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  if (c.ps_bytes && !public_shares) return JX_E_INVALID;
  e->have_batch = false;
  e->batch_id = 0;
  if (n == 0) {
    e->have_batch = true;
    e->leader_batch = false;
    e->last_n = 0;
    e->batch_id = ++e->batch_gen;
    return JX_OK;
  }
  HIPCHK(e, hipSetDevice(e->device));
  int32_t rc = ensure_capacity(e, n);
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(e->d_nonces, nonces, n * 16, hipMemcpyHostToDevice, e->stream));
  if (c.ps_bytes) HIPCHK(e, hipMemcpyAsync(e->d_ps, public_shares, n * c.ps_bytes, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(e->d_his, helper_input_shares, n * c.his_bytes, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(e->d_lps, leader_prep_shares, n * c.lps_bytes, hipMemcpyHostToDevice, e->stream));
  rc = prep_core(e, n, e->d_nonces, e->d_ps, e->d_his, e->d_lps, e->d_verdicts, e->d_msgs);
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(out_verdicts, e->d_verdicts, n, hipMemcpyDeviceToHost, e->stream));
  if (out_prep_msgs && c.jr_len)
    HIPCHK(e, hipMemcpyAsync(out_prep_msgs, e->d_msgs, n * c.seed, hipMemcpyDeviceToHost, e->stream));
  if (out_output_shares) {
    const uint32_t fb = c.fb;
    rc = ensure_tmp(e, n * c.out_len * fb);
    if (rc) return rc;
    const uint4* outs = (c.out_is_meas && c.algo != ALGO_COUNT) ? e->d_meas : e->d_outs;
    HIPCHK(e, launch_transpose_out(c, outs, n, e->d_tmp, e->stream));
    HIPCHK(e, hipMemcpyAsync(out_output_shares, e->d_tmp, n * c.out_len * fb, hipMemcpyDeviceToHost, e->stream));
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  e->last_n = n;
  e->have_batch = true;
  e->batch_id = ++e->batch_gen;
  return drain_timing(e);
}

int32_t jx_engine_batch_id(const jx_engine* e, uint64_t* batch_id) {
  if (!e || !batch_id) return JX_E_INVALID;
  *batch_id = e->have_batch ? e->batch_id : 0;
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
  if (!e || !nonces || !leader_input_shares || !out_prep_shares || !out_verdicts) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  if (c.ps_bytes && !public_shares) return JX_E_INVALID;
  e->have_batch = false;
  e->batch_id = 0;
  if (out_batch_id) *out_batch_id = 0;
  if (n == 0) {
    e->have_batch = true;
    e->leader_batch = true;
    e->last_n = 0;
    e->batch_id = ++e->batch_gen;
    if (out_batch_id) *out_batch_id = e->batch_id;
    return JX_OK;
  }
  HIPCHK(e, hipSetDevice(e->device));
  int32_t rc = ensure_leader_capacity(e, n);
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(e->d_nonces, nonces, n * 16, hipMemcpyHostToDevice, e->stream));
  if (c.ps_bytes) HIPCHK(e, hipMemcpyAsync(e->d_ps, public_shares, n * c.ps_bytes, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(e->d_lis, leader_input_shares, n * c.lis_bytes, hipMemcpyHostToDevice, e->stream));
  rc = prep_core(e, n, e->d_nonces, e->d_ps, nullptr, nullptr, e->d_verdicts, e->d_msgs, e->d_lis, e->d_lps_out);
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(out_verdicts, e->d_verdicts, n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(out_prep_shares, e->d_lps_out, n * c.lps_bytes, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  e->last_n = n;
  e->have_batch = true;
  e->batch_id = ++e->batch_gen;
  if (out_batch_id) *out_batch_id = e->batch_id;
  return drain_timing(e);
}

int32_t jx_leader_prep_init_device(jx_engine* e, uint64_t n, const void* d_nonces, const void* d_public_shares,
                                   const void* d_leader_input_shares, void* d_out_prep_shares, void* d_out_verdicts,
                                   uint64_t* out_batch_id) {
  if (!e || !d_nonces || !d_leader_input_shares || !d_out_prep_shares || !out_batch_id) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  if (c.ps_bytes && !d_public_shares) return JX_E_INVALID;
  e->have_batch = false;
  e->batch_id = 0;
  *out_batch_id = 0;
  HIPCHK(e, hipSetDevice(e->device));
  if (n) {
    int32_t rc = ensure_capacity(e, n);
    if (rc) return rc;
    rc = prep_core(e, n, (const uint8_t*)d_nonces, (const uint8_t*)d_public_shares, nullptr, nullptr, e->d_verdicts,
                   e->d_msgs, (const uint8_t*)d_leader_input_shares, (uint8_t*)d_out_prep_shares);
    if (rc) return rc;
    if (d_out_verdicts) HIPCHK(e, hipMemcpyAsync(d_out_verdicts, e->d_verdicts, n, hipMemcpyDeviceToDevice, e->stream));
  }
  e->leader_batch = true;
  e->last_n = n;
  e->have_batch = true;
  e->batch_id = ++e->batch_gen;
  *out_batch_id = e->batch_id;
  return JX_OK;
}

int32_t jx_leader_prep_finish_batch(jx_engine* e, uint64_t batch_id, uint64_t n, const uint8_t* prep_msgs,
                                    uint8_t* out_verdicts, uint8_t* out_output_shares) {
  if (!e || !out_verdicts) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  int32_t rc0 = check_batch(e, batch_id, n, "leader finish");
  if (rc0) return rc0;
  if (!e->leader_batch) return fail(e, JX_E_STATE, "leader finish: the resident batch is a helper batch");
  if (c.jr_len && !prep_msgs) return JX_E_INVALID;
  if (n == 0) return JX_OK;
  HIPCHK(e, hipSetDevice(e->device));
  if (c.jr_len) {
    HIPCHK(e, hipMemcpyAsync(e->d_in_msgs, prep_msgs, n * c.seed, hipMemcpyHostToDevice, e->stream));
    Bufs b{};
    b.n = n;
    b.verdicts = e->d_verdicts;
    b.msgs = e->d_msgs;
    HIPCHK(e, launch_leader_finish(c, b, e->d_in_msgs, nullptr, e->stream));
  }
  HIPCHK(e, hipMemcpyAsync(out_verdicts, e->d_verdicts, n, hipMemcpyDeviceToHost, e->stream));
  if (out_output_shares) {
    const uint32_t fb = c.fb;
    int32_t rc = ensure_tmp(e, n * c.out_len * fb);
    if (rc) return rc;
    const uint4* outs = (c.out_is_meas && c.algo != ALGO_COUNT) ? e->d_meas : e->d_outs;
    HIPCHK(e, launch_transpose_out(c, outs, n, e->d_tmp, e->stream));
    HIPCHK(e, hipMemcpyAsync(out_output_shares, e->d_tmp, n * c.out_len * fb, hipMemcpyDeviceToHost, e->stream));
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return JX_OK;
}

int32_t jx_leader_prep_finish_device(jx_engine* e, uint64_t batch_id, uint64_t n, const void* d_prep_msgs,
                                     const void* d_peer_verdicts, void* d_out_verdicts) {
  if (!e) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  int32_t rc = check_batch(e, batch_id, n, "leader finish");
  if (rc) return rc;
  if (!e->leader_batch) return fail(e, JX_E_STATE, "leader finish: the resident batch is a helper batch");
  if (c.jr_len && !d_prep_msgs) return JX_E_INVALID;
  if (n == 0) return JX_OK;
  HIPCHK(e, hipSetDevice(e->device));
  Bufs b{};
  b.n = n;
  b.verdicts = e->d_verdicts;
  b.msgs = e->d_msgs;
  HIPCHK(e, launch_leader_finish(c, b, (const uint8_t*)d_prep_msgs, (const uint8_t*)d_peer_verdicts, e->stream));
  if (d_out_verdicts) HIPCHK(e, hipMemcpyAsync(d_out_verdicts, e->d_verdicts, n, hipMemcpyDeviceToDevice, e->stream));
  return JX_OK;
}

int32_t jx_accumulate(jx_engine* e, uint64_t batch_id, uint64_t n, const uint8_t* accept_mask,
                      const uint32_t* segment) {
  if (!e) return JX_E_INVALID;
  int32_t rc = check_batch(e, batch_id, n, "accumulate");
  if (rc) return rc;
  e->have_batch = false;  // a batch is accumulated at most once
  e->batch_id = 0;
  if (n == 0) return JX_OK;
  HIPCHK(e, hipSetDevice(e->device));
  const uint8_t* dm = nullptr;
  if (accept_mask) {
    HIPCHK(e, hipMemcpyAsync(e->d_mask, accept_mask, n, hipMemcpyHostToDevice, e->stream));
    dm = e->d_mask;
  }
  std::vector<uint32_t> ids{0};
  const uint32_t* ds = nullptr;
  if (segment) {
    densify(segment, n, e->h_dense, ids);
    if (ids.size() > 1) {
      HIPCHK(e, hipMemcpyAsync(e->d_seg, e->h_dense.data(), n * 4, hipMemcpyHostToDevice, e->stream));
      ds = e->d_seg;
    }
  }
  rc = accumulate_any(e, n, e->d_verdicts, dm, ds, ids);
  if (rc) return rc;
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return drain_timing(e);
}

int32_t jx_accumulate_device(jx_engine* e, uint64_t batch_id, uint64_t n, const void* d_accept_mask,
                             const void* d_segment, const uint32_t* segment_ids, uint32_t nsegments) {
  if (!e || !segment_ids || nsegments == 0) return JX_E_INVALID;
  int32_t rc = check_batch(e, batch_id, n, "accumulate");
  if (rc) return rc;
  e->have_batch = false;
  e->batch_id = 0;
  if (n == 0) return JX_OK;
  HIPCHK(e, hipSetDevice(e->device));
  std::vector<uint32_t> ids(segment_ids, segment_ids + nsegments);
  return accumulate_any(e, n, e->d_verdicts, (const uint8_t*)d_accept_mask, (const uint32_t*)d_segment, ids);
}

int32_t jx_helper_prep_aggregate(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* public_shares,
                                 const uint8_t* helper_input_shares, const uint8_t* leader_prep_shares,
                                 uint32_t segment, uint8_t* out_prep_msgs, uint8_t* out_verdicts) {
  if (!e || !nonces || !helper_input_shares || !leader_prep_shares) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  if (c.ps_bytes && !public_shares) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  const uint64_t chunk = launch_chunk(e, n);
  int32_t rc = ensure_capacity(e, chunk);
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
    rc = prep_core(e, m, e->d_nonces, e->d_ps, e->d_his, e->d_lps, e->d_verdicts, e->d_msgs);
    if (rc) return rc;
    rc = accumulate_core(e, m, e->d_verdicts, nullptr, nullptr, segment);
    if (rc) return rc;
    if (out_verdicts)
      HIPCHK(e, hipMemcpyAsync(out_verdicts + off, e->d_verdicts, m, hipMemcpyDeviceToHost, e->stream));
    if (out_prep_msgs && c.jr_len)
      HIPCHK(e, hipMemcpyAsync(out_prep_msgs + off * c.seed, e->d_msgs, m * c.seed, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  e->have_batch = false;  // staging no longer holds one whole batch
  e->batch_id = 0;
  return drain_timing(e);
}

int32_t jx_helper_prep_aggregate_device(jx_engine* e, uint64_t n, const void* d_nonces, const void* d_ps,
                                        const void* d_his, const void* d_lps, const void* d_segment,
                                        const uint32_t* segment_ids, uint32_t nsegments, void* d_out_prep_msgs,
                                        void* d_out_verdicts) {
  if (!e || !d_nonces || !d_his || !d_lps || !segment_ids || nsegments == 0) return JX_E_INVALID;
  const Cfg& c = e->cfg;
  if (c.ps_bytes && !d_ps) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  const uint64_t chunk = launch_chunk(e, n);
  int32_t rc = ensure_capacity(e, chunk);
  if (rc) return rc;
  e->have_batch = false;
  e->batch_id = 0;
  const std::vector<uint32_t> ids(segment_ids, segment_ids + nsegments);
  const uint8_t *N = (const uint8_t*)d_nonces, *PS = (const uint8_t*)d_ps, *H = (const uint8_t*)d_his,
                *L = (const uint8_t*)d_lps;
  const uint32_t* SG = (const uint32_t*)d_segment;
  // Several launches into one aggregation, when enabled: pipeline them over two streams and two
  // staging sets. K1 (VALU-bound, every VGPR of its SIMDs) of launch i+1 runs while K3 (bound by the
  // staging read stream) and K4 of launch i drain on stream2; K3/K4 stay ordered among themselves on
  // stream2 (one aggregation). Measured slower than the serial path (see `overlap`).
  const bool generic = c.algo != ALGO_COUNT && c.algo != ALGO_SUMVEC_F64_MULTIPROOF;
  if (e->overlap && generic && n > chunk && !SG && nsegments == 1 && ensure_second_set(e)) {
    Segment* seg = nullptr;
    rc = get_segment(e, ids[0], &seg);  // its zero-fill is queued on stream, before the first K1
    if (rc) return rc;
    HIPCHK(e, hipEventRecord(e->ev_join, e->stream));
    HIPCHK(e, hipStreamWaitEvent(e->stream2, e->ev_join, 0));
    uint64_t i = 0;
    for (uint64_t off = 0; off < n; off += chunk, i++) {
      const uint64_t m = (n - off) < chunk ? (n - off) : chunk;
      const int set = (int)(i & 1);
      uint8_t* vout = d_out_verdicts ? (uint8_t*)d_out_verdicts + off : e->d_verdicts;
      uint8_t* mout = (d_out_prep_msgs && c.jr_len) ? (uint8_t*)d_out_prep_msgs + off * c.seed : e->d_msgs;
      if (i >= 2) HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev_free[set], 0));  // set reused: K3/K4 of i-2 done
      rc = prep_core(e, m, N + off * 16, PS ? PS + off * c.ps_bytes : nullptr, H + off * c.his_bytes,
                     L + off * c.lps_bytes, vout, mout, nullptr, nullptr, set, 1, e->stream, e->stream2);
      if (rc) return rc;
      HIPCHK(e, hipEventRecord(e->ev_k1[set], e->stream));
      HIPCHK(e, hipStreamWaitEvent(e->stream2, e->ev_k1[set], 0));
      rc = prep_core(e, m, N + off * 16, PS ? PS + off * c.ps_bytes : nullptr, H + off * c.his_bytes,
                     L + off * c.lps_bytes, vout, mout, nullptr, nullptr, set, 2, e->stream, e->stream2);
      if (rc) return rc;
      rc = accumulate_core(e, m, vout, nullptr, nullptr, ids[0], false, e->stream2, set, N + off * 16);
      if (rc) return rc;
      HIPCHK(e, hipEventRecord(e->ev_free[set], e->stream2));
    }
    HIPCHK(e, hipEventRecord(e->ev_join, e->stream2));
    HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev_join, 0));  // callers sync the engine stream
    return JX_OK;
  }
  for (uint64_t off = 0; off < n; off += chunk) {
    const uint64_t m = (n - off) < chunk ? (n - off) : chunk;
    uint8_t* vout = d_out_verdicts ? (uint8_t*)d_out_verdicts + off : e->d_verdicts;
    uint8_t* mout = (d_out_prep_msgs && c.jr_len) ? (uint8_t*)d_out_prep_msgs + off * c.seed : e->d_msgs;
    rc = prep_core(e, m, N + off * 16, PS ? PS + off * c.ps_bytes : nullptr, H + off * c.his_bytes,
                   L + off * c.lps_bytes, vout, mout);
    if (rc) return rc;
    rc = accumulate_any(e, m, vout, nullptr, SG ? SG + off : nullptr, ids);
    if (rc) return rc;
  }
  return JX_OK;
}

int32_t jx_aggregate_read(jx_engine* e, uint32_t segment, uint8_t* out_agg, uint64_t* count) {
  if (!e) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  const Cfg& c = e->cfg;
  const uint32_t fb = c.fb;
  Segment* s = nullptr;
  int32_t rc = get_segment(e, segment, &s);
  if (rc) return rc;
  rc = ensure_tmp(e, (size_t)c.out_len * fb);
  if (rc) return rc;
  HIPCHK(e, launch_agg_encode(c, s->agg, e->d_tmp, e->stream));
  if (out_agg) HIPCHK(e, hipMemcpyAsync(out_agg, e->d_tmp, (size_t)c.out_len * fb, hipMemcpyDeviceToHost, e->stream));
  unsigned long long cnt = 0;
  HIPCHK(e, hipMemcpyAsync(&cnt, s->count, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (count) *count = cnt;
  return drain_timing(e);
}

int32_t jx_aggregate_checksum(jx_engine* e, uint32_t segment, uint8_t out_checksum[32]) {
  if (!e || !out_checksum) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  Segment* s = nullptr;
  int32_t rc = get_segment(e, segment, &s);
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(out_checksum, s->checksum, 32, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return JX_OK;
}

int32_t jx_aggregate_reset(jx_engine* e) {
  if (!e) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
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
  HIPCHK(e, hipSetDevice(e->device));
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
  HIPCHK(e, hipSetDevice(e->device));
  int32_t rc = ensure_err(e);
  if (rc) return rc;
  HIPCHK(e, launch_combine(e->cfg, (const uint8_t*)d_parts, nparts, (uint8_t*)d_out, e->d_err, e->stream));
  return JX_OK;
}

int32_t jx_shard_record_export_device(jx_engine* e, uint32_t segment, void* d_dst) {
  if (!e || !d_dst) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  Segment* s = nullptr;
  int32_t rc = get_segment(e, segment, &s);
  if (rc) return rc;
  HIPCHK(e, launch_record_export(e->cfg, s->agg, s->count, s->checksum, (uint8_t*)d_dst, e->stream));
  return JX_OK;
}

int32_t jx_shard_record_combine_device(jx_engine* e, const void* d_records, uint32_t nrecords, void* d_out) {
  if (!e || !d_records || !d_out || nrecords == 0) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
  int32_t rc = ensure_err(e);
  if (rc) return rc;
  HIPCHK(e, launch_record_combine(e->cfg, (const uint8_t*)d_records, nrecords, (uint8_t*)d_out, e->d_err, e->stream));
  return JX_OK;
}

int32_t jx_shard_record_bytes(const jx_engine* e, uint32_t* bytes) {
  if (!e || !bytes) return JX_E_INVALID;
  *bytes = e->cfg.out_len * e->cfg.fb + 40u;
  return JX_OK;
}

int32_t jx_engine_sync(jx_engine* e) {
  if (!e) return JX_E_INVALID;
  HIPCHK(e, hipSetDevice(e->device));
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

int32_t jx_engine_stream(jx_engine* e, void** stream) {
  if (!e || !stream) return JX_E_INVALID;
  *stream = (void*)e->stream;
  return JX_OK;
}

int32_t jx_engine_timing(jx_engine* e, int32_t enable) {
  if (!e) return JX_E_INVALID;
  int32_t rc = drain_timing(e);
  if (rc) return rc;
  e->timing = enable != 0;
  for (int i = 0; i < NST; i++) {
    e->ms[i] = 0;
    e->launches[i] = 0;
  }
  return JX_OK;
}

int32_t jx_engine_timing_read(jx_engine* e, float ms[4], uint64_t launches[4]) {
  if (!e) return JX_E_INVALID;
  int32_t rc = drain_timing(e);
  if (rc) return rc;
  for (int i = 0; i < NST; i++) {
    if (ms) ms[i] = (float)e->ms[i];
    if (launches) launches[i] = e->launches[i];
  }
  return JX_OK;
}

int32_t jx_engine_debug(jx_engine* e, int32_t option, int64_t value) {
  if (!e) return JX_E_INVALID;
  if (option == 1) {
    e->force_slow = value != 0;
    return JX_OK;
  }
  if (option == 3) {  // helper K1 variant
    if (value < 0 || value > 5) return JX_E_INVALID;
    // 0: automatic (fused; lane-split below one fused wave per SIMD), 1 / 2: squeeze-only + absorb-only
    // launches (absorb at 3 / 2 waves/SIMD), 3: lane-split, 4: sequential S, J permutations, 5: fused
    e->k1_split = (uint32_t)value;
    return JX_OK;
  }
  if (option == 5) {  // overlapped two-stream fused path for multi-launch device calls (1) or not (0, default)
    e->overlap = value != 0;
    return JX_OK;
  }
  if (option == 4) {  // K3 load pipeline: 1 or 2 calls ahead; 12 / 13 = 2 / 3 ahead at 3 waves/SIMD; 20 / 21 LDS-DMA ring
    if (value != 1 && value != 2 && value != 12 && value != 13 && value != 20 && value != 21 && value != 26)
      return JX_E_INVALID;
    e->k3_pf = (uint32_t)value;
    return JX_OK;
  }
  if (option == 2) {  // accumulate chunking (tests)
    if (value < 1 || value > 4096) return JX_E_INVALID;
    free_staging(e);
    e->acc_chunks = (uint32_t)value;
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

const char* jx_last_error(const jx_engine* e) { return e ? e->err.c_str() : ""; }

}  // extern "C"
