// jx_mp64.hip — gfx950 kernels for Prio3SumVecField64MultiproofHmacSha256Aes128
// (SURVEY.md §8(f) #3): prio 0.16.1 Prio3<SumVec<Field64, ParallelSum<Field64, Mul<Field64>>>,
// XofHmacSha256Aes128, 32> with num_proofs >= 2, built by Janus at core/src/vdaf.rs:173-199 and
// dispatched by the aggregator at aggregator.rs:890-903,1226-1236.
//
// Same stage structure as jx_kernels.hip:
//   K1  mp_xof_kernel<ROLE>  one report per lane. Helper: the measurement share is the AES-128-CTR
//       keystream of HMAC-SHA256(k_meas, dst || [1]); every 64-byte keystream chunk (8 elements, 4
//       AES blocks) is stored, truncated into the output share and absorbed at once into the
//       joint_rand_part HMAC (one SHA-256 compression per chunk, no second pass over the share).
//       Leader: the chunks are its explicit share. Then the proofs share, joint randomness, query
//       randomness and the per-proof FLP coefficients (mp_tail).
//   K1' mp_slow_kernel      reports whose keystream produced a value >= p (2^-32 per element):
//       exact recomputation with rejection sampling.
//   K3  mp_flp_part/final   one wave per (64-report block, chunk-slot group, proof): Field64 wire
//       sums as 32x22-bit limb column sums; then per report: add the leader's verifier shares and
//       decide every proof.
// K4 (accumulate) is shared with the other instances: output shares go to the uint4 staging.
//
// AES runs on a T-table in LDS replicated 32 times (lane l reads copy l mod 32: every ds_read_b32
// of a wave is bank-conflict-free). Staging is interleaved [block][element][lane] in 8-byte
// elements: a wave touching element e moves one coalesced 512 B.
#include "jx_field.h"
#include "jx_kernels.h"
#include "jx_sha_aes.h"

namespace jx {

namespace {

constexpr uint32_t USAGE_MEAS = 1, USAGE_PROOF = 2, USAGE_JR = 3, USAGE_QR = 5, USAGE_JR_SEED = 6,
                   USAGE_JR_PART = 7;

// AES tables in LDS (128 KiB): T_t[x] = rotl(T0[x], 8t), T0[x] = (2s, s, s, 3s), t = 0..3, each in 32
// copies; lane l reads copy l mod 32, which sits in bank l mod 32, so every ds_read_b32 of a wave is
// conflict-free. Lane l's copy of T_t[x] is at byte (t >> 1) << 16 | x << 8 | (t & 1) << 7 | 4 (l mod
// 32): one v_perm_b32 merges the state byte (-> bits 8..15) with the lane's per-table address word
// a_t. A MixColumns column is four lookups (four perms) and two 3-input XORs.
constexpr uint32_t TT_WORDS = 4 * 256 * 32;
struct TTab {
  const uint8_t* base;  // the tables (LDS)
  uint32_t a0;          // 4 (lane mod 32)
  // T0[x] (key schedule, one-off blocks)
  __device__ __forceinline__ uint32_t operator()(uint32_t x) const {
    return *reinterpret_cast<const uint32_t*>(base + ((x << 8) | a0));
  }
};
__device__ __forceinline__ TTab ttab(const uint32_t* tt, uint32_t lane) {
  return TTab{reinterpret_cast<const uint8_t*>(tt), 4u * (lane & 31u)};
}

__device__ __forceinline__ void tt_fill(uint32_t* tt) {
  for (uint32_t i = threadIdx.x; i < TT_WORDS; i += blockDim.x) {
    const uint32_t t = 2 * (i >> 14) + ((i >> 5) & 1u);
    const uint32_t t0 = aes_t0_entry(AES_SBOX[(i >> 6) & 255u]);
    tt[i] = t ? rotl32(t0, 8 * t) : t0;
  }
}
// T_t of byte K of s
template <int t, int K>
__device__ __forceinline__ uint32_t lt(const TTab& T, uint32_t s) {
  const uint32_t a = T.a0 | ((uint32_t)(t >> 1) << 16) | ((uint32_t)(t & 1) << 7);
  return *reinterpret_cast<const uint32_t*>(T.base + __builtin_amdgcn_perm(s, a, 0x0C020000u | ((4u + K) << 8)));
}
// one MixColumns output column from state columns (a, b, c, d) = (c, c+1, c+2, c+3)
__device__ __forceinline__ uint32_t aes_col(const TTab& T, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                            uint32_t k) {
  return xor3(xor3(lt<0, 0>(T, a), lt<1, 1>(T, b), lt<2, 2>(T, c)), lt<3, 3>(T, d), k);
}
// last round: S[x] is byte 1 and byte 2 of T0[x] and byte 3 of T1[x]
__device__ __forceinline__ uint32_t aes_col_last(const TTab& T, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                                 uint32_t k) {
  const uint32_t lo = __builtin_amdgcn_perm(lt<0, 1>(T, b), lt<0, 0>(T, a), 0x0C0C0501u);
  const uint32_t hi = __builtin_amdgcn_perm(lt<1, 3>(T, d), lt<0, 2>(T, c), 0x07020C0Cu);
  return (lo | hi) ^ k;
}
__device__ __forceinline__ void aes_enc_fast(const TTab& T, const uint32_t rk[44], const uint32_t in[4],
                                             uint32_t out[4]) {
  uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
  for (int r = 1; r < 10; r++) {
    const uint32_t t0 = aes_col(T, s0, s1, s2, s3, rk[4 * r]);
    const uint32_t t1 = aes_col(T, s1, s2, s3, s0, rk[4 * r + 1]);
    const uint32_t t2 = aes_col(T, s2, s3, s0, s1, rk[4 * r + 2]);
    const uint32_t t3 = aes_col(T, s3, s0, s1, s2, rk[4 * r + 3]);
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  out[0] = aes_col_last(T, s0, s1, s2, s3, rk[40]);
  out[1] = aes_col_last(T, s1, s2, s3, s0, rk[41]);
  out[2] = aes_col_last(T, s2, s3, s0, s1, rk[42]);
  out[3] = aes_col_last(T, s3, s0, s1, s2, rk[43]);
}

__device__ __forceinline__ uint64_t u2v(uint2 v) { return (uint64_t)v.x | ((uint64_t)v.y << 32); }
__device__ __forceinline__ uint2 v2u(uint64_t v) { return make_uint2(lo32(v), hi32(v)); }
__device__ __forceinline__ bool ge_p64(uint32_t lo, uint32_t hi) { return hi == 0xFFFFFFFFu && lo != 0u; }

__device__ __forceinline__ void load32(const uint8_t* p, uint32_t w[8]) {
  const uint4 a = *reinterpret_cast<const uint4*>(p), b = *reinterpret_cast<const uint4*>(p + 16);
  w[0] = a.x;
  w[1] = a.y;
  w[2] = a.z;
  w[3] = a.w;
  w[4] = b.x;
  w[5] = b.y;
  w[6] = b.z;
  w[7] = b.w;
}
// 8-byte aligned variant (rows of the leader's buffers)
__device__ __forceinline__ void load32_u2(const uint8_t* p, uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint2 v = *reinterpret_cast<const uint2*>(p + 8 * i);
    w[2 * i] = v.x;
    w[2 * i + 1] = v.y;
  }
}
__device__ __forceinline__ void load16(const uint8_t* p, uint32_t w[4]) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
}

// ---------------------------------------------------------------------------- XofHmacSha256Aes128
// init(seed, dst): HMAC key = seed; message = byte(len(dst)) || dst || binder...
// into_seed_stream: tag = HMAC tag; AES-128-CTR key tag[0:16], counter block tag[16:32] with a
// 64-bit big-endian counter in bytes 8..15 (ctr 0.9.2 Ctr64BE).

// byte(8) || dst, dst = [VERSION 8, class 0, algorithm id (BE32), usage (BE16)]
__device__ __forceinline__ int m_prefix(Msg128& m, uint32_t id, uint32_t usage) {
  m_byte(m, 0, 8);
  m_byte(m, 1, 8);
  m_byte(m, 2, 0);
  m_byte(m, 3, id >> 24);
  m_byte(m, 4, id >> 16);
  m_byte(m, 5, id >> 8);
  m_byte(m, 6, id);
  m_byte(m, 7, usage >> 8);
  m_byte(m, 8, usage);
  return 9;
}
// ---- one-off hashing and encryption (per-report setup and tail: ~20 SHA-256 blocks and ~10 AES
// blocks per report against ~1000 and ~4400 in the streams). These are out-of-line calls with
// register arguments so that each kernel holds one copy of the unrolled code.
struct S8 {
  uint32_t s[8];
};
__device__ __noinline__ S8 sha_call(S8 st, uint4 a, uint4 b, uint4 c, uint4 d) {
  const uint32_t w[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
  sha256_compress(st.s, w);
  return st;
}
__device__ __forceinline__ void sha_blk(uint32_t st[8], const uint32_t* w) {
  S8 x;
#pragma unroll
  for (int i = 0; i < 8; i++) x.s[i] = st[i];
  x = sha_call(x, make_uint4(w[0], w[1], w[2], w[3]), make_uint4(w[4], w[5], w[6], w[7]),
               make_uint4(w[8], w[9], w[10], w[11]), make_uint4(w[12], w[13], w[14], w[15]));
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = x.s[i];
}
__device__ __noinline__ uint4 aes_call(const uint8_t* base, uint32_t a0, uint4 key, uint4 in) {
  const TTab T{base, a0};
  const uint32_t k[4] = {key.x, key.y, key.z, key.w}, x[4] = {in.x, in.y, in.z, in.w};
  uint32_t o[4];
  aes128_encrypt_t_otf(T, k, x, o);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// HMAC pads for a 32-byte key held as little-endian memory words
__device__ __forceinline__ void hmac_key_le(const uint32_t k[8], uint32_t ist[8], uint32_t ost[8]) {
  uint32_t bi[16], bo[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t kb = i < 8 ? bswap32(k[i]) : 0u;
    bi[i] = kb ^ 0x36363636u;
    bo[i] = kb ^ 0x5c5c5c5cu;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    ist[i] = SHA256_IV[i];
    ost[i] = SHA256_IV[i];
  }
  sha_blk(ist, bi);
  sha_blk(ost, bo);
}
// hash of (64-byte block already in st0) || m[0:len]
__device__ __forceinline__ void finish64(uint32_t out[8], const uint32_t st0[8], Msg128& m, int len) {
  m_byte(m, len, 0x80);
  const int nblk = (len + 9 + 63) / 64;
  const uint64_t bits = 8ull * (64 + len);
  m.w[nblk * 16 - 2] = (uint32_t)(bits >> 32);
  m.w[nblk * 16 - 1] = (uint32_t)bits;
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = st0[i];
  sha_blk(out, m.w);
  if (nblk == 2) sha_blk(out, m.w + 16);
}
__device__ __forceinline__ void hmac_outer_c(uint32_t out[8], const uint32_t ost[8], const uint32_t inner[8]) {
  Msg128 m;
  m_zero(m);
  m_be32(m, 0, inner);
  finish64(out, ost, m, 32);
}
__device__ __forceinline__ void hmac_tag(uint32_t tag[8], const uint32_t ist[8], const uint32_t ost[8], Msg128& m,
                                         int len) {
  uint32_t inner[8];
  finish64(inner, ist, m, len);
  hmac_outer_c(tag, ost, inner);
}

// AES-128-CTR stream state (hot streams: the 44-word schedule stays in registers)
struct Ctr {
  uint32_t rk[44];
  uint32_t iv0, iv1;
  uint64_t ctr;
};
__device__ __forceinline__ void ctr_init(Ctr& s, const TTab& T, const uint32_t tag[8]) {
  uint32_t key[4];
#pragma unroll
  for (int i = 0; i < 4; i++) key[i] = bswap32(tag[i]);
  aes128_expand_key_t(T, key, s.rk);
  s.iv0 = bswap32(tag[4]);
  s.iv1 = bswap32(tag[5]);
  s.ctr = ((uint64_t)tag[6] << 32) | tag[7];
}
__device__ __forceinline__ void ctr_next(Ctr& s, const TTab& T, uint32_t out[4]) {
  const uint32_t in[4] = {s.iv0, s.iv1, bswap32(hi32(s.ctr)), bswap32(lo32(s.ctr))};
  aes_enc_fast(T, s.rk, in, out);
  s.ctr++;
}
// block j of the stream of tag, one-off
__device__ __forceinline__ uint4 ctr_block_c(const TTab& T, const uint32_t tag[8], uint64_t j) {
  const uint64_t ctr = (((uint64_t)tag[6] << 32) | tag[7]) + j;
  return aes_call(T.base, T.a0, make_uint4(bswap32(tag[0]), bswap32(tag[1]), bswap32(tag[2]), bswap32(tag[3])),
                  make_uint4(bswap32(tag[4]), bswap32(tag[5]), bswap32(hi32(ctr)), bswap32(lo32(ctr))));
}
// the first 32 bytes of the stream (Xof::into_seed), as 8 little-endian words
__device__ __forceinline__ void ctr_seed(const TTab& T, const uint32_t tag[8], uint32_t out[8]) {
  const uint4 a = ctr_block_c(T, tag, 0), b = ctr_block_c(T, tag, 1);
  out[0] = a.x;
  out[1] = a.y;
  out[2] = a.z;
  out[3] = a.w;
  out[4] = b.x;
  out[5] = b.y;
  out[6] = b.z;
  out[7] = b.w;
}
// the first n (<= MAXN) accepted Field64 elements of a fresh stream (next_vec with rejection)
template <int MAXN>
__device__ void ctr_sample(const TTab& T, const uint32_t tag[8], uint32_t n, uint64_t out[MAXN]) {
  uint32_t cnt = 0;
#pragma unroll 1
  for (uint32_t blk = 0; blk < 64 && cnt < n; blk++) {
    const uint4 v = ctr_block_c(T, tag, blk);
    const uint32_t ks[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint64_t x = (uint64_t)ks[2 * h] | ((uint64_t)ks[2 * h + 1] << 32);
      const bool acc = x < P64 && cnt < n;
#pragma unroll
      for (int i = 0; i < MAXN; i++)
        if (acc && cnt == (uint32_t)i) out[i] = x;
      cnt += acc ? 1u : 0u;
    }
  }
}
template <int N>
__device__ __forceinline__ uint64_t pick(const uint64_t a[N], uint32_t i) {
  uint64_t v = a[0];
#pragma unroll
  for (int k = 1; k < N; k++)
    if (i == (uint32_t)k) v = a[k];
  return v;
}

// XOF(0^32, DST(6), a || b)[0:32] (joint_rand_seed; the prepare message)
__device__ void jr_seed(const Cfg& c, const TTab& T, const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {
  Msg128 m;
  m_zero(m);
  int pos = m_prefix(m, c.dst_id, USAGE_JR_SEED);
  pos = m_le32(m, pos, a);
  pos = m_le32(m, pos, b);
  uint32_t tag[8];
  hmac_tag(tag, c.zero_ist, c.zero_ost, m, pos);
  ctr_seed(T, tag, out);
}

// ---------------------------------------------------------------------------- joint_rand_part
// joint_rand_part = XOF(k_blind, DST(7), [agg_id] || nonce || enc(meas_share))[0:32]. The HMAC
// inner message is hdr (26 bytes: byte(8) || dst || agg_id || nonce) || the share's bytes, so SHA
// block m holds share bytes [64m - 26, 64m + 38): words 9..15 of 64-byte chunk m-1 and words 0..9
// of chunk m, shifted by 16 bits (be_word_shift16). hv: words 9..15 of a virtual chunk -1 whose
// last 26 bytes are the header.
__device__ __forceinline__ void jr_part_header(const Cfg& c, uint32_t agg_id, const uint32_t nonce[4],
                                               uint32_t hv[7]) {
  const uint32_t id = c.dst_id;
  hv[0] = (8u << 16) | (8u << 24);  // byte(len(dst)) = 8, VERSION = 8
  hv[1] = ((id >> 24) << 8) | (((id >> 16) & 0xffu) << 16) | (((id >> 8) & 0xffu) << 24);  // class 0, id
  hv[2] = (id & 0xffu) | (0u << 8) | (USAGE_JR_PART << 16) | (agg_id << 24);
  hv[3] = nonce[0];
  hv[4] = nonce[1];
  hv[5] = nonce[2];
  hv[6] = nonce[3];
}

// Runs the inner SHA-256 of the joint_rand_part HMAC over the share. gen(q, K) supplies the 16
// little-endian words of share bytes [64q, 64q + 64); emit(q, K) does the side effects on them
// (store, truncate, screen). J: inner state after the key block on entry, the digest on return.
// Software-pipelined: chunk q + 1 is generated in the same basic block as the compression of
// block q, so the AES lookups in LDS fill the SHA-256 dependency chains.
template <class GenFn, class EmitFn>
__device__ __forceinline__ void jr_part_inner(const Cfg& c, uint32_t J[8], const uint32_t hv[7], GenFn&& gen,
                                              EmitFn&& emit) {
  const uint32_t M = c.meas_len;
  const uint32_t NC = (M + 7) / 8;
  const uint32_t Lmsg = 26 + 8 * M;
  const uint32_t nfull = Lmsg / 64;  // blocks made only of message bytes (NC - 1 or NC)
  uint32_t prev[7], cur[16];
#pragma unroll
  for (int i = 0; i < 7; i++) prev[i] = hv[i];
  gen(0, cur);
  const uint32_t qs = NC - 1;  // nfull is NC - 1 or NC
  uint32_t q = 0;
#pragma unroll 1
  for (; q < qs; q++) {
    emit(q, cur);  // branchy (uniform) side effects first; generation and hashing share a block
    uint32_t nxt[16];
    gen(q + 1, nxt);
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint32_t lo = i < 7 ? prev[i] : cur[i - 7];
      const uint32_t hi = i < 6 ? prev[i + 1] : cur[i - 6];
      W[i] = be_word_shift16(lo, hi);
    }
    sha256_compress(J, W);
#pragma unroll
    for (int i = 0; i < 7; i++) prev[i] = cur[9 + i];
#pragma unroll
    for (int i = 0; i < 16; i++) cur[i] = nxt[i];
  }
  emit(q, cur);
  if (q < nfull) {  // the last chunk's block is full too
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint32_t lo = i < 7 ? prev[i] : cur[i - 7];
      const uint32_t hi = i < 6 ? prev[i + 1] : cur[i - 6];
      W[i] = be_word_shift16(lo, hi);
    }
    sha_blk(J, W);
#pragma unroll
    for (int i = 0; i < 7; i++) prev[i] = cur[9 + i];
#pragma unroll
    for (int i = 0; i < 16; i++) cur[i] = 0;
  }
  // block mstar (the first that is not all message bytes): the tail, padding, and the bit length
  // of (key block || message)
  const uint32_t mstar = nfull;
  const int rem = (int)(Lmsg - 64 * mstar);  // message bytes in block mstar, 0..63
  uint32_t W[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t lo = i < 7 ? prev[i] : cur[i - 7];
    const uint32_t hi = i < 6 ? prev[i + 1] : cur[i - 6];
    uint32_t w = be_word_shift16(lo, hi);
    const int nv = rem - 4 * i;  // message bytes in this word
    if (nv <= 0)
      w = 0;
    else if (nv < 4)
      w &= ~(0xFFFFFFFFu >> (8 * nv));
    if (nv >= 0 && nv < 4) w |= 0x80u << (24 - 8 * nv);
    W[i] = w;
  }
  const uint64_t bits = 8ull * (64 + Lmsg);
  if (rem <= 55) {
    W[14] = hi32(bits);
    W[15] = lo32(bits);
    sha_blk(J, W);
  } else {
    sha_blk(J, W);
#pragma unroll
    for (int i = 0; i < 14; i++) W[i] = 0;
    W[14] = hi32(bits);
    W[15] = lo32(bits);
    sha_blk(J, W);
  }
}

// ---------------------------------------------------------------------------- output share
// truncate: out_i = sum_{j < bits} 2^j x_{bits i + j} as word columns (bits <= 32), reduced once
struct TruncF64 {
  uint64_t lo, hi;
  uint32_t j, i;
};
__device__ __forceinline__ void emit64(const Cfg& c, uint2* mp, uint4* op, uint32_t e, uint32_t lo, uint32_t hi,
                                       TruncF64& tr) {
  mp[(uint64_t)e * IL] = make_uint2(lo, hi);
  const uint32_t sh = 1u << tr.j;
  tr.lo += (uint64_t)lo * sh;
  tr.hi += (uint64_t)hi * sh;
  if (++tr.j == c.bits) {
    uint32_t cc = 0;
    const uint64_t w0 = addc64(tr.lo, tr.hi << 32, cc);
    const uint64_t w1 = (tr.hi >> 32) + cc;
    const uint64_t v = reduce192_p64(w0, w1, 0);
    op[(uint64_t)tr.i * IL] = make_uint4(lo32(v), hi32(v), 0, 0);
    tr.lo = tr.hi = 0;
    tr.j = 0;
    tr.i++;
  }
}

// ---------------------------------------------------------------------------- tail
// Joint randomness, the prepare message, query randomness and the per-proof FLP coefficients.
// own: this aggregator's joint_rand_part. Returns the updated flags.
__device__ uint32_t mp_tail(const Cfg& c, const Bufs& b, const TTab& T, uint64_t blk, uint32_t lane, uint64_t r,
                            bool write, const uint32_t nonce[4], const uint32_t own[8], uint32_t flags, bool leader) {
  const uint8_t* ps = b.ps + (uint64_t)c.ps_bytes * r;
  uint32_t pl[8], ph[8];
  if (leader) {
#pragma unroll
    for (int i = 0; i < 8; i++) pl[i] = own[i];
    load32(ps + 32, ph);
  } else {
    load32(ps, pl);
#pragma unroll
    for (int i = 0; i < 8; i++) ph[i] = own[i];
  }
  // corrected joint-rand seed
  uint32_t corr[8];
  jr_seed(c, T, pl, ph, corr);
  uint32_t msg[8];
#pragma unroll
  for (int i = 0; i < 8; i++) msg[i] = corr[i];
  if (!leader) {
    // prepare message = XOF(0^32, DST(6), leader's part || part_H); prepare_next fails unless it
    // equals the corrected seed
    uint32_t lp[8];
    load32_u2(b.lps + (uint64_t)c.lps_bytes * r + 8ull * c.np * c.ver_len, lp);
    bool same = true;
#pragma unroll
    for (int i = 0; i < 8; i++) same &= lp[i] == pl[i];
    if (!same) {
      jr_seed(c, T, lp, ph, msg);
      bool eq = true;
#pragma unroll
      for (int i = 0; i < 8; i++) eq &= msg[i] == corr[i];
      if (!eq) flags |= FLAG_NEXT_FAIL;
    }
  }
  if (write) {
    uint4* o = reinterpret_cast<uint4*>(b.msgs + 32 * r);
    o[0] = make_uint4(msg[0], msg[1], msg[2], msg[3]);
    o[1] = make_uint4(msg[4], msg[5], msg[6], msg[7]);
  }
  // joint_rands = expand(corrected, DST(3), [PROOFS], PROOFS); query_rands = expand(verify_key,
  // DST(5), [PROOFS] || nonce, PROOFS)
  uint64_t jr[MP_MAX_PROOFS], qr[MP_MAX_PROOFS];
  {
    uint32_t ist[8], ost[8], tag[8];
    hmac_key_le(corr, ist, ost);
    Msg128 m;
    m_zero(m);
    int pos = m_prefix(m, c.dst_id, USAGE_JR);
    m_byte(m, pos, c.np);
    hmac_tag(tag, ist, ost, m, pos + 1);
    ctr_sample<MP_MAX_PROOFS>(T, tag, c.np, jr);
  }
  {
    uint32_t tag[8];
    Msg128 m;
    m_zero(m);
    int pos = m_prefix(m, c.dst_id, USAGE_QR);
    m_byte(m, pos, c.np);
#pragma unroll
    for (int i = 0; i < 16; i++) m_byte(m, pos + 1 + i, nonce[i >> 2] >> (8 * (i & 3)));
    // the verify key's pads: this report's row of a coalesced launch's keys, or the engine's
    uint32_t vist[8], vost[8];
    if (b.vkeys) {
      const uint4* kp = reinterpret_cast<const uint4*>(b.vkeys + 64 * r);
      const uint4 k0 = kp[0], k1 = kp[1], k2 = kp[2], k3 = kp[3];
      vist[0] = k0.x, vist[1] = k0.y, vist[2] = k0.z, vist[3] = k0.w;
      vist[4] = k1.x, vist[5] = k1.y, vist[6] = k1.z, vist[7] = k1.w;
      vost[0] = k2.x, vost[1] = k2.y, vost[2] = k2.z, vost[3] = k2.w;
      vost[4] = k3.x, vost[5] = k3.y, vost[6] = k3.z, vost[7] = k3.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) vist[i] = c.vk_ist[i], vost[i] = c.vk_ost[i];
    }
    hmac_tag(tag, vist, vost, m, pos + 17);
    ctr_sample<MP_MAX_PROOFS>(T, tag, c.np, qr);
  }
  // ---- per-proof barycentric coefficients (canonical Field64):
  //   wire_j(t) = L sum_k c_k wire_j[k], c_k = w^k / (t - w^k), L = (t^P - 1)/P, d_k = c_k r^{(k-1) chunk}
  const uint4* omega = b.consts + c.c_omega;
  const uint4* misc = b.consts + c.c_misc;
  const uint64_t invP = (uint64_t)misc[0].x | ((uint64_t)misc[0].y << 32);
  const uint64_t half = (uint64_t)misc[1].x | ((uint64_t)misc[1].y << 32);
  const uint32_t C = c.calls, NCO = c.nco;
#pragma unroll 1
  for (uint32_t p = 0; p < c.np; p++) {
    uint2* cb = reinterpret_cast<uint2*>(b.coef) + ((blk * c.np + p) * NCO) * IL + lane;
    auto slot = [&](uint32_t k) -> uint2& { return cb[(uint64_t)(k == 0 ? MCOEF_C0 : MCOEF_K + 2 * (k - 1)) * IL]; };
    const uint64_t t = pick<MP_MAX_PROOFS>(qr, p), rr = pick<MP_MAX_PROOFS>(jr, p);
    uint64_t tp = t;
    for (uint32_t i = 0; i < c.logP; i++) tp = mul64(tp, tp);
    if (tp == 1) flags |= FLAG_INIT_FAIL;
    cb[MCOEF_L * IL] = v2u(mul64(sub64(tp, 1), invP));
    cb[MCOEF_T * IL] = v2u(t);
    cb[MCOEF_R * IL] = v2u(rr);
    // batch inversion of den_k = t - w^k, k = 0..C (prefix products parked in the c_k slots)
    uint64_t acc = sub64(t, 1);
    slot(0) = v2u(acc);
    for (uint32_t k = 1; k <= C; k++) {
      acc = mul64(acc, sub64(t, (uint64_t)omega[k].x | ((uint64_t)omega[k].y << 32)));
      slot(k) = v2u(acc);
    }
    uint64_t inv = pow64_h(acc, P64 - 2);
    uint64_t sumc = 0;
    for (uint32_t k = C; k >= 1; k--) {
      const uint64_t w = (uint64_t)omega[k].x | ((uint64_t)omega[k].y << 32);
      const uint64_t invden = mul64(inv, u2v(slot(k - 1)));
      inv = mul64(inv, sub64(t, w));
      const uint64_t ck = mul64(w, invden);
      slot(k) = v2u(ck);
      sumc = add64(sumc, ck);
    }
    slot(0) = v2u(inv);  // c_0 = 1/(t - 1)
    cb[MCOEF_HALFSUM * IL] = v2u(mul64(sumc, half));
    const uint64_t rc = pow64_h(rr, c.chunk);
    uint64_t rp = 1;
    for (uint32_t k = 1; k <= C; k++) {
      cb[(uint64_t)(MCOEF_K + 2 * (k - 1) + 1) * IL] = v2u(mul64(u2v(slot(k)), rp));
      rp = mul64(rp, rc);
    }
  }
  return flags;
}

// ---------------------------------------------------------------------------- K1
// HELPER (agg_id 1, aggregator.rs:1947): shares expanded from the 32-byte seeds of the helper input
// share (k_meas || k_proofs || k_blind). LEADER (agg_id 0, aggregation_job_driver.rs:345): explicit
// shares (meas || proofs || k_blind), decoded here (elements >= p fail prepare_init).
// MP_XOF_WAVES waves per workgroup share the 128 KiB of tables; one workgroup per CU
constexpr uint32_t MP_XOF_WAVES = 8;
template <bool LEADER>
__global__ __launch_bounds__(64 * MP_XOF_WAVES) void mp_xof_kernel(Cfg c, Bufs b) {
  __shared__ uint32_t tt[TT_WORDS];
  tt_fill(tt);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t blk = (uint64_t)blockIdx.x * MP_XOF_WAVES + (threadIdx.x >> 6);
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint64_t r0 = blk * 64 + lane;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const TTab T = ttab(tt, lane);
  const uint32_t M = c.meas_len, MB = 8 * M, NPL = c.np * c.proof_len;
  const uint8_t* hs = LEADER ? nullptr : b.his + (uint64_t)c.his_bytes * r;
  const uint8_t* ls = LEADER ? b.lis + b.lis_rs * r : nullptr;
  uint2* const mp = reinterpret_cast<uint2*>(b.meas) + (blk * M) * IL + lane;
  uint4* const op = b.outs + (blk * c.out_len) * IL + lane;
  uint32_t nonce[4];
  load16(b.nonces + 16 * r, nonce);
  bool bad = !LEADER && b.force_slow;
  TruncF64 tr{0, 0, 0, 0};

  // ---- measurement share fused with the joint_rand_part HMAC
  uint32_t kb[8], J[8], Jo[8], hv[7];
  if (LEADER)
    load32_u2(ls + MB + 8ull * NPL, kb);
  else
    load32(hs + 64, kb);
  hmac_key_le(kb, J, Jo);
  jr_part_header(c, LEADER ? 0u : 1u, nonce, hv);
  if (!LEADER) {
    uint32_t km[8], ist[8], ost[8], tag[8];
    load32(hs, km);
    hmac_key_le(km, ist, ost);
    Msg128 m;
    m_zero(m);
    const int pos = m_prefix(m, c.dst_id, USAGE_MEAS);
    m_byte(m, pos, 1);  // binder: agg_id
    hmac_tag(tag, ist, ost, m, pos + 1);
    Ctr sm;
    ctr_init(sm, T, tag);
    jr_part_inner(
        c, J, hv,
        [&](uint32_t, uint32_t K[16]) {
#pragma unroll
          for (int a = 0; a < 4; a++) ctr_next(sm, T, K + 4 * a);
        },
        [&](uint32_t q, const uint32_t K[16]) {
#pragma unroll
          for (int i = 0; i < 8; i++) {
            const uint32_t e = 8 * q + i;
            if (e < M) {
              bad |= ge_p64(K[2 * i], K[2 * i + 1]);
              emit64(c, mp, op, e, K[2 * i], K[2 * i + 1], tr);
            }
          }
        });
  } else {
    jr_part_inner(
        c, J, hv,
        [&](uint32_t q, uint32_t K[16]) {
#pragma unroll
          for (int i = 0; i < 8; i++) {
            const uint32_t e = 8 * q + i;
            const uint2 v = e < M ? *reinterpret_cast<const uint2*>(ls + 8ull * e) : make_uint2(0, 0);
            K[2 * i] = v.x;
            K[2 * i + 1] = v.y;
          }
        },
        [&](uint32_t q, const uint32_t K[16]) {
#pragma unroll
          for (int i = 0; i < 8; i++) {
            const uint32_t e = 8 * q + i;
            if (e < M) {
              bad |= ge_p64(K[2 * i], K[2 * i + 1]);
              emit64(c, mp, op, e, K[2 * i], K[2 * i + 1], tr);
            }
          }
        });
  }
  uint32_t own[8];
  {
    uint32_t tag[8];
    hmac_outer_c(tag, Jo, J);
    ctr_seed(T, tag, own);
  }
  // ---- proofs share: expand(k_proofs, DST(2), [PROOFS, agg_id], PROOFS * PROOF_LEN)
  uint2* const pp = reinterpret_cast<uint2*>(b.proof) + (blk * NPL) * IL + lane;
  if (!LEADER) {
    uint32_t kp[8], ist[8], ost[8], tag[8];
    load32(hs + 32, kp);
    hmac_key_le(kp, ist, ost);
    Msg128 m;
    m_zero(m);
    const int pos = m_prefix(m, c.dst_id, USAGE_PROOF);
    m_byte(m, pos, c.np);
    m_byte(m, pos + 1, 1);
    hmac_tag(tag, ist, ost, m, pos + 2);
    Ctr sp;
    ctr_init(sp, T, tag);
#pragma unroll 1
    for (uint32_t e = 0; e < NPL; e += 2) {
      uint32_t ks[4];
      ctr_next(sp, T, ks);
      bad |= ge_p64(ks[0], ks[1]);
      pp[(uint64_t)e * IL] = make_uint2(ks[0], ks[1]);
      if (e + 1 < NPL) {
        bad |= ge_p64(ks[2], ks[3]);
        pp[(uint64_t)(e + 1) * IL] = make_uint2(ks[2], ks[3]);
      }
    }
  } else {
#pragma unroll 1
    for (uint32_t e = 0; e < NPL; e++) {
      const uint2 v = *reinterpret_cast<const uint2*>(ls + MB + 8ull * e);
      bad |= ge_p64(v.x, v.y);
      pp[(uint64_t)e * IL] = v;
    }
  }
  if (!LEADER && bad) {  // a rejected sample shifted a stream: the slow kernel redoes this report
    if (r0 < b.n) b.flags[r0] = FLAG_SLOW;
    return;
  }
  uint32_t flags = bad ? FLAG_INPUT_FAIL : 0u;
  if (LEADER && r0 < b.n) {  // the leader's joint_rand_part closes its prep share
    uint2* o = reinterpret_cast<uint2*>(b.lps_out + (uint64_t)c.lps_bytes * r + 8ull * c.np * c.ver_len);
#pragma unroll
    for (int i = 0; i < 4; i++) o[i] = make_uint2(own[2 * i], own[2 * i + 1]);
  }
  flags = mp_tail(c, b, T, blk, lane, r, r0 < b.n, nonce, own, flags, LEADER);
  if (r0 < b.n) b.flags[r0] = flags;
}

// ---------------------------------------------------------------------------- K1' (helper)
// Exact recomputation with rejection sampling for the reports K1 flagged (or all, force_slow).
__global__ __launch_bounds__(64) void mp_slow_kernel(Cfg c, Bufs b) {
  __shared__ uint32_t tt[TT_WORDS];
  const uint32_t lane = threadIdx.x;
  const uint64_t blk = blockIdx.x;
  const uint64_t r = blk * 64 + lane;
  const bool mine = r < b.n && (b.flags[r] & FLAG_SLOW) != 0;
  if (__ballot(mine) == 0) return;  // wave-uniform: the whole workgroup leaves
  tt_fill(tt);
  __syncthreads();
  if (!mine) return;
  const TTab T = ttab(tt, lane);
  const uint32_t M = c.meas_len, NPL = c.np * c.proof_len;
  const uint8_t* hs = b.his + (uint64_t)c.his_bytes * r;
  uint2* const mp = reinterpret_cast<uint2*>(b.meas) + (blk * M) * IL + lane;
  uint4* const op = b.outs + (blk * c.out_len) * IL + lane;
  uint2* const pp = reinterpret_cast<uint2*>(b.proof) + (blk * NPL) * IL + lane;
  uint32_t nonce[4];
  load16(b.nonces + 16 * r, nonce);
  // streams with rejection: next accepted element
  auto stream = [&](uint32_t usage, const uint8_t* key, uint32_t binder_len, uint2* dst, uint32_t n, bool meas) {
    uint32_t k[8], ist[8], ost[8], tag[8];
    load32(key, k);
    hmac_key_le(k, ist, ost);
    Msg128 m;
    m_zero(m);
    const int pos = m_prefix(m, c.dst_id, usage);
    if (binder_len == 1) {
      m_byte(m, pos, 1);
    } else {
      m_byte(m, pos, c.np);
      m_byte(m, pos + 1, 1);
    }
    hmac_tag(tag, ist, ost, m, pos + (int)binder_len);
    Ctr s;
    ctr_init(s, T, tag);
    TruncF64 tr{0, 0, 0, 0};
    uint32_t ks[4] = {0, 0, 0, 0}, h = 2;
    for (uint32_t e = 0; e < n; e++) {
      uint32_t lo, hi;
      do {
        if (h == 2) {
          ctr_next(s, T, ks);
          h = 0;
        }
        lo = h == 0 ? ks[0] : ks[2];
        hi = h == 0 ? ks[1] : ks[3];
        h++;
      } while (ge_p64(lo, hi));
      if (meas)
        emit64(c, dst, op, e, lo, hi, tr);
      else
        dst[(uint64_t)e * IL] = make_uint2(lo, hi);
    }
  };
  stream(USAGE_MEAS, hs, 1, mp, M, true);
  stream(USAGE_PROOF, hs + 32, 2, pp, NPL, false);
  // joint_rand_part over the share just written
  uint32_t kb[8], J[8], Jo[8], hv[7];
  load32(hs + 64, kb);
  hmac_key_le(kb, J, Jo);
  jr_part_header(c, 1, nonce, hv);
  jr_part_inner(
      c, J, hv,
      [&](uint32_t q, uint32_t K[16]) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const uint32_t e = 8 * q + i;
          const uint2 v = e < M ? mp[(uint64_t)e * IL] : make_uint2(0, 0);
          K[2 * i] = v.x;
          K[2 * i + 1] = v.y;
        }
      },
      [](uint32_t, const uint32_t*) {});
  uint32_t own[8];
  {
    uint32_t tag[8];
    hmac_outer_c(tag, Jo, J);
    ctr_seed(T, tag, own);
  }
  b.flags[r] = mp_tail(c, b, T, blk, lane, r, true, nonce, own, 0u, false);
}

// ---------------------------------------------------------------------------- K3
__device__ __forceinline__ uint64_t ld_lead64(const Bufs& b, const Cfg& c, uint64_t r, uint32_t idx, bool& dfail) {
  const uint2 v = *reinterpret_cast<const uint2*>(b.lps + (uint64_t)c.lps_bytes * r + 8ull * idx);
  dfail |= ge_p64(v.x, v.y);
  return u2v(v);
}

// One wave per (64-report block, group of PPW chunk slots, pair of proofs): the measurement
// elements are read once for both proofs (the share is the kernel's dominant HBM stream). For its
// slots and proofs it forms the wire sums E = sum_k d_k x_{k,i} and O = sum_k c_k x_{k,i} as limb
// column sums, the wires at t (leader: written into its prep share), sum_i Ve_i Vo_i over the slots
// with the leader's shares added (helper), and its share of v = sum_m g_m S_m and of G(t).
template <int PPW, bool LEADER>
__global__ __launch_bounds__(64, 3) void mp_flp_part_kernel(Cfg c, Bufs b) {
  constexpr int NPW = 2;
  const uint32_t NG = c.ngroups, NP = c.np, NPG = (NP + NPW - 1) / NPW, U = NG * NPG;
  // XCD-aware: the U waves of one block run back to back on one XCD (shared L2 for the
  // coefficients and the leader's share)
  const uint32_t bid = blockIdx.x;
  const uint32_t xcd = bid & 7u, q = bid >> 3;
  const uint32_t u = q % U;
  const uint64_t blk = (uint64_t)(q / U) * 8 + xcd;
  const uint64_t nblk = (b.n + 63) / 64;
  if (blk >= nblk) return;
  const uint32_t g = u % NG, p0 = (u / NG) * NPW;
  const bool two = p0 + 1 < NP;  // wave-uniform
  const uint32_t lane = threadIdx.x;
  const uint64_t r0 = blk * 64 + lane;
  const uint64_t r = r0 < b.n ? r0 : b.n - 1;
  const uint32_t C = c.calls, chunk = c.chunk, M = c.meas_len, A = 2 * chunk, PL = c.proof_len, VL = c.ver_len;
  const uint32_t j0 = g * PPW;
  const uint2* coefb[NPW];
#pragma unroll
  for (int w = 0; w < NPW; w++)
    coefb[w] = reinterpret_cast<const uint2*>(b.coef) + ((blk * NP + min(p0 + w, NP - 1)) * c.nco) * IL + lane;
  const uint2* measb = reinterpret_cast<const uint2*>(b.meas) + (blk * M) * IL + lane;

  wacc64 ae[NPW][PPW], ao[NPW][PPW];
  uint64_t E[NPW][PPW], O[NPW][PPW];
#pragma unroll
  for (int w = 0; w < NPW; w++)
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      wacc64_zero(ae[w][i]);
      wacc64_zero(ao[w][i]);
      E[w][i] = 0;
      O[w][i] = 0;
    }
  auto fold = [&]() {
#pragma unroll
    for (int w = 0; w < NPW; w++)
#pragma unroll
      for (int i = 0; i < PPW; i++) {
        E[w][i] = add64(E[w][i], wacc64_reduce(ae[w][i]));
        O[w][i] = add64(O[w][i], wacc64_reduce(ao[w][i]));
        wacc64_zero(ae[w][i]);
        wacc64_zero(ao[w][i]);
      }
  };
  auto ldc = [&](int w, uint32_t k, bool d) -> uint2 {
    return coefb[w][(uint64_t)(MCOEF_K + 2 * (k - 1) + (d ? 1 : 0)) * IL];
  };
  // calls whose PPW slots are all real measurement elements run branch-free
  uint32_t kf = 0;
  if (j0 + PPW <= chunk && M >= j0 + PPW) kf = min(C, (M - j0 - PPW) / chunk + 1);
  for (uint32_t k0 = 1; k0 <= kf; k0 += WACC64_MAX_TERMS) {
    const uint32_t k1 = min(kf, k0 + WACC64_MAX_TERMS - 1);
    uint2 cn[NPW], dn[NPW], xn[PPW];
#pragma unroll
    for (int w = 0; w < NPW; w++) {
      cn[w] = ldc(w, k0, false);
      dn[w] = ldc(w, k0, true);
    }
#pragma unroll
    for (int i = 0; i < PPW; i++) xn[i] = measb[(uint64_t)((k0 - 1) * chunk + j0 + i) * IL];
#pragma unroll 1
    for (uint32_t k = k0; k <= k1; k++) {
      c64limbs ck[NPW], dk[NPW];
#pragma unroll
      for (int w = 0; w < NPW; w++) {
        ck[w] = to_c64limbs(u2v(cn[w]));
        dk[w] = to_c64limbs(u2v(dn[w]));
      }
      uint64_t x[PPW];
#pragma unroll
      for (int i = 0; i < PPW; i++) x[i] = u2v(xn[i]);
      if (k < k1) {  // software pipeline: call k + 1's loads in flight during call k's products
#pragma unroll
        for (int w = 0; w < NPW; w++) {
          cn[w] = ldc(w, k + 1, false);
          dn[w] = ldc(w, k + 1, true);
        }
#pragma unroll
        for (int i = 0; i < PPW; i++) xn[i] = measb[(uint64_t)(k * chunk + j0 + i) * IL];
      }
#pragma unroll
      for (int w = 0; w < NPW; w++)
#pragma unroll
        for (int i = 0; i < PPW; i++) {
          wacc64_mac(ae[w][i], x[i], dk[w]);
          wacc64_mac(ao[w][i], x[i], ck[w]);
        }
    }
    fold();
  }
#pragma unroll 1
  for (uint32_t k = kf + 1; k <= C; k++) {  // the ragged last call(s), or every call of a padded group
    const uint32_t nb = (k - 1) * chunk + j0;
#pragma unroll
    for (int w = 0; w < NPW; w++) {
      const c64limbs ck = to_c64limbs(u2v(ldc(w, k, false))), dk = to_c64limbs(u2v(ldc(w, k, true)));
#pragma unroll
      for (int i = 0; i < PPW; i++) {
        if (j0 + i < chunk && nb + i < M) {
          const uint64_t x = u2v(measb[(uint64_t)(nb + i) * IL]);
          wacc64_mac(ae[w][i], x, dk);
          wacc64_mac(ao[w][i], x, ck);
        }
      }
    }
    if (((k - kf) % WACC64_MAX_TERMS) == 0) fold();
  }
  fold();
  bool dfail = false;
  const uint32_t GL = c.gpoly_len;
  const uint32_t per = (GL + NG - 1) / NG;
  const uint32_t m0 = g * per, m1 = min(GL, m0 + per);
  const uint4* Sm = b.consts + c.c_S;
#pragma unroll
  for (int w = 0; w < NPW; w++) {
    if (w == 1 && !two) break;
    const uint32_t p = p0 + w;
    const uint2* cb = coefb[w];
    const uint2* proofb = reinterpret_cast<const uint2*>(b.proof) + (blk * NP * PL + (uint64_t)p * PL) * IL + lane;
    // ---- wires at t for this group's slots
    const uint64_t L = u2v(cb[MCOEF_L * IL]), c0 = u2v(cb[MCOEF_C0 * IL]);
    const uint64_t hsum = u2v(cb[MCOEF_HALFSUM * IL]), t = u2v(cb[MCOEF_T * IL]);
    const uint64_t rr = u2v(cb[MCOEF_R * IL]);
    uint64_t prod = 0;
    uint64_t rpow = pow64_h(rr, j0 + 1);
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      const uint32_t j = j0 + i;
      if (j < chunk) {
        const uint64_t se = u2v(proofb[(uint64_t)(2 * j) * IL]), so = u2v(proofb[(uint64_t)(2 * j + 1) * IL]);
        const uint64_t We = mul64(add64(mul64(se, c0), mul64(E[w][i], rpow)), L);
        const uint64_t Wo = mul64(sub64(add64(mul64(so, c0), O[w][i]), hsum), L);
        rpow = mul64(rpow, rr);
        if (LEADER) {
          if (r0 < b.n) {
            uint2* o = reinterpret_cast<uint2*>(b.lps_out + (uint64_t)c.lps_bytes * r);
            o[(uint64_t)p * VL + 1 + 2 * j] = v2u(We);
            o[(uint64_t)p * VL + 2 + 2 * j] = v2u(Wo);
          }
        } else {
          const uint64_t Ve = add64(We, ld_lead64(b, c, r, p * VL + 1 + 2 * j, dfail));
          const uint64_t Vo = add64(Wo, ld_lead64(b, c, r, p * VL + 2 + 2 * j, dfail));
          prod = add64(prod, mul64(Ve, Vo));
        }
      }
    }
    // ---- gadget polynomial over this group's coefficient range
    uint64_t vpart = 0, gpart = 0;
    if (m0 < m1) {
      for (uint32_t m = m1; m-- > m0;) {
        const uint64_t gm = u2v(proofb[(uint64_t)(A + m) * IL]);
        vpart = add64(vpart, mul64(gm, (uint64_t)Sm[m].x | ((uint64_t)Sm[m].y << 32)));
        gpart = add64(mul64(gpart, t), gm);
      }
      gpart = mul64(gpart, pow64_h(t, m0));
    }
    uint2* pp = reinterpret_cast<uint2*>(b.part) + (((blk * NP + p) * NG + g) * 3) * IL + lane;
    pp[0] = v2u(prod);
    pp[IL] = v2u(vpart);
    pp[2 * IL] = v2u(gpart);
  }
  if (dfail && r0 < b.n) atomicOr(&b.flags[r0], FLAG_DFAIL);
}

template <bool LEADER>
__global__ __launch_bounds__(256) void mp_flp_final_kernel(Cfg c, Bufs b) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= b.n) return;
  const uint64_t blk = r / 64;
  const uint32_t lane = r % 64, NG = c.ngroups, NP = c.np, A = 2 * c.chunk, VL = c.ver_len;
  const uint32_t flags = b.flags[r];
  bool df = (flags & FLAG_DFAIL) != 0, ok = true;
  for (uint32_t p = 0; p < NP; p++) {
    uint64_t P = 0, V = 0, G = 0;
    const uint2* pp = reinterpret_cast<const uint2*>(b.part) + (((blk * NP + p) * NG) * 3) * IL + lane;
    for (uint32_t g = 0; g < NG; g++, pp += 3 * IL) {
      P = add64(P, u2v(pp[0]));
      V = add64(V, u2v(pp[IL]));
      G = add64(G, u2v(pp[2 * IL]));
    }
    if (LEADER) {  // verifier share [v, wires(t)..., G(t)] of proof p
      uint2* o = reinterpret_cast<uint2*>(b.lps_out + (uint64_t)c.lps_bytes * r);
      o[(uint64_t)p * VL] = v2u(V);
      o[(uint64_t)p * VL + A + 1] = v2u(G);
    } else {
      const uint64_t lv = ld_lead64(b, c, r, p * VL, df), lg = ld_lead64(b, c, r, p * VL + A + 1, df);
      if (add64(V, lv) != 0 || P != add64(G, lg)) ok = false;
    }
  }
  uint32_t verdict;
  if (LEADER) {
    verdict = (flags & (FLAG_INIT_FAIL | FLAG_INPUT_FAIL)) ? 1u : 0u;
  } else if (flags & FLAG_INIT_FAIL) {
    verdict = 1;
  } else if (df) {
    verdict = 2;
  } else if (!ok) {
    verdict = 3;
  } else {
    verdict = (flags & FLAG_NEXT_FAIL) ? 4u : 0u;
  }
  b.verdicts[r] = (uint8_t)verdict;
}

inline uint32_t nblk_of(uint64_t n) { return (uint32_t)((n + 63) / 64); }

template <int PPW, bool LEADER>
void launch_mp_flp_r(const Cfg& c, const Bufs& b, hipStream_t s) {
  const uint32_t nb = nblk_of(b.n);
  const uint32_t grid = ((nb + 7) / 8) * 8 * c.ngroups * ((c.np + 1) / 2);
  hipLaunchKernelGGL((mp_flp_part_kernel<PPW, LEADER>), dim3(grid), dim3(64), 0, s, c, b);
  hipLaunchKernelGGL((mp_flp_final_kernel<LEADER>), dim3((uint32_t)((b.n + 255) / 256)), dim3(256), 0, s, c, b);
}

}  // namespace

hipError_t launch_mp_xof(const Cfg& c, const Bufs& b, hipStream_t s) {
  const uint32_t nb = nblk_of(b.n);
  if (b.leader)
    hipLaunchKernelGGL(mp_xof_kernel<true>, dim3((nb + MP_XOF_WAVES - 1) / MP_XOF_WAVES), dim3(64 * MP_XOF_WAVES), 0, s,
                       c, b);
  else
    hipLaunchKernelGGL(mp_xof_kernel<false>, dim3((nb + MP_XOF_WAVES - 1) / MP_XOF_WAVES), dim3(64 * MP_XOF_WAVES), 0,
                       s, c, b);
  return hipGetLastError();
}

uint64_t mp_k1_round_reports(int device) {
  int cus = 0, wgs = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&wgs, mp_xof_kernel<false>, 64 * MP_XOF_WAVES, 0) != hipSuccess ||
      wgs <= 0)
    return 0;
  return (uint64_t)cus * (uint64_t)wgs * 64u * MP_XOF_WAVES;
}

hipError_t launch_mp_slow(const Cfg& c, const Bufs& b, hipStream_t s) {
  hipLaunchKernelGGL(mp_slow_kernel, dim3(nblk_of(b.n)), dim3(64), 0, s, c, b);
  return hipGetLastError();
}

hipError_t launch_mp_flp(const Cfg& c, const Bufs& b, hipStream_t s) {
  if (c.ppw == 2) {
    if (b.leader)
      launch_mp_flp_r<2, true>(c, b, s);
    else
      launch_mp_flp_r<2, false>(c, b, s);
  } else if (c.ppw == 1) {
    if (b.leader)
      launch_mp_flp_r<1, true>(c, b, s);
    else
      launch_mp_flp_r<1, false>(c, b, s);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace jx
