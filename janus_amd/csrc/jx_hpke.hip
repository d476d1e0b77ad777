// jx_hpke.hip — batched HPKE open of report shares on the GPU.
//
// Replaces the per-report `hpke::open(&helper_keypair, &HpkeApplicationInfo::new(
// &Label::InputShare, &Role::Client, &Role::Helper), encrypted_input_share, &input_share_aad)`
// of the helper's aggregate-init loop (aggregator/src/aggregator.rs:1772-1832; core/src/hpke.rs:
// 200-230): RFC 9180 base mode, DHKEM(X25519, HKDF-SHA256), HKDF-SHA256, AES-128-GCM. One
// report per lane: X25519 decapsulation, the HKDF key schedule, AES-128-GCM open.
//
// Two kernels:
//  - hpke_open_kernel: the standalone batch open of include/jx_hpke.h (caller's ciphertexts and AADs);
//  - hpke_rows_kernel: the open INSIDE a helper prepare launch (jx_helper_prep_encrypted_batch, alone or
//    coalesced): per report it builds the InputShareAad from the report's task id, id, time and public share
//    rows, tries the task's and then the global keypair (aggregator.rs:1807-1820), decodes the
//    PlaintextInputShare and checks its extensions (:1834-1893) and writes the payload into the helper
//    input-share row K1 reads, with one status byte per report (include/jx_prio3.h, JX_OPEN_*).
// C ABI in include/jx_hpke.h; the rows kernel's launcher is internal (jx_engine_internal.h).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/jx_hpke.h"
#include "jx_engine_internal.h"
#include "jx_hpke.h"

using namespace jx;

namespace {

struct HpkeCfg {
  HpkeKeyRow key;          // clamped recipient scalar, public key, key_schedule_context
  uint32_t zero_ist[8];    // HMAC-SHA256 pads of the empty salt (LabeledExtract with salt "")
  uint32_t zero_ost[8];
};

struct HpkeBufs {
  uint64_t n;
  const uint8_t* encs;
  const uint8_t* cts;
  const uint64_t* ct_off;
  const uint8_t* aads;
  const uint64_t* aad_off;
  uint8_t* pts;
  uint8_t* ok;
};

// HPKE suite ids: "KEM" || 0x0020 and "HPKE" || 0x0020 || 0x0001 || 0x0001
JX_HD int m_suite_kem(Msg128& m, int pos) {
  pos = m_str(m, pos, "KEM");
  m_byte(m, pos, 0x00);
  m_byte(m, pos + 1, 0x20);
  return pos + 2;
}
JX_HD int m_suite(Msg128& m, int pos) {
  pos = m_str(m, pos, "HPKE");
  const uint8_t ids[6] = {0x00, 0x20, 0x00, 0x01, 0x00, 0x01};
  for (int i = 0; i < 6; i++) m_byte(m, pos + i, ids[i]);
  return pos + 6;
}

// LabeledExpand(secret, label, ksc, L) for L <= 32: HMAC(secret, I2OSP(L,2) || "HPKE-v1" ||
// suite || label || ksc || 0x01)
JX_HD void expand_ksc(uint32_t out[8], const uint32_t ist[8], const uint32_t ost[8], int L, const char* label,
                      const uint8_t* ksc) {
  Msg128 m;
  m_zero(m);
  m_byte(m, 0, 0);
  m_byte(m, 1, L);
  int pos = m_str(m, 2, "HPKE-v1");
  pos = m_suite(m, pos);
  pos = m_str(m, pos, label);
  for (int i = 0; i < 65; i++) m_byte(m, pos + i, ksc[i]);
  pos += 65;
  m_byte(m, pos, 1);
  uint32_t inner[8];
  sha256_finish64(inner, ist, m, pos + 1);
  hmac_outer(out, ost, inner);
}

JX_HD uint8_t ld_byte(const uint8_t* p, uint64_t i, uint64_t n) { return i < n ? p[i] : 0; }
JX_HD void ld_block_be(const uint8_t* p, uint64_t n, uint32_t b[4]) {  // up to 16 bytes, zero padded
  for (int w = 0; w < 4; w++) {
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) v = (v << 8) | ld_byte(p, 4 * w + k, n);
    b[w] = v;
  }
}

// The AES-128-GCM context of one recipient key for encapsulated key `enc` (8 LE words): DHKEM decap
// (RFC 9180 §4.1), the mode_base key schedule (§5.1), the round keys, the hash key H (4 BE words) and the
// base nonce (3 BE words). False when the DH output is all zero (a low-order point: the open fails).
__device__ bool hpke_context(const uint8_t* sbox, const HpkeKeyRow& key, const uint32_t zist[8], const uint32_t zost[8],
                             const uint32_t enc[8], uint32_t rk[44], uint32_t h[4], uint32_t nonce3[3]) {
  uint32_t dh[8];
  x25519_ladder(dh, key.sk, enc);
  uint32_t nz = 0;
  for (int i = 0; i < 8; i++) nz |= dh[i];
  uint32_t eae_prk[8], ss[8], secret[8], kk[8], nonce[8];
  {
    Msg128 m;
    m_zero(m);
    int pos = m_str(m, 0, "HPKE-v1");
    pos = m_suite_kem(m, pos);
    pos = m_str(m, pos, "eae_prk");
    pos = m_le32(m, pos, dh);
    uint32_t inner[8];
    sha256_finish64(inner, zist, m, pos);
    hmac_outer(eae_prk, zost, inner);
  }
  {
    uint32_t ist[8], ost[8];
    hmac_pads(eae_prk, ist, ost);
    Msg128 m;
    m_zero(m);
    m_byte(m, 0, 0);
    m_byte(m, 1, 32);
    int pos = m_str(m, 2, "HPKE-v1");
    pos = m_suite_kem(m, pos);
    pos = m_str(m, pos, "shared_secret");
    pos = m_le32(m, pos, enc);
    pos = m_le32(m, pos, key.pk);
    m_byte(m, pos, 1);
    uint32_t inner[8];
    sha256_finish64(inner, ist, m, pos + 1);
    hmac_outer(ss, ost, inner);
  }
  {
    uint32_t ist[8], ost[8];
    hmac_pads(ss, ist, ost);
    Msg128 m;
    m_zero(m);
    int pos = m_str(m, 0, "HPKE-v1");
    pos = m_suite(m, pos);
    pos = m_str(m, pos, "secret");
    uint32_t inner[8];
    sha256_finish64(inner, ist, m, pos);
    hmac_outer(secret, ost, inner);
  }
  {
    uint32_t ist[8], ost[8];
    hmac_pads(secret, ist, ost);
    expand_ksc(kk, ist, ost, 16, "key", key.ksc);
    expand_ksc(nonce, ist, ost, 12, "base_nonce", key.ksc);
  }
  uint32_t kw[4], hblk[4], zero4[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4; i++) kw[i] = bswap32(kk[i]);  // digest bytes 0..15 as LE words
  aes128_expand_key(sbox, kw, rk);
  aes128_encrypt(sbox, rk, zero4, hblk);
  for (int i = 0; i < 4; i++) h[i] = bswap32(hblk[i]);
  for (int i = 0; i < 3; i++) nonce3[i] = bswap32(nonce[i]);
  return nz != 0;
}

// GCM tag check of ciphertext ct[0, clen) with tag ct[clen, clen + 16) and associated data produced 16
// bytes at a time by aad_block(i, w) (alen bytes): GHASH, then E(J0) ^ S == tag.
template <class AadBlock>
__device__ bool gcm_tag_ok(const uint8_t* sbox, const uint32_t rk[44], const uint32_t h[4], const uint32_t nonce3[3],
                           uint64_t alen, AadBlock aad_block, const uint8_t* ct, uint64_t clen) {
  uint32_t y[4] = {0, 0, 0, 0};
  for (uint64_t i = 0; i < alen; i += 16) {
    uint32_t x[4];
    aad_block(i, x);
    for (int k = 0; k < 4; k++) y[k] ^= x[k];
    ghash_mul(y, h);
  }
  for (uint64_t i = 0; i < clen; i += 16) {
    uint32_t x[4];
    ld_block_be(ct + i, clen - i, x);
    for (int k = 0; k < 4; k++) y[k] ^= x[k];
    ghash_mul(y, h);
  }
  y[0] ^= (uint32_t)((8 * alen) >> 32);
  y[1] ^= (uint32_t)(8 * alen);
  y[2] ^= (uint32_t)((8 * clen) >> 32);
  y[3] ^= (uint32_t)(8 * clen);
  ghash_mul(y, h);
  // counter blocks: nonce (12 bytes) || BE32 counter; J0 has counter 1
  uint32_t cb[4] = {nonce3[0], nonce3[1], nonce3[2], bswap32(1u)}, ks[4];
  aes128_encrypt(sbox, rk, cb, ks);
  uint32_t diff = 0;
  for (int k = 0; k < 4; k++) {
    uint32_t tag_w = 0;
    for (int q = 0; q < 4; q++) tag_w = (tag_w << 8) | ld_byte(ct + clen, 4 * k + q, 16);
    diff |= (bswap32(ks[k]) ^ y[k]) ^ tag_w;
  }
  return diff == 0;
}

// CTR decryption of ct[0, clen) into pt (counter blocks from 2)
__device__ void gcm_decrypt(const uint8_t* sbox, const uint32_t rk[44], const uint32_t nonce3[3], const uint8_t* ct,
                            uint64_t clen, uint8_t* pt) {
  uint32_t cb[4] = {nonce3[0], nonce3[1], nonce3[2], 0}, ks[4];
  for (uint64_t i = 0; i < clen; i += 16) {
    cb[3] = bswap32((uint32_t)(2 + i / 16));
    aes128_encrypt(sbox, rk, cb, ks);
    for (uint64_t j = 0; j < 16 && i + j < clen; j++) pt[i + j] = ct[i + j] ^ (uint8_t)(ks[j >> 2] >> (8 * (j & 3)));
  }
}

__device__ void load_enc(const uint8_t* p, uint32_t enc[8]) {
  for (int i = 0; i < 8; i++)
    enc[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
             ((uint32_t)p[4 * i + 3] << 24);
}

__global__ __launch_bounds__(64) void hpke_open_kernel(HpkeCfg cfg, HpkeBufs b) {
  __shared__ uint8_t sbox[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) sbox[i] = AES_SBOX[i];
  __syncthreads();
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= b.n) return;
  uint32_t enc[8], rk[44], h[4], nonce3[3];
  load_enc(b.encs + 32 * r, enc);
  const bool nz = hpke_context(sbox, cfg.key, cfg.zero_ist, cfg.zero_ost, enc, rk, h, nonce3);
  const uint64_t c0 = b.ct_off[r], c1 = b.ct_off[r + 1];
  const uint64_t a0 = b.aad_off[r], a1 = b.aad_off[r + 1];
  bool ok = nz && c1 - c0 >= 16;
  const uint64_t clen = ok ? c1 - c0 - 16 : 0, alen = a1 - a0;
  const uint8_t* ct = b.cts + c0;
  const uint8_t* aad = b.aads + a0;
  ok = ok && gcm_tag_ok(sbox, rk, h, nonce3, alen, [&](uint64_t i, uint32_t x[4]) { ld_block_be(aad + i, alen - i, x); },
                        ct, clen);
  if (ok) gcm_decrypt(sbox, rk, nonce3, ct, clen, b.pts + c0 - 16 * r);
  b.ok[r] = (uint8_t)ok;
}

// ---------------------------------------------------------------------------- open inside a prepare launch

struct RowsArgs {
  HpkeRowsArgs a;
  uint32_t zero_ist[8], zero_ost[8];
};

// byte i of the InputShareAad (messages/src/lib.rs:1854-1858): task_id (32) || report id (16) || time (8, BE)
// || u32 BE length of the public share || the public share
__device__ uint8_t aad_byte(const EncRow& e, const uint8_t* nonce, const uint8_t* ps, uint32_t ps_bytes, uint64_t i) {
  if (i < 32) return e.task_id[i];
  if (i < 48) return nonce[i - 32];
  if (i < 56) return e.time_be[i - 48];
  if (i < 60) return (uint8_t)(ps_bytes >> (8 * (59 - i)));
  return i - 60 < ps_bytes ? ps[i - 60] : 0;
}

__global__ __launch_bounds__(64) void hpke_rows_kernel(RowsArgs ra) {
  __shared__ uint8_t sbox[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) sbox[i] = AES_SBOX[i];
  __syncthreads();
  const HpkeRowsArgs& a = ra.a;
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  const EncRow& e = a.rows[r];
  if (!(e.flags & ENC_ROW_ENCRYPTED)) {  // a plain report of the launch: its helper input share was uploaded
    a.status[r] = JX_OPEN_OK;
    return;
  }
  uint8_t* his = a.his + (uint64_t)a.his_bytes * r;
  uint32_t st = JX_OPEN_OK;
  const uint64_t c0 = e.ct_off, clen_all = e.ct_len;
  const uint8_t* ct = a.cts + c0;
  uint8_t* pt = a.pts + c0;
  const uint64_t clen = clen_all >= 16 ? clen_all - 16 : 0;
  if (e.key0 == JX_KEY_NONE) {
    st = JX_OPEN_UNKNOWN_CONFIG;  // neither the task nor the global keys hold the config id
  } else if ((e.flags & ENC_ROW_MALFORMED) || clen_all < 16) {
    st = JX_OPEN_HPKE_DECRYPT_ERROR;  // an encapsulated key that is not 32 bytes, a ciphertext without a tag
  } else {
    uint32_t enc[8];
    load_enc(e.enc, enc);
    const uint8_t* nonce = a.nonces + 16 * r;
    const uint8_t* ps = a.ps + (uint64_t)a.ps_bytes * r;
    const uint64_t alen = 60 + a.ps_bytes;
    bool ok = false;
    // the task's keypair first, then the global one (aggregator.rs:1807-1820): a second trial only when the
    // first fails to decrypt
    for (int t = 0; t < 2 && !ok; t++) {
      const uint32_t kidx = t == 0 ? e.key0 : e.key1;
      if (kidx >= a.nkeys) break;
      uint32_t rk[44], h[4], nonce3[3];
      const bool nz = hpke_context(sbox, a.keys[kidx], ra.zero_ist, ra.zero_ost, enc, rk, h, nonce3);
      ok = nz && gcm_tag_ok(sbox, rk, h, nonce3, alen,
                            [&](uint64_t i, uint32_t x[4]) {
                              for (int w = 0; w < 4; w++) {
                                uint32_t v = 0;
                                for (int k = 0; k < 4; k++) {
                                  const uint64_t j = i + 4 * w + k;
                                  v = (v << 8) | (j < alen ? aad_byte(e, nonce, ps, a.ps_bytes, j) : 0u);
                                }
                                x[w] = v;
                              }
                            },
                            ct, clen);
      if (ok) gcm_decrypt(sbox, rk, nonce3, ct, clen, pt);
    }
    if (!ok) st = JX_OPEN_HPKE_DECRYPT_ERROR;
  }
  uint64_t pay = 0, plen = 0;
  if (st == JX_OPEN_OK) {
    // PlaintextInputShare (messages/src/lib.rs:1323-1326): u16-prefixed extensions, u32-prefixed payload,
    // nothing after it; an extension is type u16 (TBD 0x0000 or Taskprov 0xFF00, else a decode error) || u16-
    // prefixed data
    const uint64_t L = clen;
    if (L < 2) {
      st = JX_OPEN_PLAINTEXT_DECODE_FAILURE;
    } else {
      const uint64_t end = 2 + (((uint32_t)pt[0] << 8) | pt[1]);
      uint32_t n_tbd = 0, n_tp = 0, tp_len = 0;
      if (end > L) st = JX_OPEN_PLAINTEXT_DECODE_FAILURE;
      for (uint64_t i = 2; st == JX_OPEN_OK && i < end;) {  // advances >= 4 bytes per extension
        if (i + 4 > end) {
          st = JX_OPEN_PLAINTEXT_DECODE_FAILURE;
          break;
        }
        const uint32_t t = ((uint32_t)pt[i] << 8) | pt[i + 1], dl = ((uint32_t)pt[i + 2] << 8) | pt[i + 3];
        if ((t != 0x0000u && t != 0xFF00u) || i + 4 + dl > end) {
          st = JX_OPEN_PLAINTEXT_DECODE_FAILURE;
          break;
        }
        if (t == 0) {
          n_tbd++;
        } else {
          n_tp++;
          tp_len = dl;
        }
        i += 4 + dl;
      }
      if (st == JX_OPEN_OK) {
        if (end + 4 > L) {
          st = JX_OPEN_PLAINTEXT_DECODE_FAILURE;
        } else {
          plen = ((uint64_t)pt[end] << 24) | ((uint64_t)pt[end + 1] << 16) | ((uint64_t)pt[end + 2] << 8) | pt[end + 3];
          pay = end + 4;
          if (pay + plen != L) st = JX_OPEN_PLAINTEXT_DECODE_FAILURE;
        }
      }
      const bool req = (e.flags & ENC_ROW_REQUIRE_TASKPROV) != 0;
      if (st == JX_OPEN_OK && (n_tbd > 1 || n_tp > 1))
        st = JX_OPEN_DUPLICATE_EXTENSION;  // aggregator.rs:1852-1867
      else if (st == JX_OPEN_OK && req && !(n_tp == 1 && tp_len == 0))
        st = JX_OPEN_MISSING_TASKPROV;  // :1869-1879
      else if (st == JX_OPEN_OK && !req && n_tp)
        st = JX_OPEN_UNEXPECTED_TASKPROV;  // :1880-1890
      if (st == JX_OPEN_OK && plen != a.his_bytes) st = JX_OPEN_INPUT_SHARE_DECODE_FAILURE;  // :1895-1910
    }
  }
  // the helper input share K1 reads (zeros for a failed report: prepared, then masked by launch_open_mask)
  for (uint32_t i = 0; i < a.his_bytes; i++) his[i] = st == JX_OPEN_OK ? pt[pay + i] : 0;
  a.status[r] = (uint8_t)st;
}

__global__ __launch_bounds__(256) void open_mask_kernel(const uint8_t* status, uint8_t* verdicts, uint64_t n) {
  const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (r < n && status[r] != JX_OPEN_OK) verdicts[r] = JX_OPEN_FAILURE;
}

}  // namespace

struct jx_hpke {
  HpkeCfg cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  jxi::Arena* arena = nullptr;  // the device's arena: the host-buffer open's device buffers
  std::mutex mu;                // one call at a time per handle (its stream and staging)
};

// errors: per calling thread (jx_hpke_last_error)
static thread_local std::string t_hpke_err;

static int32_t hfail(int32_t code, const std::string& m) {
  t_hpke_err = m;
  return code;
}
#define HCHK(call)                                                                                   \
  do {                                                                                               \
    hipError_t _st = (call);                                                                         \
    if (_st != hipSuccess) return hfail(JX_HPKE_E_HIP, std::string(#call) + ": " + hipGetErrorString(_st)); \
  } while (0)

// host HMAC-SHA256 over arbitrary short messages (configuration only)
static void host_hmac(const uint8_t* key, size_t klen, const std::vector<uint8_t>& msg, uint8_t out[32]) {
  auto sha = [](const std::vector<uint8_t>& data, uint8_t dig[32]) {
    uint32_t st[8];
    for (int i = 0; i < 8; i++) st[i] = SHA256_IV[i];
    std::vector<uint8_t> d = data;
    const uint64_t bits = 8ull * data.size();
    d.push_back(0x80);
    while (d.size() % 64 != 56) d.push_back(0);
    for (int i = 7; i >= 0; i--) d.push_back((uint8_t)(bits >> (8 * i)));
    for (size_t o = 0; o < d.size(); o += 64) {
      uint32_t w[16];
      for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)d[o + 4 * i] << 24) | ((uint32_t)d[o + 4 * i + 1] << 16) | ((uint32_t)d[o + 4 * i + 2] << 8) |
               d[o + 4 * i + 3];
      sha256_compress(st, w);
    }
    for (int i = 0; i < 8; i++)
      for (int k = 0; k < 4; k++) dig[4 * i + k] = (uint8_t)(st[i] >> (24 - 8 * k));
  };
  uint8_t kb[64] = {0};
  memcpy(kb, key, klen);
  std::vector<uint8_t> in(64), outer(64);
  for (int i = 0; i < 64; i++) {
    in[i] = kb[i] ^ 0x36;
    outer[i] = kb[i] ^ 0x5c;
  }
  in.insert(in.end(), msg.begin(), msg.end());
  uint8_t ih[32];
  sha(in, ih);
  outer.insert(outer.end(), ih, ih + 32);
  sha(outer, out);
}

namespace jxi {

int hpke_device(const jx_hpke* h) { return h->device; }
void hpke_key_row(const jx_hpke* h, HpkeKeyRow* out) { *out = h->cfg.key; }

hipError_t launch_hpke_rows(const HpkeRowsArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  RowsArgs ra;
  ra.a = a;
  const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  hmac_pads(zero, ra.zero_ist, ra.zero_ost);
  hipLaunchKernelGGL(hpke_rows_kernel, dim3((uint32_t)((a.n + 63) / 64)), dim3(64), 0, s, ra);
  return hipGetLastError();
}

hipError_t launch_open_mask(const uint8_t* status, uint8_t* verdicts, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(open_mask_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, status, verdicts, n);
  return hipGetLastError();
}

}  // namespace jxi

extern "C" {

int32_t jx_hpke_create(const uint8_t sk[32], const uint8_t pk[32], const uint8_t* info, uint32_t info_len,
                       int32_t device, jx_hpke** out) {
  if (!sk || !pk || !out || (info_len && !info)) return JX_HPKE_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return JX_HPKE_E_NODEVICE;
  if (device < 0 || device >= ndev) return JX_HPKE_E_INVALID;
  jx_hpke* h = new jx_hpke();
  h->device = device;
  uint8_t k[32];
  memcpy(k, sk, 32);
  k[0] &= 248;
  k[31] &= 127;
  k[31] |= 64;
  for (int i = 0; i < 8; i++) {
    memcpy(&h->cfg.key.sk[i], k + 4 * i, 4);
    memcpy(&h->cfg.key.pk[i], pk + 4 * i, 4);
  }
  const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  hmac_pads(zero, h->cfg.zero_ist, h->cfg.zero_ost);
  // key_schedule_context = mode_base || LabeledExtract("", "psk_id_hash", "") || LabeledExtract("", "info_hash", info)
  const char* ver = "HPKE-v1";
  const uint8_t suite[10] = {'H', 'P', 'K', 'E', 0x00, 0x20, 0x00, 0x01, 0x00, 0x01};
  auto labeled = [&](const char* label, const uint8_t* ikm, size_t n, uint8_t o[32]) {
    std::vector<uint8_t> msg(ver, ver + 7);
    msg.insert(msg.end(), suite, suite + 10);
    msg.insert(msg.end(), label, label + strlen(label));
    msg.insert(msg.end(), ikm, ikm + n);
    host_hmac(nullptr, 0, msg, o);
  };
  h->cfg.key.ksc[0] = 0;
  labeled("psk_id_hash", nullptr, 0, h->cfg.key.ksc + 1);
  labeled("info_hash", info, info_len, h->cfg.key.ksc + 33);
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return JX_HPKE_E_HIP;
  }
  h->arena = jxi::arena_for(device);
  *out = h;
  return JX_HPKE_OK;
}

void jx_hpke_destroy(jx_hpke* h) {
  if (!h) return;
  if (h->stream) {
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    (void)hipStreamDestroy(h->stream);
  }
  delete h;
}

int32_t jx_hpke_open_batch_device(jx_hpke* h, uint64_t n, const void* d_encs, const void* d_cts,
                                  const uint64_t* d_ct_offsets, const void* d_aads, const uint64_t* d_aad_offsets,
                                  void* d_out_plaintexts, void* d_out_ok) {
  if (!h || (n && (!d_encs || !d_cts || !d_ct_offsets || !d_aad_offsets || !d_out_plaintexts || !d_out_ok))) {
    return JX_HPKE_E_INVALID;
  }
  if (n == 0) return JX_HPKE_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  HCHK(hipSetDevice(h->device));
  HpkeBufs b{n,
             (const uint8_t*)d_encs,
             (const uint8_t*)d_cts,
             d_ct_offsets,
             (const uint8_t*)d_aads,
             d_aad_offsets,
             (uint8_t*)d_out_plaintexts,
             (uint8_t*)d_out_ok};
  hipLaunchKernelGGL(hpke_open_kernel, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, h->stream, h->cfg, b);
  HCHK(hipGetLastError());
  return JX_HPKE_OK;
}

// Host buffers: one staging slab from the device's arena (no per-call hipMalloc / hipFree, which would wait
// for the whole device), handed back stream-ordered; only this handle's stream is synchronized.
int32_t jx_hpke_open_batch(jx_hpke* h, uint64_t n, const uint8_t* encs, const uint8_t* cts,
                           const uint64_t* ct_offsets, const uint8_t* aads, const uint64_t* aad_offsets,
                           uint8_t* out_plaintexts, uint8_t* out_ok) {
  if (!h || (n && (!encs || !cts || !ct_offsets || !aad_offsets || !out_plaintexts || !out_ok)))
    return JX_HPKE_E_INVALID;
  if (n == 0) return JX_HPKE_OK;
  for (uint64_t i = 0; i < n; i++)
    if (ct_offsets[i + 1] < ct_offsets[i] + 16 || aad_offsets[i + 1] < aad_offsets[i])
      return hfail(JX_HPKE_E_INVALID, "offsets must be non-decreasing and every ciphertext >= 16 bytes");
  std::lock_guard<std::mutex> lk(h->mu);
  HCHK(hipSetDevice(h->device));
  const uint64_t ct_bytes = ct_offsets[n], aad_bytes = aad_offsets[n], pt_bytes = ct_bytes - 16 * n;
  const size_t o_enc = 0, o_ct = o_enc + jxi::align256(n * 32), o_aad = o_ct + jxi::align256(ct_bytes),
               o_pt = o_aad + jxi::align256(aad_bytes ? aad_bytes : 1), o_ok = o_pt + jxi::align256(pt_bytes ? pt_bytes : 1),
               o_co = o_ok + jxi::align256(n), o_ao = o_co + jxi::align256((n + 1) * 8), bytes = o_ao + jxi::align256((n + 1) * 8);
  jxi::Slab slab;
  const hipError_t ga = jxi::arena_get(h->arena, bytes, h->stream, true, true, slab);
  if (ga == hipErrorOutOfMemory) return hfail(JX_HPKE_E_NOMEM, "device allocation failed (arena)");
  HCHK(ga);
  uint8_t* base = (uint8_t*)slab.p;
  int32_t rc = JX_HPKE_OK;
  do {
    if (hipMemcpyAsync(base + o_enc, encs, n * 32, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        hipMemcpyAsync(base + o_ct, cts, ct_bytes, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        (aad_bytes && hipMemcpyAsync(base + o_aad, aads, aad_bytes, hipMemcpyHostToDevice, h->stream) != hipSuccess) ||
        hipMemcpyAsync(base + o_co, ct_offsets, (n + 1) * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        hipMemcpyAsync(base + o_ao, aad_offsets, (n + 1) * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess) {
      rc = hfail(JX_HPKE_E_HIP, "host-to-device copy failed");
      break;
    }
    HpkeBufs b{n, base + o_enc, base + o_ct, (const uint64_t*)(base + o_co), base + o_aad, (const uint64_t*)(base + o_ao),
               base + o_pt, base + o_ok};
    hipLaunchKernelGGL(hpke_open_kernel, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, h->stream, h->cfg, b);
    if (hipGetLastError() != hipSuccess) {
      rc = hfail(JX_HPKE_E_HIP, "kernel launch failed");
      break;
    }
    if ((pt_bytes && hipMemcpyAsync(out_plaintexts, base + o_pt, pt_bytes, hipMemcpyDeviceToHost, h->stream) != hipSuccess) ||
        hipMemcpyAsync(out_ok, base + o_ok, n, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess) {
      rc = hfail(JX_HPKE_E_HIP, "device-to-host copy failed");
      break;
    }
  } while (0);
  jxi::arena_put(h->arena, slab, h->stream);  // reused after this stream's work
  return rc;
}

const char* jx_hpke_last_error(const jx_hpke* h) {
  (void)h;
  return t_hpke_err.c_str();
}

}  // extern "C"
