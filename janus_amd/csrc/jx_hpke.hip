// jx_hpke.hip — batched HPKE open of report shares on the GPU.
//
// Replaces the per-report `hpke::open(&helper_keypair, &HpkeApplicationInfo::new(
// &Label::InputShare, &Role::Client, &Role::Helper), encrypted_input_share, &input_share_aad)`
// of the helper's aggregate-init loop (aggregator/src/aggregator.rs:1772-1832; core/src/hpke.rs:
// 200-230): RFC 9180 base mode, DHKEM(X25519, HKDF-SHA256), HKDF-SHA256, AES-128-GCM. One
// report per lane: X25519 decapsulation, the HKDF key schedule, AES-128-GCM open.
// C ABI in include/jx_hpke.h.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/jx_hpke.h"
#include "jx_hpke.h"

using namespace jx;

namespace {

struct HpkeCfg {
  uint32_t sk[8];          // clamped recipient scalar, LE words
  uint32_t pk[8];          // recipient public key, LE words
  uint32_t zero_ist[8];    // HMAC-SHA256 pads of the empty salt (LabeledExtract with salt "")
  uint32_t zero_ost[8];
  uint8_t ksc[68];         // key_schedule_context = 0x00 || psk_id_hash || info_hash (65 bytes)
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

__global__ __launch_bounds__(64) void hpke_open_kernel(HpkeCfg cfg, HpkeBufs b) {
  __shared__ uint8_t sbox[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) sbox[i] = AES_SBOX[i];
  __syncthreads();
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= b.n) return;

  // ---- DHKEM(X25519, HKDF-SHA256) Decap (RFC 9180 §4.1)
  uint32_t enc[8], dh[8];
  for (int i = 0; i < 8; i++) {
    const uint8_t* p = b.encs + 32 * r + 4 * i;
    enc[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
  }
  x25519_ladder(dh, cfg.sk, enc);
  uint32_t nz = 0;
  for (int i = 0; i < 8; i++) nz |= dh[i];
  uint32_t eae_prk[8], ss[8], secret[8], key[8], nonce[8];
  {
    Msg128 m;
    m_zero(m);
    int pos = m_str(m, 0, "HPKE-v1");
    pos = m_suite_kem(m, pos);
    pos = m_str(m, pos, "eae_prk");
    pos = m_le32(m, pos, dh);
    uint32_t inner[8];
    sha256_finish64(inner, cfg.zero_ist, m, pos);
    hmac_outer(eae_prk, cfg.zero_ost, inner);
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
    pos = m_le32(m, pos, cfg.pk);
    m_byte(m, pos, 1);
    uint32_t inner[8];
    sha256_finish64(inner, ist, m, pos + 1);
    hmac_outer(ss, ost, inner);
  }
  // ---- KeySchedule, mode_base (RFC 9180 §5.1)
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
    expand_ksc(key, ist, ost, 16, "key", cfg.ksc);
    expand_ksc(nonce, ist, ost, 12, "base_nonce", cfg.ksc);
  }
  // ---- AES-128-GCM open (sequence number 0: nonce = base_nonce)
  uint32_t kw[4], rk[44];
  for (int i = 0; i < 4; i++) kw[i] = bswap32(key[i]);  // digest bytes 0..15 as LE words
  aes128_expand_key(sbox, kw, rk);
  uint32_t hblk[4], zero4[4] = {0, 0, 0, 0}, h[4];
  aes128_encrypt(sbox, rk, zero4, hblk);
  for (int i = 0; i < 4; i++) h[i] = bswap32(hblk[i]);
  const uint64_t c0 = b.ct_off[r], c1 = b.ct_off[r + 1];
  const uint64_t a0 = b.aad_off[r], a1 = b.aad_off[r + 1];
  uint32_t ok = nz != 0 && c1 - c0 >= 16;
  const uint64_t clen = ok ? c1 - c0 - 16 : 0, alen = a1 - a0;
  const uint8_t* ct = b.cts + c0;
  const uint8_t* aad = b.aads + a0;
  uint32_t y[4] = {0, 0, 0, 0};
  for (uint64_t i = 0; i < alen; i += 16) {
    uint32_t x[4];
    ld_block_be(aad + i, alen - i, x);
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
  const uint32_t n0 = bswap32(nonce[0]), n1 = bswap32(nonce[1]), n2 = bswap32(nonce[2]);
  uint32_t cb[4] = {n0, n1, n2, bswap32(1u)}, ks[4];
  aes128_encrypt(sbox, rk, cb, ks);
  uint32_t diff = 0;
  for (int k = 0; k < 4; k++) {
    uint32_t tag_w = 0;
    for (int q = 0; q < 4; q++) tag_w = (tag_w << 8) | ld_byte(ct + clen, 4 * k + q, 16);
    diff |= (bswap32(ks[k]) ^ y[k]) ^ tag_w;
  }
  ok = ok && diff == 0;
  uint8_t* pt = b.pts + c0 - 16 * r;
  if (ok) {
    for (uint64_t i = 0; i < clen; i += 16) {
      cb[3] = bswap32((uint32_t)(2 + i / 16));
      aes128_encrypt(sbox, rk, cb, ks);
      for (uint64_t j = 0; j < 16 && i + j < clen; j++)
        pt[i + j] = ct[i + j] ^ (uint8_t)(ks[j >> 2] >> (8 * (j & 3)));
    }
  }
  b.ok[r] = (uint8_t)ok;
}

}  // namespace

struct jx_hpke {
  HpkeCfg cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
};

static int32_t hfail(jx_hpke* h, int32_t code, const std::string& m) {
  if (h) h->err = m;
  return code;
}
#define HCHK(h, call)                                                                                 \
  do {                                                                                                \
    hipError_t _st = (call);                                                                          \
    if (_st != hipSuccess) return hfail((h), JX_HPKE_E_HIP, std::string(#call) + ": " + hipGetErrorString(_st)); \
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
    memcpy(&h->cfg.sk[i], k + 4 * i, 4);
    memcpy(&h->cfg.pk[i], pk + 4 * i, 4);
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
  h->cfg.ksc[0] = 0;
  labeled("psk_id_hash", nullptr, 0, h->cfg.ksc + 1);
  labeled("info_hash", info, info_len, h->cfg.ksc + 33);
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return JX_HPKE_E_HIP;
  }
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
  HCHK(h, hipSetDevice(h->device));
  HpkeBufs b{n,
             (const uint8_t*)d_encs,
             (const uint8_t*)d_cts,
             d_ct_offsets,
             (const uint8_t*)d_aads,
             d_aad_offsets,
             (uint8_t*)d_out_plaintexts,
             (uint8_t*)d_out_ok};
  hipLaunchKernelGGL(hpke_open_kernel, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, h->stream, h->cfg, b);
  HCHK(h, hipGetLastError());
  return JX_HPKE_OK;
}

int32_t jx_hpke_open_batch(jx_hpke* h, uint64_t n, const uint8_t* encs, const uint8_t* cts,
                           const uint64_t* ct_offsets, const uint8_t* aads, const uint64_t* aad_offsets,
                           uint8_t* out_plaintexts, uint8_t* out_ok) {
  if (!h || (n && (!encs || !cts || !ct_offsets || !aad_offsets || !out_plaintexts || !out_ok)))
    return JX_HPKE_E_INVALID;
  if (n == 0) return JX_HPKE_OK;
  for (uint64_t i = 0; i < n; i++)
    if (ct_offsets[i + 1] < ct_offsets[i] + 16 || aad_offsets[i + 1] < aad_offsets[i])
      return hfail(h, JX_HPKE_E_INVALID, "offsets must be non-decreasing and every ciphertext >= 16 bytes");
  HCHK(h, hipSetDevice(h->device));
  const uint64_t ct_bytes = ct_offsets[n], aad_bytes = aad_offsets[n], pt_bytes = ct_bytes - 16 * n;
  uint8_t *d_encs = nullptr, *d_cts = nullptr, *d_aads = nullptr, *d_pts = nullptr, *d_ok = nullptr;
  uint64_t *d_co = nullptr, *d_ao = nullptr;
  auto cleanup = [&]() {
    for (void* p : {(void*)d_encs, (void*)d_cts, (void*)d_aads, (void*)d_pts, (void*)d_ok, (void*)d_co, (void*)d_ao})
      if (p) (void)hipFree(p);
  };
  int32_t rc = JX_HPKE_OK;
  do {
    if (hipMalloc(&d_encs, n * 32) != hipSuccess || hipMalloc(&d_cts, ct_bytes ? ct_bytes : 1) != hipSuccess ||
        hipMalloc(&d_aads, aad_bytes ? aad_bytes : 1) != hipSuccess ||
        hipMalloc(&d_pts, pt_bytes ? pt_bytes : 1) != hipSuccess || hipMalloc(&d_ok, n) != hipSuccess ||
        hipMalloc(&d_co, (n + 1) * 8) != hipSuccess || hipMalloc(&d_ao, (n + 1) * 8) != hipSuccess) {
      rc = hfail(h, JX_HPKE_E_NOMEM, "device allocation failed");
      break;
    }
    if (hipMemcpyAsync(d_encs, encs, n * 32, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        hipMemcpyAsync(d_cts, cts, ct_bytes, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        (aad_bytes && hipMemcpyAsync(d_aads, aads, aad_bytes, hipMemcpyHostToDevice, h->stream) != hipSuccess) ||
        hipMemcpyAsync(d_co, ct_offsets, (n + 1) * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        hipMemcpyAsync(d_ao, aad_offsets, (n + 1) * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess) {
      rc = hfail(h, JX_HPKE_E_HIP, "host-to-device copy failed");
      break;
    }
    rc = jx_hpke_open_batch_device(h, n, d_encs, d_cts, d_co, d_aads, d_ao, d_pts, d_ok);
    if (rc) break;
    if (hipMemcpyAsync(out_plaintexts, d_pts, pt_bytes, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipMemcpyAsync(out_ok, d_ok, n, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess) {
      rc = hfail(h, JX_HPKE_E_HIP, "device-to-host copy failed");
      break;
    }
  } while (0);
  (void)hipStreamSynchronize(h->stream);
  cleanup();
  return rc;
}

const char* jx_hpke_last_error(const jx_hpke* h) { return h ? h->err.c_str() : ""; }

}  // extern "C"
