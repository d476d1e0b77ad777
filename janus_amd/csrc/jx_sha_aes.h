// jx_sha_aes.h — SHA-256 / HMAC-SHA256 and AES-128 building blocks shared by the batched HPKE
// open (jx_hpke.hip) and the XofHmacSha256Aes128 Prio3 path (jx_mp64.hip). __host__ __device__ so
// that tests/csrc/hosttest.cpp checks them on the CPU against the test oracles.
#pragma once
#include "jx_sha256.h"

namespace jx {

// ============================================================================ SHA-256 / HMAC

// a message of up to 128 bytes following a 64-byte prefix already absorbed into the state
// (HMAC's key block); bytes are written big-endian into 32 words at compile-time positions
struct Msg128 {
  uint32_t w[32];
};
JX_HD void m_zero(Msg128& m) {
#pragma unroll
  for (int i = 0; i < 32; i++) m.w[i] = 0;
}
JX_HD void m_byte(Msg128& m, int pos, uint32_t v) { m.w[pos >> 2] |= (v & 0xffu) << (24 - 8 * (pos & 3)); }
JX_HD int m_str(Msg128& m, int pos, const char* s) {  // string literal (compile-time)
  for (int i = 0; s[i]; i++) m_byte(m, pos++, (uint8_t)s[i]);
  return pos;
}
// 32 bytes held as 8 little-endian memory words
JX_HD int m_le32(Msg128& m, int pos, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 32; i++) m_byte(m, pos + i, w[i >> 2] >> (8 * (i & 3)));
  return pos + 32;
}
// 32 bytes held as 8 big-endian words (a SHA-256 digest)
JX_HD int m_be32(Msg128& m, int pos, const uint32_t h[8]) {
#pragma unroll
  for (int i = 0; i < 32; i++) m_byte(m, pos + i, h[i >> 2] >> (24 - 8 * (i & 3)));
  return pos + 32;
}

constexpr uint32_t SHA256_IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

JX_HD void sha256_compress(uint32_t st[8], const uint32_t* blk) {  // 16 big-endian words
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = xor3(ror32(w15, 7), ror32(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(ror32(w2, 17), ror32(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = xor3(ror32(e, 6), ror32(e, 11), ror32(e, 25));
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA256_K[i] + wi;
    uint32_t S0 = xor3(ror32(a, 2), ror32(a, 13), ror32(a, 22));
    uint32_t mj = maj3(a, b, c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// finish a hash whose state st already absorbed one 64-byte block: message m of len bytes
JX_HD void sha256_finish64(uint32_t out[8], const uint32_t st0[8], Msg128& m, int len) {
  m_byte(m, len, 0x80);
  const int nblk = (len + 9 + 63) / 64;  // 1 or 2
  const uint64_t bits = 8ull * (64 + len);
  m.w[nblk * 16 - 2] = (uint32_t)(bits >> 32);
  m.w[nblk * 16 - 1] = (uint32_t)bits;
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = st0[i];
  sha256_compress(out, m.w);
  if (nblk == 2) sha256_compress(out, m.w + 16);
}

// HMAC-SHA256 key pads for a 32-byte key given as 8 big-endian words (RFC 2104)
JX_HD void hmac_pads(const uint32_t key[8], uint32_t ist[8], uint32_t ost[8]) {
  uint32_t bi[16], bo[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t k = i < 8 ? key[i] : 0u;
    bi[i] = k ^ 0x36363636u;
    bo[i] = k ^ 0x5c5c5c5cu;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    ist[i] = SHA256_IV[i];
    ost[i] = SHA256_IV[i];
  }
  sha256_compress(ist, bi);
  sha256_compress(ost, bo);
}
// HMAC outer hash over an inner digest
JX_HD void hmac_outer(uint32_t out[8], const uint32_t ost[8], const uint32_t inner[8]) {
  Msg128 m;
  m_zero(m);
  m_be32(m, 0, inner);
  sha256_finish64(out, ost, m, 32);
}

// ============================================================================ AES-128 / GCM

// round keys: 44 words, word = 4 bytes little-endian (byte 0 in bits 0..7)
JX_HD uint32_t sub_word(const uint8_t* sbox, uint32_t w) {
  return (uint32_t)sbox[w & 0xff] | ((uint32_t)sbox[(w >> 8) & 0xff] << 8) | ((uint32_t)sbox[(w >> 16) & 0xff] << 16) |
         ((uint32_t)sbox[w >> 24] << 24);
}
JX_HD void aes128_expand_key(const uint8_t* sbox, const uint32_t key[4], uint32_t rk[44]) {
#pragma unroll
  for (int i = 0; i < 4; i++) rk[i] = key[i];
  uint32_t rcon = 1;
#pragma unroll
  for (int i = 4; i < 44; i++) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = sub_word(sbox, (t >> 8) | (t << 24)) ^ rcon;
      rcon = (rcon << 1) ^ ((rcon >> 7) * 0x11bu);
    }
    rk[i] = rk[i - 4] ^ t;
  }
}
JX_HD uint32_t xtime4(uint32_t x) { return ((x & 0x7f7f7f7fu) << 1) ^ (((x >> 7) & 0x01010101u) * 0x1bu); }
// one 16-byte block as 4 little-endian column words
JX_HD void aes128_encrypt(const uint8_t* sbox, const uint32_t rk[44], const uint32_t in[4], uint32_t out[4]) {
  uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
  for (int r = 1; r <= 10; r++) {
    // SubBytes + ShiftRows: row i of column c comes from column (c + i) mod 4
    uint32_t t0 = (uint32_t)sbox[s0 & 0xff] | ((uint32_t)sbox[(s1 >> 8) & 0xff] << 8) |
                  ((uint32_t)sbox[(s2 >> 16) & 0xff] << 16) | ((uint32_t)sbox[s3 >> 24] << 24);
    uint32_t t1 = (uint32_t)sbox[s1 & 0xff] | ((uint32_t)sbox[(s2 >> 8) & 0xff] << 8) |
                  ((uint32_t)sbox[(s3 >> 16) & 0xff] << 16) | ((uint32_t)sbox[s0 >> 24] << 24);
    uint32_t t2 = (uint32_t)sbox[s2 & 0xff] | ((uint32_t)sbox[(s3 >> 8) & 0xff] << 8) |
                  ((uint32_t)sbox[(s0 >> 16) & 0xff] << 16) | ((uint32_t)sbox[s1 >> 24] << 24);
    uint32_t t3 = (uint32_t)sbox[s3 & 0xff] | ((uint32_t)sbox[(s0 >> 8) & 0xff] << 8) |
                  ((uint32_t)sbox[(s1 >> 16) & 0xff] << 16) | ((uint32_t)sbox[s2 >> 24] << 24);
    if (r != 10) {  // MixColumns: b_i = 2(a_i ^ a_{i+1}) ^ a_{i+1} ^ a_{i+2} ^ a_{i+3}
      uint32_t c[4] = {t0, t1, t2, t3};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t w = c[q];
        const uint32_t r1 = (w >> 8) | (w << 24), r2 = (w >> 16) | (w << 16), r3 = (w >> 24) | (w << 8);
        c[q] = xtime4(w ^ r1) ^ r1 ^ r2 ^ r3;
      }
      t0 = c[0];
      t1 = c[1];
      t2 = c[2];
      t3 = c[3];
    }
    s0 = t0 ^ rk[4 * r];
    s1 = t1 ^ rk[4 * r + 1];
    s2 = t2 ^ rk[4 * r + 2];
    s3 = t3 ^ rk[4 * r + 3];
  }
  out[0] = s0;
  out[1] = s1;
  out[2] = s2;
  out[3] = s3;
}

// FIPS 197 S-box
constexpr uint8_t AES_SBOX[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82, 0xc9,
    0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f,
    0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, 0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07,
    0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3,
    0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58,
    0xcf, 0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3,
    0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec, 0x5f,
    0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73, 0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88,
    0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac,
    0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a,
    0xae, 0x08, 0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, 0x70,
    0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11,
    0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, 0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42,
    0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

// ---------------------------------------------------------------------------- AES-128, T-table form
// The XOF stream kernels encrypt thousands of counter blocks per lane. They use one 1 KiB table
// T0[x] = (2s, s, s, 3s) (s = S[x], rows 0..3 of a little-endian column word), replicated 32 times
// in LDS so that lane l always reads copy l mod 32 (its own ds_read_b32 bank: conflict-free), and
// the rotations T1..T3 = rotl(T0, 8/16/24). TL is any callable x -> T0[x].

JX_HD uint32_t aes_xtime(uint32_t s) { return ((s << 1) ^ ((s >> 7) * 0x1bu)) & 0xffu; }
JX_HD uint32_t aes_t0_entry(uint32_t s) {
  const uint32_t s2 = aes_xtime(s);
  return s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
}
JX_HD uint32_t rotl32(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

template <class TL>
JX_HD uint32_t aes_sub_word_t(const TL& T, uint32_t w) {
  return ((T(w & 0xffu) >> 8) & 0xffu) | (T((w >> 8) & 0xffu) & 0xff00u) | ((T((w >> 16) & 0xffu) & 0xff00u) << 8) |
         ((T(w >> 24) & 0xff00u) << 16);
}
template <class TL>
JX_HD void aes128_expand_key_t(const TL& T, const uint32_t key[4], uint32_t rk[44]) {
#pragma unroll
  for (int i = 0; i < 4; i++) rk[i] = key[i];
  uint32_t rcon = 1;
#pragma unroll
  for (int i = 4; i < 44; i++) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = aes_sub_word_t(T, (t >> 8) | (t << 24)) ^ rcon;
      rcon = aes_xtime(rcon);
    }
    rk[i] = rk[i - 4] ^ t;
  }
}
// one block; state and round keys as little-endian column words
template <class TL>
JX_HD void aes128_encrypt_t(const TL& T, const uint32_t rk[44], const uint32_t in[4], uint32_t out[4]) {
  uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
  for (int r = 1; r < 10; r++) {
    // column c: row i comes from column (c + i) mod 4 (ShiftRows), then SubBytes + MixColumns
    const uint32_t t0 = T(s0 & 0xffu) ^ rotl32(T((s1 >> 8) & 0xffu), 8) ^ rotl32(T((s2 >> 16) & 0xffu), 16) ^
                        rotl32(T(s3 >> 24), 24) ^ rk[4 * r];
    const uint32_t t1 = T(s1 & 0xffu) ^ rotl32(T((s2 >> 8) & 0xffu), 8) ^ rotl32(T((s3 >> 16) & 0xffu), 16) ^
                        rotl32(T(s0 >> 24), 24) ^ rk[4 * r + 1];
    const uint32_t t2 = T(s2 & 0xffu) ^ rotl32(T((s3 >> 8) & 0xffu), 8) ^ rotl32(T((s0 >> 16) & 0xffu), 16) ^
                        rotl32(T(s1 >> 24), 24) ^ rk[4 * r + 2];
    const uint32_t t3 = T(s3 & 0xffu) ^ rotl32(T((s0 >> 8) & 0xffu), 8) ^ rotl32(T((s1 >> 16) & 0xffu), 16) ^
                        rotl32(T(s2 >> 24), 24) ^ rk[4 * r + 3];
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  // last round: SubBytes + ShiftRows only; S[x] is byte 1 of T0[x]
  out[0] = (((T(s0 & 0xffu) >> 8) & 0xffu) | (T((s1 >> 8) & 0xffu) & 0xff00u) |
            ((T((s2 >> 16) & 0xffu) & 0xff00u) << 8) | ((T(s3 >> 24) & 0xff00u) << 16)) ^ rk[40];
  out[1] = (((T(s1 & 0xffu) >> 8) & 0xffu) | (T((s2 >> 8) & 0xffu) & 0xff00u) |
            ((T((s3 >> 16) & 0xffu) & 0xff00u) << 8) | ((T(s0 >> 24) & 0xff00u) << 16)) ^ rk[41];
  out[2] = (((T(s2 & 0xffu) >> 8) & 0xffu) | (T((s3 >> 8) & 0xffu) & 0xff00u) |
            ((T((s0 >> 16) & 0xffu) & 0xff00u) << 8) | ((T(s1 >> 24) & 0xff00u) << 16)) ^ rk[42];
  out[3] = (((T(s3 & 0xffu) >> 8) & 0xffu) | (T((s0 >> 8) & 0xffu) & 0xff00u) |
            ((T((s1 >> 16) & 0xffu) & 0xff00u) << 8) | ((T(s2 >> 24) & 0xff00u) << 16)) ^ rk[43];
}

// one block with the key schedule computed on the fly (for one-off blocks: no 44-word schedule
// held in registers)
template <class TL>
JX_HD void aes128_encrypt_t_otf(const TL& T, const uint32_t key[4], const uint32_t in[4], uint32_t out[4]) {
  uint32_t k0 = key[0], k1 = key[1], k2 = key[2], k3 = key[3];
  uint32_t s0 = in[0] ^ k0, s1 = in[1] ^ k1, s2 = in[2] ^ k2, s3 = in[3] ^ k3;
  uint32_t rcon = 1;
#pragma unroll
  for (int r = 1; r <= 10; r++) {
    k0 ^= aes_sub_word_t(T, (k3 >> 8) | (k3 << 24)) ^ rcon;
    k1 ^= k0;
    k2 ^= k1;
    k3 ^= k2;
    rcon = aes_xtime(rcon);
    uint32_t t0, t1, t2, t3;
    if (r < 10) {
      t0 = T(s0 & 0xffu) ^ rotl32(T((s1 >> 8) & 0xffu), 8) ^ rotl32(T((s2 >> 16) & 0xffu), 16) ^ rotl32(T(s3 >> 24), 24);
      t1 = T(s1 & 0xffu) ^ rotl32(T((s2 >> 8) & 0xffu), 8) ^ rotl32(T((s3 >> 16) & 0xffu), 16) ^ rotl32(T(s0 >> 24), 24);
      t2 = T(s2 & 0xffu) ^ rotl32(T((s3 >> 8) & 0xffu), 8) ^ rotl32(T((s0 >> 16) & 0xffu), 16) ^ rotl32(T(s1 >> 24), 24);
      t3 = T(s3 & 0xffu) ^ rotl32(T((s0 >> 8) & 0xffu), 8) ^ rotl32(T((s1 >> 16) & 0xffu), 16) ^ rotl32(T(s2 >> 24), 24);
    } else {
      t0 = ((T(s0 & 0xffu) >> 8) & 0xffu) | (T((s1 >> 8) & 0xffu) & 0xff00u) | ((T((s2 >> 16) & 0xffu) & 0xff00u) << 8) |
           ((T(s3 >> 24) & 0xff00u) << 16);
      t1 = ((T(s1 & 0xffu) >> 8) & 0xffu) | (T((s2 >> 8) & 0xffu) & 0xff00u) | ((T((s3 >> 16) & 0xffu) & 0xff00u) << 8) |
           ((T(s0 >> 24) & 0xff00u) << 16);
      t2 = ((T(s2 & 0xffu) >> 8) & 0xffu) | (T((s3 >> 8) & 0xffu) & 0xff00u) | ((T((s0 >> 16) & 0xffu) & 0xff00u) << 8) |
           ((T(s1 >> 24) & 0xff00u) << 16);
      t3 = ((T(s3 & 0xffu) >> 8) & 0xffu) | (T((s0 >> 8) & 0xffu) & 0xff00u) | ((T((s1 >> 16) & 0xffu) & 0xff00u) << 8) |
           ((T(s2 >> 24) & 0xff00u) << 16);
    }
    s0 = t0 ^ k0;
    s1 = t1 ^ k1;
    s2 = t2 ^ k2;
    s3 = t3 ^ k3;
  }
  out[0] = s0;
  out[1] = s1;
  out[2] = s2;
  out[3] = s3;
}

// big-endian message word from bytes 2..5 of the little-endian word pair (lo, hi): the 26-byte
// XOF header shifts the measurement bytes by 2 within SHA-256 words (one v_perm_b32)
JX_HD uint32_t be_word_shift16(uint32_t lo, uint32_t hi) { return bswap32((lo >> 16) | (hi << 16)); }

}  // namespace jx
