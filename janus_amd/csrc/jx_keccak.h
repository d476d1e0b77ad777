// jx_keccak.h — Keccak-p[1600,12] / TurboSHAKE128 sponge for one report per lane.
//
// Replaces the keccak 0.1.4 `p1600(state, 12)` that prio 0.16.1's XofTurboShake128
// drives (Cargo.lock:2537,4252). The 1600-bit state lives in
// 50 VGPRs as (lo, hi) 32-bit halves of the 25 lanes; 64-bit rotations are two
// v_alignbit_b32, theta's 5-way XOR and chi's a^(~b&c) lower to v_bitop3_b32 on
// gfx950. Rounds are fully unrolled inside: every state index is a compile-time
// constant, so nothing spills to scratch.
#pragma once
#include "jx_field.h"

namespace jx {

#if defined(__HIP_DEVICE_COMPILE__)
JX_HD uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbit(hi, lo, s); }
#else
JX_HD uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
}
#endif

// rotate the 64-bit lane (lo, hi) left by N (compile-time)
template <int N>
JX_HD void rotl64(uint32_t& lo, uint32_t& hi) {
  if constexpr (N == 0) {
    return;
  } else if constexpr (N < 32) {
    uint32_t nh = alignbit(hi, lo, 32 - N);
    uint32_t nl = alignbit(lo, hi, 32 - N);
    lo = nl;
    hi = nh;
  } else if constexpr (N == 32) {
    uint32_t t = lo;
    lo = hi;
    hi = t;
  } else {
    constexpr int M = N - 32;
    uint32_t nh = alignbit(lo, hi, 32 - M);
    uint32_t nl = alignbit(hi, lo, 32 - M);
    lo = nl;
    hi = nh;
  }
}

// rho offsets r[x + 5y]
#define JX_ROT_LIST 0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14

template <int I>
struct RotOf {
  static constexpr int table[25] = {JX_ROT_LIST};
  static constexpr int value = table[I];
};

// pi: B[y + 5*((2x+3y)%5)] = rot(A[x+5y])
template <int I>
struct PiDst {
  static constexpr int x = I % 5, y = I / 5;
  static constexpr int value = y + 5 * ((2 * x + 3 * y) % 5);
};

constexpr uint32_t KECCAK_RC_LO[24] = {
    0x00000001u, 0x00008082u, 0x0000808Au, 0x80008000u, 0x0000808Bu, 0x80000001u, 0x80008081u, 0x00008009u,
    0x0000008Au, 0x00000088u, 0x80008009u, 0x8000000Au, 0x8000808Bu, 0x0000008Bu, 0x00008089u, 0x00008003u,
    0x00008002u, 0x00000080u, 0x0000800Au, 0x8000000Au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
constexpr uint32_t KECCAK_RC_HI[24] = {
    0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u,
    0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u,
    0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};

template <int I>
JX_HD void rho_pi_one(const uint32_t* A, uint32_t* B) {
  uint32_t lo = A[2 * I], hi = A[2 * I + 1];
  rotl64<RotOf<I>::value>(lo, hi);
  B[2 * PiDst<I>::value] = lo;
  B[2 * PiDst<I>::value + 1] = hi;
}

template <int... Is>
struct IndexSeq {};
template <int N, int... Is>
struct MakeSeq : MakeSeq<N - 1, N - 1, Is...> {};
template <int... Is>
struct MakeSeq<0, Is...> {
  using type = IndexSeq<Is...>;
};

template <int... Is>
JX_HD void rho_pi_all(const uint32_t* A, uint32_t* B, IndexSeq<Is...>) {
  (rho_pi_one<Is>(A, B), ...);
}


// One round of Keccak-f[1600] on a state of 25 (lo, hi) lanes: theta's 5-way column parity
// is two 3-input XORs (v_bitop3_b32 0x96) per word, rho is two v_alignbit_b32 per lane,
// chi's a ^ (~b & c) is one v_bitop3_b32 per word: 190 VALU instructions.
JX_HD void keccak_round(uint32_t* s, uint32_t rc_lo, uint32_t rc_hi) {
  uint32_t C[10], B[50];
#pragma unroll
  for (int x = 0; x < 5; x++) {
    C[2 * x] = xor3(xor3(s[2 * x], s[2 * (x + 5)], s[2 * (x + 10)]), s[2 * (x + 15)], s[2 * (x + 20)]);
    C[2 * x + 1] =
        xor3(xor3(s[2 * x + 1], s[2 * (x + 5) + 1], s[2 * (x + 10) + 1]), s[2 * (x + 15) + 1], s[2 * (x + 20) + 1]);
  }
#pragma unroll
  for (int x = 0; x < 5; x++) {
    uint32_t lo = C[2 * ((x + 1) % 5)], hi = C[2 * ((x + 1) % 5) + 1];
    rotl64<1>(lo, hi);
    uint32_t dlo = C[2 * ((x + 4) % 5)] ^ lo, dhi = C[2 * ((x + 4) % 5) + 1] ^ hi;
#pragma unroll
    for (int y = 0; y < 5; y++) {
      s[2 * (x + 5 * y)] ^= dlo;
      s[2 * (x + 5 * y) + 1] ^= dhi;
    }
  }
  rho_pi_all(s, B, typename MakeSeq<25>::type{});
#pragma unroll
  for (int y = 0; y < 5; y++) {
#pragma unroll
    for (int x = 0; x < 5; x++) {
      int i = x + 5 * y, i1 = (x + 1) % 5 + 5 * y, i2 = (x + 2) % 5 + 5 * y;
      s[2 * i] = B[2 * i] ^ (~B[2 * i1] & B[2 * i2]);
      s[2 * i + 1] = B[2 * i + 1] ^ (~B[2 * i1 + 1] & B[2 * i2 + 1]);
    }
  }
  s[0] ^= rc_lo;
  s[1] ^= rc_hi;
}

// Keccak-p[1600, 12]: rounds 12..23 of Keccak-f[1600]. s[2i] = lo, s[2i+1] = hi of lane i.
JX_HD void keccak_p12(uint32_t* s) {
#pragma unroll 1
  for (int ir = 12; ir < 24; ir++) keccak_round(s, KECCAK_RC_LO[ir], KECCAK_RC_HI[ir]);
}

// Keccak-p[1600, 12] with the rounds unrolled: the round constants become literals (no per-round scalar
// load, no loop control). It pays in the block loops of kernels that run one wave per SIMD, where a lone
// wave waits on each round's constant load: the word-per-lane K1 2.7-2.9 -> 2.5-2.7 ms, the lane-pair K1
// 4.03 -> 3.59 ms (profiles/r05_words_sweep*.jsonl). In the lane-split helper and the leader K1, whose
// configs[4] launches put two waves on some SIMDs, it measured slower (helper 152 -> 156 ms, leader 94 ->
// 99 ms beside each other; profiles/r05_unroll_fixedpoint.json), so they keep the loop.
JX_HD void keccak_p12_unrolled(uint32_t* s) {
#pragma unroll
  for (int ir = 12; ir < 24; ir++) keccak_round(s, KECCAK_RC_LO[ir], KECCAK_RC_HI[ir]);
}

// Two independent Keccak-p[1600, 12] permutations advanced round by round in one loop:
// two independent instruction streams for the scheduler (the measurement-share squeeze and
// the joint-randomness-part absorb of K1).
JX_HD void keccak_p12_x2(uint32_t* a, uint32_t* b) {
#pragma unroll 1
  for (int ir = 12; ir < 24; ir++) {
    const uint32_t lo = KECCAK_RC_LO[ir], hi = KECCAK_RC_HI[ir];
    keccak_round(a, lo, hi);
    keccak_round(b, lo, hi);
  }
}

// ----------------------------------------------------------------------------
// Single-block message builder (messages of <= 167 bytes, e.g. XOF inits).
// Bytes are little-endian within 32-bit words, as in the Keccak state.

struct Block {
  uint32_t w[42];
};

JX_HD void blk_zero(Block& b) {
#pragma unroll
  for (int i = 0; i < 42; i++) b.w[i] = 0;
}
JX_HD void blk_put_byte(Block& b, int pos, uint32_t v) { b.w[pos >> 2] |= (v & 0xffu) << (8 * (pos & 3)); }
// put a 32-bit little-endian word at byte position pos
JX_HD void blk_put_word(Block& b, int pos, uint32_t v) {
  int q = pos >> 2, r = pos & 3;
  if (r == 0) {
    b.w[q] |= v;
  } else {
    b.w[q] |= v << (8 * r);
    b.w[q + 1] |= v >> (32 - 8 * r);
  }
}
// VDAF-08 XofTurboShake128 message prefix: len(dst)=8 || dst || seed; dst = [8, 0, id BE32, usage BE16].
// Returns the next free byte position (25).
JX_HD int blk_xof_prefix(Block& b, uint32_t algo_id, uint32_t usage, const uint32_t seed[4]) {
  blk_put_byte(b, 0, 8);
  blk_put_byte(b, 1, 8);  // VERSION (draft-08)
  blk_put_byte(b, 2, 0);  // algorithm class (VDAF)
  blk_put_byte(b, 3, algo_id >> 24);
  blk_put_byte(b, 4, algo_id >> 16);
  blk_put_byte(b, 5, algo_id >> 8);
  blk_put_byte(b, 6, algo_id);
  blk_put_byte(b, 7, usage >> 8);
  blk_put_byte(b, 8, usage);
#pragma unroll
  for (int i = 0; i < 4; i++) blk_put_word(b, 9 + 4 * i, seed[i]);
  return 25;
}
// TurboSHAKE padding with D = 0x01 for a message of `len` bytes (< 168)
JX_HD void blk_pad(Block& b, int len) {
  blk_put_byte(b, len, 0x01);
  b.w[41] ^= 0x80000000u;
}
// state := 0; absorb one final block; permute. The state then holds output block 0.
JX_HD void sponge_oneblock(uint32_t* s, const Block& b) {
#pragma unroll
  for (int i = 0; i < 42; i++) s[i] = b.w[i];
#pragma unroll
  for (int i = 42; i < 50; i++) s[i] = 0;
  keccak_p12(s);
}

}  // namespace jx
