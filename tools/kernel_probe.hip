// kernel_probe.hip — measurement harness, never part of the library: the helper's K1 (XOF stage) and K3
// (FLP ring) of SumVec 8x1000/88 launched directly on n reports of random bytes, in their product form and
// in their measurement variants (template parameters the library never instantiates):
//   K1 xof_kernel<false, 1>: the measurement-share staging stores skipped (a uniform run-time branch);
//   K1 xof_kernel<false, 2>: no per-block emission at all (stores, truncation, >= p screen);
//   K1 xof_kernel<false, 3>: the stores without the truncation and the >= p screen;
//   K3 flp_psum_part_glds_kernel<..., RING_ONLY = true>: the ring without the group finish.
// Timed by HIP events (ms per launch); run under rocprofv3 --pmc for each variant's clock and VALU
// utilisation ("K1's clock"). Results of the variants are wrong by design.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kernel_probe.hip -Iinclude -Ljanus_amd/lib -ljanus_prio3 \
//         -Wl,-rpath,'$ORIGIN/../../janus_amd/lib' -o tools/bin/kernel_probe
//   tools/bin/kernel_probe [reports=262144] [launches=5]
//   tools/bin/kernel_probe fpmix   (configs[4] helper K1: lane-split alone against lane-split + lane pairs on two
//                                   streams, 40,960 FixedPoint 16 x 10000 reports)
//   tools/bin/kernel_probe sweep   (small launches: the lane-pair K1, rounds unrolled and looped, against the
//                                   word-per-lane K1 + its truncation kernel, ms per launch at 16 .. 32,768 reports)
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../janus_amd/csrc/jx_engine_internal.h"
#include "../janus_amd/csrc/jx_kernels.hip"

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t _s = (x);                                                      \
    if (_s != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(_s));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ void fill_kernel(uint32_t* p, uint64_t words, uint32_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9E3779B9u ^ seed;
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    p[i] = x;
  }
}

static void* dalloc(size_t bytes, uint32_t seed) {
  void* p = nullptr;
  CK(hipMalloc(&p, bytes ? bytes : 16));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, (uint32_t*)p, (uint64_t)(bytes / 4), seed);
  return p;
}

template <typename F>
static double time_ms(F launch, int n, hipStream_t s) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();  // warm-up
  CK(hipEventRecord(a, s));
  for (int i = 0; i < n; i++) launch();
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / n;
}

static int sweep() {
  jx_prio3_params p{2, 8, 1000, 88, 1};
  uint8_t vk[16] = {0};
  jx_engine* e = nullptr;
  if (jx_engine_create(&p, vk, 0, &e)) return 2;
  const jx::Cfg c = e->cfg;
  const uint64_t N = 32768;
  jx::Bufs b{};
  b.nonces = (const uint8_t*)dalloc(N * 16, 1);
  b.ps = (const uint8_t*)dalloc(N * c.ps_bytes, 2);
  b.his = (const uint8_t*)dalloc(N * c.his_bytes, 3);
  b.lps = (const uint8_t*)dalloc(N * c.lps_bytes, 4);
  b.meas = (uint4*)dalloc(N * c.meas_len * 16, 5);
  b.proof = (uint4*)dalloc(N * c.proof_len * 16, 6);
  b.outs = (uint4*)dalloc(N * c.out_len * 16, 7);
  b.coef = (uint4*)dalloc(N * c.ncoef * 16, 8);
  b.flags = (uint32_t*)dalloc(N * 4, 9);
  b.part = (uint4*)dalloc(N * 64 * c.ngt, 10);
  b.verdicts = (uint8_t*)dalloc(N, 11);
  b.msgs = (uint8_t*)dalloc(N * 16, 12);
  b.consts = e->d_consts;
  b.lis_rs = c.lis_bytes;
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint64_t sizes[] = {16, 100, 256, 512, 1024, 2048, 3072, 4096, 6400, 8192, 16384, 32768};
  for (uint64_t n : sizes) {
    b.n = n;
    b.k1_split = 8;  // the lane pairs as the engine picks them below one pair-wave per SIMD (unrolled rounds)
    const double pairs = time_ms([&] { CK(jx::launch_xof(c, b, s)); }, 3, s);
    b.k1_split = 6;
    const double pairs_loop = time_ms([&] { CK(jx::launch_xof(c, b, s)); }, 3, s);
    b.k1_split = 7;
    const double words = time_ms([&] { CK(jx::launch_xof(c, b, s)); }, 3, s);
    printf("{\"reports\": %llu, \"pairs_ms\": %.3f, \"pairs_looped_ms\": %.3f, \"words_ms\": %.3f}\n",
           (unsigned long long)n, pairs, pairs_loop, words);
    fflush(stdout);
  }
  jx_engine_destroy(e);
  return 0;
}

// configs[4]'s helper K1 (FixedPointBoundedL2VecSum 16 x 10000, 40,960 reports, lone): the lane-split kernel
// over all reports against a mixed launch (the first S reports lane-split on one stream, the rest as lane pairs on
// a second stream at the same time), for a few split points.
static int fpmix() {
  jx_prio3_params p{5, 16, 10000, 0, 1};
  uint8_t vk[16] = {0};
  jx_engine* e = nullptr;
  if (jx_engine_create(&p, vk, 0, &e)) return 2;
  const jx::Cfg c = e->cfg;
  const uint64_t N = 40960;
  jx::Bufs b{};
  b.n = N;
  b.nonces = (const uint8_t*)dalloc(N * 16, 1);
  b.ps = (const uint8_t*)dalloc(N * c.ps_bytes, 2);
  b.his = (const uint8_t*)dalloc(N * c.his_bytes, 3);
  b.lps = (const uint8_t*)dalloc(N * c.lps_bytes, 4);
  b.meas = (uint4*)dalloc(N * (uint64_t)c.meas_len * 16, 5);
  b.proof = (uint4*)dalloc(N * (uint64_t)c.proof_len * 16, 6);
  b.outs = (uint4*)dalloc(N * (uint64_t)c.out_len * 16, 7);
  b.coef = (uint4*)dalloc(N * (uint64_t)c.ncoef * 16, 8);
  b.flags = (uint32_t*)dalloc(N * 4, 9);
  b.verdicts = (uint8_t*)dalloc(N, 11);
  b.msgs = (uint8_t*)dalloc(N * 16, 12);
  b.consts = e->d_consts;
  b.lis_rs = c.lis_bytes;
  b.k1_lds = jx::lanes_lds_bytes(2);
  CK(hipDeviceSynchronize());
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, join, t0, t1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  // the reports [S, N) as a Bufs of their own (whole 64-report blocks: every staging array is block-interleaved)
  auto tail = [&](uint64_t S) {
    jx::Bufs t = b;
    const uint64_t blk = S / 64;
    t.n = N - S;
    t.nonces += S * 16;
    t.ps += S * c.ps_bytes;
    t.his += S * c.his_bytes;
    t.lps += S * c.lps_bytes;
    t.meas += blk * c.meas_len * jx::IL;
    t.proof += blk * c.proof_len * jx::IL;
    t.outs += blk * c.out_len * jx::IL;
    t.coef += blk * c.ncoef * jx::IL;
    t.flags += S;
    t.verdicts += S;
    t.msgs += S * 16;
    return t;
  };
  auto run = [&](uint64_t S, uint32_t split_b, int reps) {
    float best = 1e30f;
    for (int it = 0; it < reps + 1; it++) {
      jx::Bufs a = b, t = tail(S);
      a.n = S;
      a.k1_split = 3;
      t.k1_split = split_b;
      CK(hipEventRecord(t0, s1));
      CK(hipEventRecord(fork, s1));
      CK(hipStreamWaitEvent(s2, fork, 0));
      if (S) CK(jx::launch_xof(c, a, s1));
      if (S < N) CK(jx::launch_xof(c, t, s2));
      CK(hipEventRecord(join, s2));
      CK(hipStreamWaitEvent(s1, join, 0));
      CK(hipEventRecord(t1, s1));
      CK(hipEventSynchronize(t1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, t0, t1));
      if (it > 0 && ms < best) best = ms;
    }
    return (double)best;
  };
  const uint64_t splits[] = {40960, 36864, 34816, 32768, 30720, 28672, 0};
  for (uint32_t pk : {8u, 6u}) {  // the lane-pair part with unrolled (8) or looped (6) rounds
    for (uint64_t S : splits) {
      const double ms = run(S, pk, 2);
      printf("{\"lane_split_reports\": %llu, \"lane_pair_reports\": %llu, \"pairs_unrolled\": %s, \"ms\": %.2f}\n",
             (unsigned long long)S, (unsigned long long)(N - S), pk == 8 ? "true" : "false", ms);
      fflush(stdout);
    }
  }
  jx_engine_destroy(e);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "sweep") return sweep();
  if (argc > 1 && std::string(argv[1]) == "fpmix") return fpmix();
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 262144;
  const int iters = argc > 2 ? atoi(argv[2]) : 5;
  jx_prio3_params p{2, 8, 1000, 88, 1};
  uint8_t vk[16] = {0};
  jx_engine* e = nullptr;
  if (jx_engine_create(&p, vk, 0, &e)) return 2;
  const jx::Cfg c = e->cfg;
  jx::Bufs b{};
  b.n = n;
  b.nonces = (const uint8_t*)dalloc(n * 16, 1);
  b.ps = (const uint8_t*)dalloc(n * c.ps_bytes, 2);
  b.his = (const uint8_t*)dalloc(n * c.his_bytes, 3);
  b.lps = (const uint8_t*)dalloc(n * c.lps_bytes, 4);
  b.meas = (uint4*)dalloc(n * c.meas_len * 16, 5);
  b.proof = (uint4*)dalloc(n * c.proof_len * 16, 6);
  b.outs = (uint4*)dalloc(n * c.out_len * 16, 7);
  b.coef = (uint4*)dalloc(n * c.ncoef * 16, 8);
  b.flags = (uint32_t*)dalloc(n * 4, 9);
  b.part = (uint4*)dalloc(n * 64 * c.ngt, 10);
  b.verdicts = (uint8_t*)dalloc(n, 11);
  b.msgs = (uint8_t*)dalloc(n * 16, 12);
  b.consts = e->d_consts;
  b.lis_rs = c.lis_bytes;
  b.k1_split = 5;
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint32_t nb = (uint32_t)((n + 63) / 64);
  const dim3 g1((nb + jx::K1_WAVES - 1) / jx::K1_WAVES), b1(64 * jx::K1_WAVES);
  const double k1 = time_ms([&] { hipLaunchKernelGGL((jx::xof_kernel<false, 0>), g1, b1, 0, s, c, b); }, iters, s);
  const double k1_sink = time_ms([&] { hipLaunchKernelGGL((jx::xof_kernel<false, 1>), g1, b1, 0, s, c, b); }, iters, s);
  const double k1_noemit = time_ms([&] { hipLaunchKernelGGL((jx::xof_kernel<false, 2>), g1, b1, 0, s, c, b); }, iters, s);
  const double k1_stores = time_ms([&] { hipLaunchKernelGGL((jx::xof_kernel<false, 3>), g1, b1, 0, s, c, b); }, iters, s);
  const uint32_t grid = ((nb + 7) / 8) * 8 * c.ngroups;
  const uint32_t g3 = grid / c.ngroups * ((c.ngroups + jx::K3W - 1) / jx::K3W);
  const double k3 = time_ms(
      [&] {
        hipLaunchKernelGGL((jx::flp_psum_part_glds_kernel<2, false, false, 4, jx::K3W, false>), dim3(g3),
                           dim3(64 * jx::K3W), 0, s, c, b);
      },
      iters, s);
  const double k3_ring = time_ms(
      [&] {
        hipLaunchKernelGGL((jx::flp_psum_part_glds_kernel<2, false, false, 4, jx::K3W, true>), dim3(g3),
                           dim3(64 * jx::K3W), 0, s, c, b);
      },
      iters, s);
  printf("{\"reports\": %llu, \"launches\": %d, \"k1_ms\": %.3f, \"k1_no_stores_ms\": %.3f, \"k1_no_emission_ms\": %.3f, "
         "\"k1_stores_only_ms\": %.3f, \"k3_ms\": %.3f, \"k3_ring_only_ms\": %.3f}\n",
         (unsigned long long)n, iters, k1, k1_sink, k1_noemit, k1_stores, k3, k3_ring);
  jx_engine_destroy(e);
  return 0;
}
