// microbench_keccak.hip — Keccak-p[1600,12] permutation rate on gfx950 as a function of waves per
// SIMD and of independent states per lane, with the in-kernel shader clock. Answers whether K1
// (xof_kernel, two states per lane at two waves/SIMD) is bound by issue slots that more waves would
// fill, or by the chip's sustained VALU rate for this instruction mix.
// Build: hipcc --offload-arch=gfx950 -O3 -I janus_amd/csrc -o tools/bin/microbench_keccak tools/microbench_keccak.hip
// Output: one JSON line per (states, waves/SIMD) case.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "jx_keccak.h"

#define CHK(x)                                                    \
  do {                                                            \
    hipError_t e_ = (x);                                          \
    if (e_ != hipSuccess) {                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                   \
    }                                                             \
  } while (0)

// NS states per lane; W = minimum waves per SIMD the register allocation must allow.
// stamps[block] = {memtime0, realtime0, memtime1, realtime1} of wave 0 (diagnostic only: no output is
// computed from them). out[] keeps the states alive.
template <int NS, int W>
__global__ __launch_bounds__(256, W) void perm_loop(uint32_t* out, uint64_t* stamps, int iters) {
  uint32_t s[NS][50];
#pragma unroll
  for (int k = 0; k < NS; k++)
#pragma unroll
    for (int i = 0; i < 50; i++) s[k][i] = (threadIdx.x + 977u * blockIdx.x) * 2654435761u + 40503u * i + k;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
    if constexpr (NS == 1) {
      jx::keccak_p12(s[0]);
    } else {
      jx::keccak_p12_x2(s[0], s[1]);
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < NS; k++)
#pragma unroll
    for (int i = 0; i < 50; i++) acc ^= s[k][i];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0) {
    stamps[4 * blockIdx.x + 0] = t0;
    stamps[4 * blockIdx.x + 1] = r0;
    stamps[4 * blockIdx.x + 2] = t1;
    stamps[4 * blockIdx.x + 3] = r1;
  }
}

template <int NS, int W>
static int run(int waves_per_simd, int iters) {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * waves_per_simd;  // 256-thread blocks = one wave per SIMD each
  uint32_t* out;
  uint64_t* st;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CHK(hipMalloc(&st, (size_t)blocks * 32));
  hipLaunchKernelGGL((perm_loop<NS, W>), dim3(blocks), dim3(256), 0, 0, out, st, 4);  // warm-up
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((perm_loop<NS, W>), dim3(blocks), dim3(256), 0, 0, out, st, iters);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  // clock from the stamps of the last run (median over blocks)
  uint64_t* h = (uint64_t*)malloc((size_t)blocks * 32);
  CHK(hipMemcpy(h, st, (size_t)blocks * 32, hipMemcpyDeviceToHost));
  double* ghz = (double*)malloc(sizeof(double) * blocks);
  for (int b = 0; b < blocks; b++) {
    const double dt = (double)(h[4 * b + 2] - h[4 * b]), dr = (double)(h[4 * b + 3] - h[4 * b + 1]);
    ghz[b] = dr > 0 ? dt / dr * 0.1 : 0.0;  // s_memrealtime ticks at 100 MHz
  }
  for (int i = 1; i < blocks; i++)
    for (int j = i; j > 0 && ghz[j - 1] > ghz[j]; j--) {
      double t = ghz[j];
      ghz[j] = ghz[j - 1];
      ghz[j - 1] = t;
    }
  const double clk = ghz[blocks / 2];
  const double perms = (double)blocks * 256 * iters * NS;
  const double wave_instr = perms / 64.0 * 2280.0;  // 190 VALU per round x 12 rounds
  const double peak = (double)cus * 4 * 2.4e9 / 2.0;  // wave-instructions/s, 2 cycles each
  printf("{\"states_per_lane\": %d, \"min_waves_bound\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, "
         "\"perms_per_s\": %.4g, \"issue_frac_flat\": %.4f, \"clock_ghz\": %.3f, \"issue_frac_at_clock\": %.4f}\n",
         NS, W, waves_per_simd, best, perms / (best * 1e-3), wave_instr / (best * 1e-3) / peak, clk,
         wave_instr / (best * 1e-3) / (peak * clk / 2.4));
  fflush(stdout);
  free(h);
  free(ghz);
  CHK(hipFree(out));
  CHK(hipFree(st));
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  int rc = 0;
  // one state per lane: 1..8 waves per SIMD (the bound lets the allocator use <= 64 registers at 8)
  rc |= run<1, 1>(1, iters);
  rc |= run<1, 2>(2, iters);
  rc |= run<1, 4>(4, iters);
  rc |= run<1, 4>(3, iters);
  rc |= run<1, 8>(8, iters);
  // two states per lane (K1's keccak_p12_x2): 1..4 waves per SIMD
  rc |= run<2, 1>(1, iters / 2);
  rc |= run<2, 2>(2, iters / 2);
  rc |= run<2, 3>(3, iters / 2);
  rc |= run<2, 4>(4, iters / 2);
  return rc;
}
