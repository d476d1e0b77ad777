// microbench_valu.hip — issue rate of the gfx950 VALU instructions the Prio3 kernels are built
// from (Keccak: v_bitop3_b32 / v_alignbit_b32 / v_xor_b32; Field128: v_mad_u64_u32,
// v_mul_lo/hi_u32, 64-bit adds). Calibrates the cost model of DESIGN.md §5.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/microbench_valu tools/microbench_valu.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

enum {
  OP_XOR, OP_BITOP3, OP_ALIGNBIT, OP_MAD64, OP_MULLO, OP_MULHI, OP_ADD64, OP_MAD24, OP_FMA64,
  OP_XOR3, OP_ROT, OP_PERM, OP_LSHLOR, OP_ADD3, OP_ADDCO, OP_MIX_AX, OP_MIX_ABX, NOPS
};
static const char* NAMES[NOPS] = {"v_xor_b32",      "v_bitop3_b32(a^~b&c)", "v_alignbit_b32", "v_mad_u64_u32",
                                  "v_mul_lo_u32",   "v_mul_hi_u32+xor",     "add_u64",        "v_mad_u32_u24",
                                  "v_fma_f64",      "v_bitop3_b32(xor3)",   "v_alignbit(rot)", "v_perm_b32",
                                  "v_lshl_or_b32",  "v_add3_u32",           "v_add_co+addc",
                                  "mix 4 alignbit + 4 xor", "mix 3 alignbit + 3 bitop3 + 2 xor"};

template <int OP>
__global__ __launch_bounds__(256) void bench(uint32_t* out, int iters, uint32_t k) {
  uint32_t x[8];
  uint64_t y[8];
  double d[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    x[j] = threadIdx.x * 2654435761u + j * 40503u + k;
    y[j] = ((uint64_t)x[j] << 32) | (x[j] ^ 0x9e3779b9u);
    d[j] = (double)x[j];
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if constexpr (OP == OP_XOR) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = x[j] ^ x[(j + 1) & 7];
      } else if constexpr (OP == OP_BITOP3) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __builtin_amdgcn_bitop3_b32(x[j], x[(j + 1) & 7], x[(j + 2) & 7], 0xd2);
      } else if constexpr (OP == OP_ALIGNBIT) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __builtin_amdgcn_alignbit(x[j], x[(j + 1) & 7], 13);
      } else if constexpr (OP == OP_MAD64) {
#pragma unroll
        for (int j = 0; j < 8; j++) y[j] = (uint64_t)(uint32_t)y[j] * (uint32_t)(y[(j + 1) & 7] >> 32) + y[j];
      } else if constexpr (OP == OP_MULLO) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = x[j] * x[(j + 1) & 7];
      } else if constexpr (OP == OP_MULHI) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __umulhi(x[j], x[(j + 1) & 7]) ^ k;
      } else if constexpr (OP == OP_ADD64) {
#pragma unroll
        for (int j = 0; j < 8; j++) y[j] = y[j] + y[(j + 1) & 7];
      } else if constexpr (OP == OP_MAD24) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = (x[j] & 0xffffffu) * (x[(j + 1) & 7] & 0xffffffu) + x[j];
      } else if constexpr (OP == OP_FMA64) {
#pragma unroll
        for (int j = 0; j < 8; j++) d[j] = __builtin_fma(d[j], d[(j + 1) & 7], d[j]);
      } else if constexpr (OP == OP_XOR3) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __builtin_amdgcn_bitop3_b32(x[j], x[(j + 1) & 7], x[(j + 2) & 7], 0x96);
      } else if constexpr (OP == OP_ROT) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __builtin_amdgcn_alignbit(x[(j + 1) & 7], x[(j + 1) & 7], k + j);
      } else if constexpr (OP == OP_PERM) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = __builtin_amdgcn_perm(x[j], x[(j + 1) & 7], 0x05040302u);
      } else if constexpr (OP == OP_LSHLOR) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = (x[j] << (k & 31)) | x[(j + 1) & 7];
      } else if constexpr (OP == OP_ADD3) {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = x[j] + x[(j + 1) & 7] + x[(j + 2) & 7];
      } else if constexpr (OP == OP_MIX_AX) {
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          x[j] = __builtin_amdgcn_alignbit(x[j], x[(j + 1) & 7], k + j);
          x[j + 1] = __builtin_amdgcn_bitop3_b32(x[j + 1], x[(j + 2) & 7], 0u, 0x3c);  // a ^ b
        }
      } else if constexpr (OP == OP_MIX_ABX) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
          if (j % 8 < 3)
            x[j] = __builtin_amdgcn_alignbit(x[j], x[(j + 1) & 7], k + j);
          else if (j % 8 < 6)
            x[j] = __builtin_amdgcn_bitop3_b32(x[j], x[(j + 1) & 7], x[(j + 2) & 7], 0xd2);
          else
            x[j] = x[j] ^ x[(j + 3) & 7] ^ k;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) {
          uint32_t lo = (uint32_t)y[j], hi = (uint32_t)(y[j] >> 32);
          uint32_t blo = (uint32_t)y[(j + 1) & 7], bhi = (uint32_t)(y[(j + 1) & 7] >> 32);
          uint32_t c;
          lo = __builtin_addc(lo, blo, 0u, &c);
          hi = __builtin_addc(hi, bhi, c, &c);
          y[j] = ((uint64_t)hi << 32) | lo;
        }
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) acc += x[j] + (uint32_t)y[j] + (uint32_t)(y[j] >> 32) + (uint32_t)d[j];
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

template <int OP>
static int run(int blocks, int iters, uint32_t* dout) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, dout, 16, 1u);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, dout, iters, 1u);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  double lane_ops = (double)blocks * 256 * iters * 64;  // 8 unroll x 8 chains per iteration
  double rate = lane_ops / (ms * 1e-3);
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"frac_of_78.6T\": %.3f}\n", NAMES[OP], ms, rate,
         rate / 78.6432e12);
  return 0;
}

int main(int argc, char** argv) {
  int blocks = 256 * 8, iters = argc > 1 ? atoi(argv[1]) : 4096;
  uint32_t* d;
  CHK(hipMalloc(&d, 4096));
  run<OP_XOR>(blocks, iters, d);
  run<OP_BITOP3>(blocks, iters, d);
  run<OP_ALIGNBIT>(blocks, iters, d);
  run<OP_MAD64>(blocks, iters, d);
  run<OP_MULLO>(blocks, iters, d);
  run<OP_MULHI>(blocks, iters, d);
  run<OP_ADD64>(blocks, iters, d);
  run<OP_MAD24>(blocks, iters, d);
  run<OP_FMA64>(blocks, iters, d);
  run<OP_XOR3>(blocks, iters, d);
  run<OP_ROT>(blocks, iters, d);
  run<OP_PERM>(blocks, iters, d);
  run<OP_LSHLOR>(blocks, iters, d);
  run<OP_ADD3>(blocks, iters, d);
  run<OP_ADDCO>(blocks, iters, d);
  run<OP_MIX_AX>(blocks, iters, d);
  run<OP_MIX_ABX>(blocks, iters, d);
  CHK(hipFree(d));
  return 0;
}
