// microbench_stream.hip — read rate of K3's measurement-share stream without its arithmetic.
// The SumVec(8x1000/88) staging of 262,144 reports (33.5 GB, interleaved [block][element][lane] x 16 B)
// is read by
//   ring: K3's LDS-DMA ring structure (flp_psum_part_glds_kernel: 4-wave workgroups = 4 slot groups of a
//         64-report block, 2 elements per wave per call, depth-4 ring, one barrier per call), XOR only;
//   flat: plain global_load_dwordx4 sweep, 4 loads in flight per lane, grid-stride;
//   slice_*: the MFMA K3's per-eighth stream (interleaved vs eighth-major staging, ring depth 4 / 6);
//   ring_mad<N>: the ring with N v_mad_u64_u32 per call per wave (K3's products without the rest);
// and prints one JSON line per kernel with the achieved GB/s. Tells whether K3 (8.4 ms per 250k reports)
// is bound by its stream or by its VALU work.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/microbench_stream tools/microbench_stream.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                               \
    }                                                         \
  } while (0)

constexpr uint32_t M = 8000, CHUNK = 88, CALLS = 90, NG = 44, W = 4, D = 4, PPW = 2;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt(0x3f70 | (N & 15) | ((N >> 4) << 14));
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)p;
}

constexpr uint32_t NC = 200;  // per-report coefficient slots (c_k, d_k interleaved), as K1 stages them
__global__ __launch_bounds__(256, 4) void ring(const uint4* meas, const uint4* coef, uint64_t nblk, uint4* out) {
  constexpr int ROWS = 2 + W * PPW;
  __shared__ uint4 rb[D][ROWS][64];
  const uint32_t NW = NG / W;
  const uint32_t bid = blockIdx.x, xcd = bid & 7u, q = bid >> 3;
  const uint32_t wg = q % NW;
  const uint64_t blk = (uint64_t)(q / NW) * 8 + xcd;
  if (blk >= nblk) return;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = wg * W + wave, j0 = g * PPW;
  const uint4* mb = meas + blk * M * 64 + lane;
  const uint4* cb = coef + blk * NC * 64 + lane;
  auto issue = [&](uint32_t k) {
    if (wave < 2)
      __builtin_amdgcn_global_load_lds((const void*)(cb + (uint64_t)(8 + 2 * (k - 1) + wave) * 64),
                                       (void*)&rb[(k - 1) % D][wave][0], 16, 0, 0);
#pragma unroll
    for (int i = 0; i < PPW; i++)
      __builtin_amdgcn_global_load_lds((const void*)(mb + (uint64_t)((k - 1) * CHUNK + j0 + i) * 64),
                                       (void*)&rb[(k - 1) % D][2 + wave * PPW + i][0], 16, 0, 0);
  };
  for (uint32_t k = 1; k < D; k++) issue(k);
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint32_t base = lds_addr(&rb[0][0][lane]);
  for (uint32_t k = 1; k <= CALLS; k++) {
    if (k + D - 2 > CALLS)
      wait_vmcnt<0>();
    else if (wave < 2)
      wait_vmcnt<(D - 2) * (PPW + 1)>();
    else
      wait_vmcnt<(D - 2) * PPW>();
    __builtin_amdgcn_s_barrier();
    if (k + D - 1 <= CALLS) issue(k + D - 1);
    const uint32_t a = base + (((k - 1) % D) * ROWS + 2 + wave * PPW) * 1024;
    uint4 v0, v1;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v0), "=&v"(v1)
                 : "v"(a), "v"(a + 1024)
                 : "memory");
    acc.x ^= v0.x ^ v1.x;
    acc.y ^= v0.y ^ v1.y;
    acc.z ^= v0.z ^ v1.z;
    acc.w ^= v0.w ^ v1.w;
  }
  out[(blk * NG + g) * 64 + lane] = acc;
}


// The same ring with NM independent v_mad_u64_u32 per call per wave on the loaded words (K3 does 100 limb
// products per call per wave plus ~50 other VALU instructions): how the stream rate falls as the ring's
// compute grows, i.e. how much of K3's time its products add on top of the ring.
template <int NM>
__global__ __launch_bounds__(256, 4) void ring_mad(const uint4* meas, const uint4* coef, uint64_t nblk, uint4* out) {
  constexpr int ROWS = 2 + W * PPW;
  __shared__ uint4 rb[D][ROWS][64];
  const uint32_t NW = NG / W;
  const uint32_t bid = blockIdx.x, xcd = bid & 7u, q = bid >> 3;
  const uint32_t wg = q % NW;
  const uint64_t blk = (uint64_t)(q / NW) * 8 + xcd;
  if (blk >= nblk) return;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = wg * W + wave, j0 = g * PPW;
  const uint4* mb = meas + blk * M * 64 + lane;
  const uint4* cb = coef + blk * NC * 64 + lane;
  auto issue = [&](uint32_t k) {
    if (wave < 2)
      __builtin_amdgcn_global_load_lds((const void*)(cb + (uint64_t)(8 + 2 * (k - 1) + wave) * 64),
                                       (void*)&rb[(k - 1) % D][wave][0], 16, 0, 0);
#pragma unroll
    for (int i = 0; i < PPW; i++)
      __builtin_amdgcn_global_load_lds((const void*)(mb + (uint64_t)((k - 1) * CHUNK + j0 + i) * 64),
                                       (void*)&rb[(k - 1) % D][2 + wave * PPW + i][0], 16, 0, 0);
  };
  for (uint32_t k = 1; k < D; k++) issue(k);
  uint64_t acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t base = lds_addr(&rb[0][0][lane]);
  for (uint32_t k = 1; k <= CALLS; k++) {
    if (k + D - 2 > CALLS)
      wait_vmcnt<0>();
    else if (wave < 2)
      wait_vmcnt<(D - 2) * (PPW + 1)>();
    else
      wait_vmcnt<(D - 2) * PPW>();
    __builtin_amdgcn_s_barrier();
    if (k + D - 1 <= CALLS) issue(k + D - 1);
    const uint32_t a = base + ((k - 1) % D) * ROWS * 1024;
    uint4 cv, dv, v0, v1;
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(cv), "=&v"(dv), "=&v"(v0), "=&v"(v1)
        : "v"(a), "v"(a + 1024), "v"(a + (2 + wave * PPW) * 1024), "v"(a + (3 + wave * PPW) * 1024)
        : "memory");
    const uint32_t xs[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const uint32_t cs[8] = {cv.x, cv.y, cv.z, cv.w, dv.x, dv.y, dv.z, dv.w};
#pragma unroll
    for (int m = 0; m < NM; m++) {
      acc[m % 10] += (uint64_t)xs[m % 8] * cs[(m / 8) % 8];
      asm("" : "+v"(acc[m % 10]));
    }
  }
  uint64_t t = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) t ^= acc[i];
  out[(blk * NG + g) * 64 + lane] = make_uint4((uint32_t)t, (uint32_t)(t >> 32), 0, 0);
}

// The MFMA K3's access pattern: a workgroup of 8 waves streams K-steps of 2 calls x 96 slots x 8 reports
// (an eighth of a 64-report block; 24 KiB) through a depth-D LDS ring, one barrier per step. CONTIG = 0:
// the interleaved staging (each row piece is the 128 B of 8 reports inside a 1 KiB element row);
// CONTIG = 1: an eighth-major staging ([block][eighth][element][8 reports]: a step reads 2 x 12 KiB runs).
template <int CONTIG, int DD>
__global__ __launch_bounds__(512, 1) void slice(const uint4* meas, uint64_t nblk, uint4* out) {
  constexpr uint32_t SL = 96, XE = 2 * SL * 8, NI = XE / 64 / 8;
  __shared__ uint4 rb[DD][XE];
  const uint32_t bid = blockIdx.x, xcd = bid & 7u, q8 = bid >> 3;
  const uint64_t blk = (uint64_t)(q8 >> 3) * 8 + xcd;
  if (blk >= nblk) return;
  const uint32_t e8 = q8 & 7u, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t KS = (CALLS + 2) / 2;
  auto src = [&](uint32_t ks, uint32_t i) {
    const uint32_t p = 64 * (NI * wave + i) + lane, row = p >> 3, hh = row / SL, sl = row % SL;
    const uint32_t r = (p & 7u) ^ ((sl >> 1) & 7u);
    uint32_t e = (2 * ks + hh) * CHUNK + sl;
    if (sl >= CHUNK || e >= M) e = 0;
    if (CONTIG) return meas + ((blk * 8 + e8) * M + e) * 8 + r;
    return meas + (blk * M + e) * 64 + 8 * e8 + r;
  };
  auto issue = [&](uint32_t ks) {
    for (uint32_t i = 0; i < NI; i++)
      __builtin_amdgcn_global_load_lds((const void*)src(ks, i), (void*)&rb[ks % DD][64 * (NI * wave + i)], 16, 0, 0);
  };
  for (uint32_t ks = 0; ks + 1 < DD; ks++) issue(ks);
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint32_t base = lds_addr(&rb[0][0]);
  for (uint32_t ks = 0; ks < KS; ks++) {
    if (ks + DD - 2 >= KS)
      wait_vmcnt<0>();
    else
      wait_vmcnt<(DD - 2) * NI>();
    __builtin_amdgcn_s_barrier();
    if (ks + DD - 1 < KS) issue(ks + DD - 1);
    const uint32_t a = base + ((ks % DD) * XE + 64 * wave + lane) * 16;
    uint4 v0;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v0) : "v"(a) : "memory");
    acc.x ^= v0.x;
    acc.y ^= v0.y;
    acc.z ^= v0.z;
    acc.w ^= v0.w;
  }
  out[(uint64_t)bid * 512 + threadIdx.x] = acc;
}

// pseudo-random fill (splitmix64 of the index): the multipliers see K3-like operand bits, not a constant
__global__ __launch_bounds__(256) void fill_random(uint4* p, uint64_t n16, uint64_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    const uint64_t a = z ^ (z >> 31), b = a * 0xD6E8FEB86659FD93ull ^ (a >> 29);
    p[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32) & 0x7FFFFFFFu);
  }
}

__global__ __launch_bounds__(256) void flat(const uint4* p, uint64_t n16, uint4* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, nt = (uint64_t)gridDim.x * 256;
  uint4 acc = make_uint4(0, 0, 0, 0);
  uint64_t i = tid;
  for (; i + 3 * nt < n16; i += 4 * nt) {
    uint4 a = p[i], b = p[i + nt], c = p[i + 2 * nt], d = p[i + 3 * nt];
    acc.x ^= a.x ^ b.x ^ c.x ^ d.x;
    acc.y ^= a.y ^ b.y ^ c.y ^ d.y;
    acc.z ^= a.z ^ b.z ^ c.z ^ d.z;
    acc.w ^= a.w ^ b.w ^ c.w ^ d.w;
  }
  for (; i < n16; i += nt) {
    uint4 a = p[i];
    acc.x ^= a.x;
    acc.y ^= a.y;
    acc.z ^= a.z;
    acc.w ^= a.w;
  }
  out[tid] = acc;
}

int main(int argc, char** argv) {
  const uint64_t nrep = argc > 1 ? strtoull(argv[1], 0, 10) : 262144;
  const uint64_t nblk = nrep / 64, n16 = nblk * M * 64;
  const double bytes = (double)n16 * 16;
  uint4 *meas, *out, *coef;
  CHK(hipMalloc(&meas, n16 * 16));
  CHK(hipMalloc(&coef, nblk * NC * 64 * 16));
  CHK(hipMemset(coef, 0x33, nblk * NC * 64 * 16));
  CHK(hipMemset(meas, 0x5a, n16 * 16));
  const uint64_t ring_grid = nblk * (NG / W), flat_grid = 256 * 8 * 4;
  CHK(hipMalloc(&out, sizeof(uint4) * (nblk * NG * 64 > flat_grid * 256 ? nblk * NG * 64 : flat_grid * 256)));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const uint64_t slice_grid = ((nblk + 7) / 8) * 8 * 8;
  uint4* out2;
  CHK(hipMalloc(&out2, slice_grid * 512 * 16));
  const bool rnd = argc > 2 && argv[2][0] == 'r';  // random operands (K3-like switching) instead of a constant
  if (rnd) {
    hipLaunchKernelGGL(fill_random, dim3(8192), dim3(256), 0, 0, meas, n16, 1);
    hipLaunchKernelGGL(fill_random, dim3(8192), dim3(256), 0, 0, coef, nblk * NC * 64, 77);
    CHK(hipDeviceSynchronize());
  }
  for (int kern = 0; kern < 10; kern++) {
    if (rnd && kern >= 1 && kern <= 5) continue;  // the pure streams do not multiply
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      CHK(hipEventRecord(e0, 0));
      if (kern == 0)
        hipLaunchKernelGGL(ring, dim3(ring_grid), dim3(256), 0, 0, meas, coef, nblk, out);
      else if (kern == 1)
        hipLaunchKernelGGL(flat, dim3(flat_grid), dim3(256), 0, 0, meas, n16, out);
      else if (kern == 2)
        hipLaunchKernelGGL((slice<0, 4>), dim3(slice_grid), dim3(512), 0, 0, meas, nblk, out2);
      else if (kern == 3)
        hipLaunchKernelGGL((slice<1, 4>), dim3(slice_grid), dim3(512), 0, 0, meas, nblk, out2);
      else if (kern == 4)
        hipLaunchKernelGGL((slice<0, 6>), dim3(slice_grid), dim3(512), 0, 0, meas, nblk, out2);
      else if (kern == 5)
        hipLaunchKernelGGL((slice<1, 6>), dim3(slice_grid), dim3(512), 0, 0, meas, nblk, out2);
      else if (kern == 6)
        hipLaunchKernelGGL((ring_mad<50>), dim3(ring_grid), dim3(256), 0, 0, meas, coef, nblk, out);
      else if (kern == 7)
        hipLaunchKernelGGL((ring_mad<100>), dim3(ring_grid), dim3(256), 0, 0, meas, coef, nblk, out);
      else if (kern == 8)
        hipLaunchKernelGGL((ring_mad<150>), dim3(ring_grid), dim3(256), 0, 0, meas, coef, nblk, out);
      else
        hipLaunchKernelGGL((ring_mad<200>), dim3(ring_grid), dim3(256), 0, 0, meas, coef, nblk, out);
      CHK(hipEventRecord(e1, 0));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best) best = ms;
    }
    printf("{\"kernel\": \"%s\", \"data\": \"%s\", \"reports\": %llu, \"bytes\": %.0f, \"ms\": %.3f, \"GBps\": %.1f}\n",
           kern == 0 ? "ring" : kern == 1 ? "flat" : kern == 2 ? "slice_il_d4" : kern == 3 ? "slice_contig_d4"
                                  : kern == 4 ? "slice_il_d6" : kern == 5 ? "slice_contig_d6"
                                  : kern == 6 ? "ring_mad50" : kern == 7 ? "ring_mad100" : kern == 8 ? "ring_mad150"
                                  : "ring_mad200",
           rnd ? "random" : "constant",
           (unsigned long long)nrep, bytes, best, bytes / (best * 1e6));
    fflush(stdout);
  }
  return 0;
}
