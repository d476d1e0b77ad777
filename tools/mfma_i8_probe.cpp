// Probe of the gfx950 i8 MFMA operand lane maps with exact integer data (asymmetric A and B).
// 16x16x64: byte j of lane l pairs A[l&15][k] with B[k][l&15], k = 16(l>>4)+j; C: col l&15, row 4(l>>4)+reg.
// 32x32x32: k = 16(l>>5)+j, rows/cols l&31; C: col l&31, row (reg&3)+8(reg>>2)+4(l>>5).
// (Any bijection of (l>>4, j) onto k used for both A and B gives the same product; the probe
// checks that A and B bytes pair by (lane group, j) and the C maps.)
//   hipcc --offload-arch=gfx950 -O2 -x hip tools/mfma_i8_probe.cpp -o tools/mfma_i8_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void mfma_once(const v4i* a, const v4i* b, v4i* c) {
  const int l = threadIdx.x;
  v4i acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], acc, 0, 0, 0);
  c[l] = acc;
}

__global__ void mfma32_once(const v4i* a, const v4i* b, int* c) {
  typedef int v16i __attribute__((ext_vector_type(16)));
  const int l = threadIdx.x;
  v16i acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], acc, 0, 0, 0);
  for (int r = 0; r < 16; r++) c[l * 16 + r] = acc[r];
}

static int kmap(int h, int l, int j) {
  switch (h) {
    case 0: return 16 * (l >> 4) + j;
    case 1: return 8 * (l >> 4) + (j & 7) + 32 * (j >> 3);
    case 2: return 4 * (l >> 4) + (j & 3) + 16 * (j >> 2);
    default: return -1;
  }
}

int main() {
  signed char A[16][64], B[64][16];
  srand(7);
  for (int i = 0; i < 16; i++)
    for (int k = 0; k < 64; k++) A[i][k] = (signed char)(rand() % 255 - 127);
  for (int k = 0; k < 64; k++)
    for (int j = 0; j < 16; j++) B[k][j] = (signed char)(rand() % 255 - 127);
  int ref[16][16];
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) {
      int s = 0;
      for (int k = 0; k < 64; k++) s += A[i][k] * B[k][j];
      ref[i][j] = s;
    }
  v4i *da, *db, *dc;
  (void)hipMalloc(&da, 64 * 16);
  (void)hipMalloc(&db, 64 * 16);
  (void)hipMalloc(&dc, 64 * 16);
  int found = -1;
  for (int h = 0; h < 3; h++) {
    signed char ha[64][16], hb[64][16];
    for (int l = 0; l < 64; l++)
      for (int j = 0; j < 16; j++) {
        ha[l][j] = A[l & 15][kmap(h, l, j)];
        hb[l][j] = B[kmap(h, l, j)][l & 15];
      }
    (void)hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma_once, dim3(1), dim3(64), 0, 0, da, db, dc);
    int hc[64][4];
    (void)hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++)
      for (int r = 0; r < 4; r++) bad += hc[l][r] != ref[4 * (l >> 4) + r][l & 15];
    printf("hypothesis %d: %d of 256 outputs differ\n", h, bad);
    if (!bad && found < 0) found = h;
  }
  printf("MATCH %d\n", found);
  {  // 32x32x32
    static signed char A2[32][32], B2[32][32], ha[64][16], hb[64][16];
    static int ref2[32][32], hc[64][16];
    for (int i = 0; i < 32; i++)
      for (int k = 0; k < 32; k++) A2[i][k] = (signed char)(rand() % 255 - 127);
    for (int k = 0; k < 32; k++)
      for (int j = 0; j < 32; j++) B2[k][j] = (signed char)(rand() % 255 - 127);
    for (int i = 0; i < 32; i++)
      for (int j = 0; j < 32; j++) {
        int s = 0;
        for (int k = 0; k < 32; k++) s += A2[i][k] * B2[k][j];
        ref2[i][j] = s;
      }
    for (int l = 0; l < 64; l++)
      for (int j = 0; j < 16; j++) {
        ha[l][j] = A2[l & 31][16 * (l >> 5) + j];
        hb[l][j] = B2[16 * (l >> 5) + j][l & 31];
      }
    int* dc2;
    (void)hipMalloc(&dc2, sizeof hc);
    (void)hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma32_once, dim3(1), dim3(64), 0, 0, da, db, dc2);
    (void)hipMemcpy(hc, dc2, sizeof hc, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++)
      for (int r = 0; r < 16; r++) bad += hc[l][r] != ref2[(r & 3) + 8 * (r >> 2) + 4 * (l >> 5)][l & 31];
    printf("32x32x32: %d of 1024 outputs differ\n", bad);
    if (bad) found = -1;
    (void)hipFree(dc2);
  }
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dc);
  return found < 0;
}
