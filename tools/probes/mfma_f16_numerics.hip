// Probe: numerics of v_mfma_f32_16x16x32_f16 on gfx950 (how the 32 products
// of one instruction and the C input are summed; subnormal f16 inputs).
// One wave; row 0 / column 0 carry the test vector, everything else zero.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const float* a32, const float* b32, float c0, float* out) {
  const int lane = threadIdx.x;
  half8 a, b;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * (lane >> 4) + j;
    a[j] = (lane & 15) == 0 ? (_Float16)a32[k] : (_Float16)0.f;
    b[j] = (lane & 15) == 0 ? (_Float16)b32[k] : (_Float16)0.f;
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (lane == 0) acc[0] = c0;  // C[row 0][col 0]
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];  // D[row 0][col 0]
}

static float run(const float* a, const float* b, float c0) {
  float *da, *db, *dout, h;
  hipMalloc(&da, 128); hipMalloc(&db, 128); hipMalloc(&dout, 4);
  hipMemcpy(da, a, 128, hipMemcpyHostToDevice);
  hipMemcpy(db, b, 128, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, c0, dout);
  hipMemcpy(&h, dout, 4, hipMemcpyDeviceToHost);
  hipFree(da); hipFree(db); hipFree(dout);
  return h;
}

int main() {
  float a[32], b[32];
  // 1: big product first, then 31 tiny ones, C = -big
  for (int k = 0; k < 32; ++k) { a[k] = k == 0 ? 1024.f : ldexpf(1.f, -10); b[k] = k == 0 ? 1.f : ldexpf(1.f, -10); }
  printf("T1 big-first tiny: got %.10e  exact %.10e\n", run(a, b, -1024.f), 31 * ldexpf(1.f, -20));
  // 2: tiny first, big last
  for (int k = 0; k < 32; ++k) { a[k] = k == 31 ? 1024.f : ldexpf(1.f, -10); b[k] = k == 31 ? 1.f : ldexpf(1.f, -10); }
  printf("T2 big-last tiny : got %.10e  exact %.10e\n", run(a, b, -1024.f), 31 * ldexpf(1.f, -20));
  // 3: C = 0, big +x and -x cancel, tiny terms
  for (int k = 0; k < 32; ++k) { a[k] = ldexpf(1.f, -12); b[k] = ldexpf(1.f, -12); }
  a[5] = 2048.f; b[5] = 1024.f; a[20] = -2048.f; b[20] = 1024.f;
  printf("T3 cancel + tiny : got %.10e  exact %.10e\n", run(a, b, 0.f), 30 * ldexpf(1.f, -24));
  // 4: one subnormal f16 operand
  for (int k = 0; k < 32; ++k) { a[k] = 0.f; b[k] = 0.f; }
  a[3] = ldexpf(1.f, -20); b[3] = 1.f;
  printf("T4 subnormal a   : got %.10e  exact %.10e\n", run(a, b, 0.f), ldexpf(1.f, -20));
  a[3] = ldexpf(1.f, -14); b[3] = ldexpf(1.f, -14);
  printf("T5 tiny product  : got %.10e  exact %.10e\n", run(a, b, 0.f), ldexpf(1.f, -28));
  // 6: C large, products small: does C's rounding happen once?
  for (int k = 0; k < 32; ++k) { a[k] = ldexpf(1.f, -5); b[k] = ldexpf(1.f, -5); }
  printf("T6 C=1 + 32*2^-10: got %.10e  exact %.10e\n", run(a, b, 1.f), 1.f + 32 * ldexpf(1.f, -10));
  // 7: sum exceeding 24 bits in the middle: 2^24 + 1 - 2^24
  for (int k = 0; k < 32; ++k) { a[k] = 0.f; b[k] = 0.f; }
  a[0] = 2048.f; b[0] = 4096.f; a[1] = 1.f; b[1] = 1.f; a[2] = -2048.f; b[2] = 4096.f;
  printf("T7 2^23+1-2^23   : got %.10e  exact %.10e\n", run(a, b, 0.f), 1.0);
  a[0] = 2048.f; b[0] = 8192.f; a[2] = -2048.f; b[2] = 8192.f;
  printf("T8 2^24+1-2^24   : got %.10e  exact %.10e\n", run(a, b, 0.f), 1.0);
  // 9: many products, random exact
  double ex = 0; srand(1);
  for (int k = 0; k < 32; ++k) { a[k] = (float)(rand() % 2001 - 1000) / 64.f; b[k] = (float)(rand() % 2001 - 1000) / 1024.f; ex += (double)a[k] * b[k]; }
  printf("T9 random exact  : got %.10e  exact %.10e\n", run(a, b, 0.f), ex);
  // 10: small terms next to a large C
  for (int k = 0; k < 32; ++k) { a[k] = ldexpf(1.f, -14) * (k + 1); b[k] = ldexpf(1.f, -14); }
  ex = 0; for (int k = 0; k < 32; ++k) ex += (double)a[k] * b[k];
  printf("T10 C=3 + small  : got %.10e  exact %.10e\n", run(a, b, 3.f), 3.0 + ex);
  return 0;
}
