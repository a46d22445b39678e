// Probe: how v_mfma_f32_16x16x32_f16 (gfx950) sums a K group that mixes
// large and tiny products, relative to the accumulator C.  Decides whether
// the x3 density can put its last "hi" (exact-grid) slots and its first
// "lo" slots into one 8-product group (mvn_x3_kernel's two-block layout).
// One wave; row 0 / column 0 carry the test vector, everything else zero.
//   hipcc -O2 --offload-arch=gfx950 mfma_f16_groups.hip -o mfma_f16_groups
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
  if (lane == 0) acc[0] = c0;
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];
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

static void clear(float* a, float* b) { for (int k = 0; k < 32; ++k) { a[k] = 0.f; b[k] = 0.f; } }

static void report(const char* name, const float* a, const float* b, float c0) {
  double ex = c0;
  for (int k = 0; k < 32; ++k) ex += (double)a[k] * (double)b[k];
  const float got = run(a, b, c0);
  printf("%-44s got % .17e exact % .17e  %s\n", name, got, ex,
         (double)got == ex ? "EXACT" : ((double)got == (double)(float)ex ? "rounded-once" : "DIFFERS"));
}

int main() {
  float a[32], b[32];
  const float tiny = ldexpf(1.f, -10);   // tiny x tiny = 2^-20
  // big term and tiny terms in ONE group (slots 0..7), C cancels the big one
  for (int big_e = 10; big_e <= 23; big_e += 1) {
    clear(a, b);
    a[0] = ldexpf(1.f, big_e > 11 ? 11 : big_e); b[0] = ldexpf(1.f, big_e > 11 ? big_e - 11 : 0);
    for (int k = 1; k < 8; ++k) { a[k] = tiny; b[k] = tiny; }
    char nm[64];
    snprintf(nm, 64, "G0: +2^%d + 7*2^-20, C=-2^%d", big_e, big_e);
    report(nm, a, b, -ldexpf(1.f, big_e));
  }
  // big in slots 8..11 (group 1), tiny in 12..15, C = -(sum of big)
  clear(a, b);
  for (int k = 8; k < 12; ++k) { a[k] = 2048.f; b[k] = 1024.f; }
  for (int k = 12; k < 16; ++k) { a[k] = tiny; b[k] = tiny * 3; }
  report("G1: 4*2^21 + 4*3*2^-20, C=-2^23", a, b, -ldexpf(1.f, 23));
  // cancellation inside the group, C = 0
  clear(a, b);
  a[0] = 2048.f; b[0] = 2048.f; a[1] = -2048.f; b[1] = 2048.f;
  for (int k = 2; k < 8; ++k) { a[k] = tiny; b[k] = tiny; }
  report("G0: +2^22 - 2^22 + 6*2^-20, C=0", a, b, 0.f);
  // group 0 exact big (multiples of 1) bringing C to ~1, then tiny group 1
  clear(a, b);
  a[0] = 2048.f; b[0] = 2048.f; a[1] = 3.f; b[1] = 1.f;
  for (int k = 8; k < 16; ++k) { a[k] = tiny; b[k] = tiny; }
  report("G0: 2^22+3, G1: 8*2^-20, C=-2^22", a, b, -ldexpf(1.f, 22));
  // in-group order: tiny first, big last, C cancels
  clear(a, b);
  for (int k = 0; k < 7; ++k) { a[k] = tiny; b[k] = tiny; }
  a[7] = 2048.f; b[7] = 2048.f;
  report("G0: 7*2^-20 then +2^22, C=-2^22", a, b, -ldexpf(1.f, 22));
  // mixed signs: big products that cancel across the group with small ones
  clear(a, b);
  a[0] = 1500.f; b[0] = 1000.f; a[1] = -1499.f; b[1] = 1000.f; a[2] = -1.f; b[2] = 999.f;
  a[3] = ldexpf(1.f, -12); b[3] = ldexpf(1.f, -12);
  report("G0: 1.5e6 - 1.499e6 - 999 + 2^-24, C=0", a, b, 0.f);
  // subnormal products next to big ones
  clear(a, b);
  a[0] = 1024.f; b[0] = 1.f; a[1] = ldexpf(1.f, -20); b[1] = ldexpf(1.f, -4);
  report("G0: 2^10 + 2^-24 (subnormal a), C=-2^10", a, b, -1024.f);
  return 0;
}
