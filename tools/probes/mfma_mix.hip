// Throughput probe for the x3 density's inner unit (one 16x16 tile pair:
// an MFMA chain + 4 v_exp_f32 + 4 adds per lane), chain forms:
//   x32x3  : three v_mfma_f32_16x16x32_f16        (K = 96, HEAD)
//   x32x2  : two   v_mfma_f32_16x16x32_f16        (K = 64)
//   x32x2+16: two x32 + one v_mfma_f32_16x16x16_f16 (K = 80)
//   x16    : one v_mfma_f32_16x16x16_f16 alone, no exp (instruction cost)
//   x32    : one v_mfma_f32_16x16x32_f16 alone, no exp
// CT = 8 candidate tiles per wave as in mvn_x3_kernel; the exp2/sum of unit
// c - 1 is issued under the chain of unit c.  Reports ns per unit per SIMD
// and cycles at 2.4 GHz.  tools/probes, not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__device__ __forceinline__ f32x4 chain(const half8 (&a)[3], const half8 (&b)[3], half4 a4,
                                       half4 b4) {
  f32x4 r = {0.f, 0.f, 0.f, 0.f};
  if (MODE == 0 || MODE == 1 || MODE == 2 || MODE == 4) {
    r = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], r, 0, 0, 0);
  }
  if (MODE == 0 || MODE == 1 || MODE == 2)
    r = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[1], r, 0, 0, 0);
  if (MODE == 0) r = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[2], b[2], r, 0, 0, 0);
  if (MODE == 2 || MODE == 3) r = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, r, 0, 0, 0);
  return r;
}

template <int MODE, bool EXP>
__global__ __launch_bounds__(256) void k_mix(float* out, int iters) {
  constexpr int CT = 8;
  const int lane = threadIdx.x & 63;
  half8 a[3], b[CT][3];
  half4 a4, b4[CT];
  for (int k = 0; k < 3; ++k)
    for (int j = 0; j < 8; ++j) a[k][j] = (_Float16)(((lane + j + k) & 7) * 0.001f - 0.004f);
  for (int j = 0; j < 4; ++j) a4[j] = (_Float16)((lane + j) & 3) * (_Float16)0.001f;
  for (int c = 0; c < CT; ++c) {
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 8; ++j) b[c][k][j] = (_Float16)(((lane * 3 + j + c) & 7) * 0.001f);
    for (int j = 0; j < 4; ++j) b4[c][j] = (_Float16)((c + j) & 3) * (_Float16)0.001f;
  }
  float ls[CT];
  for (int c = 0; c < CT; ++c) ls[c] = 0.f;
  auto expsum = [&](const f32x4& v) {
    return (__builtin_amdgcn_exp2f(v[0]) + __builtin_amdgcn_exp2f(v[1])) +
           (__builtin_amdgcn_exp2f(v[2]) + __builtin_amdgcn_exp2f(v[3]));
  };
  for (int it = 0; it < iters; ++it) {
    f32x4 prev = chain<MODE>(a, b[0], a4, b4[0]);
#pragma unroll
    for (int c = 1; c < CT; ++c) {
      const f32x4 cur = chain<MODE>(a, b[c], a4, b4[c]);
      if (EXP) ls[c - 1] += expsum(prev);
      else ls[c - 1] += prev[0];
      prev = cur;
    }
    if (EXP) ls[CT - 1] += expsum(prev);
    else ls[CT - 1] += prev[0];
    // perturb a so the chain is not loop-invariant
    a[0][it & 7] = (_Float16)(ls[it & 7] * 1e-9f);
  }
  float s = 0.f;
  for (int c = 0; c < CT; ++c) s += ls[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, bool EXP>
void run(const char* name, float* d, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_mix<MODE, EXP>), dim3(blocks), dim3(256), 0, 0, d, 10);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_mix<MODE, EXP>), dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double units = (double)blocks * 4 * iters * 8;   // waves x iters x CT
  const double per_simd = units / 1024.0;
  printf("%-10s exp=%d: %.3f ms, %.2f ns/unit/SIMD = %.1f cycles @2.4GHz\n", name, (int)EXP,
         ms, 1e6 * ms / per_simd, 2.4e6 * ms / per_simd);
}

int main() {
  float* d;
  const int blocks = 2048, iters = 4000;
  hipMalloc(&d, sizeof(float) * blocks * 256);
  run<0, true>("x32x3", d, blocks, iters);
  run<1, true>("x32x2", d, blocks, iters);
  run<2, true>("x32x2+16", d, blocks, iters);
  run<0, false>("x32x3", d, blocks, iters);
  run<1, false>("x32x2", d, blocks, iters);
  run<2, false>("x32x2+16", d, blocks, iters);
  run<3, false>("x16", d, blocks, iters);
  run<4, false>("x32", d, blocks, iters);
  run<3, true>("x16", d, blocks, iters);
  run<4, true>("x32", d, blocks, iters);
  hipFree(d);
  return 0;
}
