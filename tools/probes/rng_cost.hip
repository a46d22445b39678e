// Throughput probe: Philox4x32-10, the Box-Muller transform and the 32-bit
// multiply forms, reported as issue cycles per wave64 instance (1024 SIMDs at
// 2.4 GHz); tools/probes, not part of the library.
#include <cstdio>
#include "../../pyabc_amd/csrc/abc_candidate.h"
using namespace abc;

__global__ void k_philox(uint32_t* out, int iters) {
  uint64_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    u32x4 r = philox(g, i, 7, 12345ull);
    acc ^= r.x ^ r.y ^ r.z ^ r.w;
  }
  out[g] = acc;
}
__global__ void k_bm(double* out, int iters) {
  __shared__ float t[BM_TAB_SIZE];
  stage_bm_tab(t);
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  double acc = 0;
  uint32_t a = g * 2654435761u, b = g * 40503u + 7;
  for (int i = 0; i < iters; ++i) {
    double n0, n1;
    box_muller(a, b, n0, n1, t);
    acc += n0 + n1;
    a = a + 0x9E3779B9u; b = b ^ (a >> 7);
  }
  out[g] = acc;
}
// 8 independent 32x32 -> 64 multiplies per iteration
__global__ void k_mad64(uint32_t* out, int iters) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c[8];
  for (int k = 0; k < 8; ++k) c[k] = g + k * 977u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t p = (uint64_t)0xD2511F53u * c[k];
      c[k] = (uint32_t)(p >> 32) ^ (uint32_t)p;
    }
  }
  uint32_t acc = 0;
  for (int k = 0; k < 8; ++k) acc ^= c[k];
  out[g] = acc;
}
__global__ void k_add(uint32_t* out, int iters) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c[8];
  for (int k = 0; k < 8; ++k) c[k] = g + k * 977u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_bitop3_b32(c[k] + 0xD2511F53u, c[k], 17u, 0x96);
  }
  uint32_t acc = 0;
  for (int k = 0; k < 8; ++k) acc ^= c[k];
  out[g] = acc;
}
int main() {
  const int blocks = 256 * 16, threads = 256, iters = 512;
  uint32_t* o; double* od;
  hipMalloc(&o, blocks * threads * 4); hipMalloc(&od, blocks * threads * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double n = (double)blocks * threads * iters;
  auto cyc = [&](double ms, double per) {  // issue cycles per wave64 instance
    return 1024.0 * 2.4e9 * 64.0 / (n * per / (ms * 1e-3));
  };
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipEventRecord(e0); hipLaunchKernelGGL(k_philox, blocks, threads, 0, 0, o, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    if (rep) printf("philox4x32-10: %.3e calls/s, %.1f cyc per wave call\n", n / ms * 1e3, cyc(ms, 1));
    hipEventRecord(e0); hipLaunchKernelGGL(k_bm, blocks, threads, 0, 0, od, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    if (rep) printf("box_muller: %.3e pairs/s, %.1f cyc per wave pair\n", n / ms * 1e3, cyc(ms, 1));
    hipEventRecord(e0); hipLaunchKernelGGL(k_mad64, blocks, threads, 0, 0, o, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    if (rep) printf("mad_u64_u32+xor: %.1f cyc per wave op pair\n", cyc(ms, 8));
    hipEventRecord(e0); hipLaunchKernelGGL(k_add, blocks, threads, 0, 0, o, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    if (rep) printf("add+bitop3: %.1f cyc per wave op pair\n", cyc(ms, 8));
  }
  return 0;
}
