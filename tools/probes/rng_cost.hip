// Throughput probe: Philox4x32-10 and the Box-Muller transform per wave64
// instruction budget (tools/probes, not part of the library).
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
    a = a * 1664525u + 1013904223u; b = b ^ (a >> 7);
  }
  out[g] = acc;
}
int main() {
  const int blocks = 256 * 16, threads = 256, iters = 512;
  uint32_t* o; double* od;
  hipMalloc(&o, blocks * threads * 4); hipMalloc(&od, blocks * threads * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0); hipLaunchKernelGGL(k_philox, blocks, threads, 0, 0, o, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double n = (double)blocks * threads * iters;
    if (rep) printf("philox: %.3e /s (%.3f ns per 1e3)\n", n / ms * 1e3, ms * 1e6 / n * 1e3);
    hipEventRecord(e0); hipLaunchKernelGGL(k_bm, blocks, threads, 0, 0, od, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    if (rep) printf("box_muller pair: %.3e /s\n", n / ms * 1e3);
  }
  return 0;
}
