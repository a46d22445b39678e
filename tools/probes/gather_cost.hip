// Random-gather throughput probe: every thread reads `per` random records of
// `rb` bytes from a table of `tb` bytes (hash-spread indices), the access
// pattern of the fused round's ancestor table (guide entry + 128-B record).
// Reports records/s and GB/s of record payload; tools/probes, not library code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
template <int RW>  // record words (8 B each)
__global__ __launch_bounds__(256) void gather(const double* __restrict__ t, uint32_t nrec,
                                              int per, double* out) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  double acc = 0.0;
  for (int i = 0; i < per; ++i) {
    const uint32_t r = mix(g * 7919u + i * 104729u) % nrec;
    const double* p = t + (size_t)r * RW;
#pragma unroll
    for (int k = 0; k < RW; ++k) acc += p[k];
  }
  out[g] = acc;
}
// dependent pair: a 4-B guide entry from a table of ng entries, then the
// 128-B record it names
__global__ __launch_bounds__(256) void guide_then_record(const int32_t* __restrict__ gd,
                                                         uint32_t ng,
                                                         const double* __restrict__ t,
                                                         uint32_t nrec, int per, double* out) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  double acc = 0.0;
  for (int i = 0; i < per; ++i) {
    const uint32_t k = mix(g * 7919u + i * 104729u) % ng;
    const uint32_t r = (uint32_t)gd[k] % nrec;
    const double* p = t + (size_t)r * 16;
#pragma unroll
    for (int q = 0; q < 11; ++q) acc += p[q];
  }
  out[g] = acc;
}

int main() {
  const size_t TB = 256ull << 20;
  double* t; int32_t* gd; double* out;
  hipMalloc(&t, TB); hipMalloc(&gd, 64ull << 20);
  hipMemset(t, 0, TB);
  const int blocks = 256 * 64, per = 64;
  hipMalloc(&out, (size_t)blocks * 256 * 8);
  {
    int32_t* h = new int32_t[16 << 20];
    for (int i = 0; i < (16 << 20); ++i) h[i] = i / 4;
    hipMemcpy(gd, h, (16 << 20) * 4, hipMemcpyHostToDevice);
    delete[] h;
  }
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double n = (double)blocks * 256 * per;
  auto run = [&](const char* name, auto launch, double bytes) {
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    printf("%-44s %.3e accesses/s  %.2f TB/s payload\n", name, n / (ms * 1e-3),
           n * bytes / (ms * 1e-3) / 1e12);
  };
  for (size_t tbytes : {4ull << 20, 16ull << 20, 64ull << 20, 128ull << 20, 256ull << 20}) {
    char nm[128];
    const uint32_t n8 = tbytes / 8, n64 = tbytes / 64, n128 = tbytes / 128;
    snprintf(nm, 128, "8-B reads, table %zu MB", tbytes >> 20);
    run(nm, [&] { hipLaunchKernelGGL(gather<1>, blocks, 256, 0, 0, t, n8, per, out); }, 8);
    snprintf(nm, 128, "64-B records, table %zu MB", tbytes >> 20);
    run(nm, [&] { hipLaunchKernelGGL(gather<8>, blocks, 256, 0, 0, t, n64, per, out); }, 64);
    snprintf(nm, 128, "128-B records, table %zu MB", tbytes >> 20);
    run(nm, [&] { hipLaunchKernelGGL(gather<16>, blocks, 256, 0, 0, t, n128, per, out); }, 128);
  }
  run("guide 16 MB -> 128-B record (128 MB)", [&] {
    hipLaunchKernelGGL(guide_then_record, blocks, 256, 0, 0, gd, 4u << 20, t, 1u << 20, per, out); }, 132);
  run("guide 2 MB -> 128-B record (128 MB)", [&] {
    hipLaunchKernelGGL(guide_then_record, blocks, 256, 0, 0, gd, 1u << 19, t, 1u << 20, per, out); }, 132);
  return 0;
}
