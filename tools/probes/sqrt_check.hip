// Exhaustive check (tools/probes, not part of the library): the fp32
// sqrt used by box_muller (v_sqrt_f32 + one-ulp fma fix-up, abc_common.h
// sqrt_rn) equals the correctly rounded sqrt ((float)sqrt((double)v)) for
// every fp32 v in [2^-26, 128), the range 2 (-ln u1) can take.
#include <cstdio>
#include <hip/hip_runtime.h>
#include "../../pyabc_amd/csrc/abc_common.h"

__global__ void k_check(uint32_t lo, uint32_t n, unsigned long long* bad,
                        uint32_t* first) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t bits = lo + i;
  const float v = __uint_as_float(bits);
  const float a = abc::sqrt_rn(v);
  const float b = (float)sqrt((double)v);
  if (__float_as_uint(a) != __float_as_uint(b)) {
    atomicAdd(bad, 1ull);
    atomicMin(first, bits);
  }
}

int main() {
  const uint32_t lo = 0x32800000u;  // 2^-26
  const uint32_t hi = 0x43000000u;  // 128
  const uint32_t n = hi - lo;
  unsigned long long* bad;
  uint32_t* first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 4);
  hipMemset(bad, 0, 8);
  hipMemset(first, 0xFF, 4);
  hipLaunchKernelGGL(k_check, dim3((n + 255) / 256), dim3(256), 0, 0, lo, n, bad, first);
  unsigned long long hb = 0;
  uint32_t hf = 0;
  hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
  printf("sqrt_rn vs correctly rounded: %u values, %llu mismatches (first 0x%08x)\n", n, hb,
         hf);
  return hb != 0;
}
