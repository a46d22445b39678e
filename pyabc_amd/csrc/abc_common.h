// Shared device/host helpers for libabcgpu (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <math.h>
#include "../../include/abcgpu.h"

namespace abc {

// ---- error reporting (abc_errors.cpp) --------------------------------------
int set_error(int code, const char* fmt, ...);
// HIP-event timing around the dominant kernel's launch (abc_profile.cpp)
void profile_start(hipStream_t s);
void profile_stop(hipStream_t s);

#define ABC_CHECK_ARG(cond, ...)                                           \
  do { if (!(cond)) return ::abc::set_error(ABC_ERR_INVALID, __VA_ARGS__); } while (0)
#define ABC_HIP(call)                                                      \
  do { hipError_t e_ = (call);                                             \
       if (e_ != hipSuccess)                                               \
         return ::abc::set_error(ABC_ERR_HIP, "%s: %s (%s:%d)", #call,     \
                                 hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)
#define ABC_LAUNCHED()                                                     \
  do { hipError_t e_ = hipGetLastError();                                  \
       if (e_ != hipSuccess)                                               \
         return ::abc::set_error(ABC_ERR_HIP, "launch: %s (%s:%d)",         \
                                 hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Carve consecutive 256-B aligned regions out of a caller workspace.
struct Carver {
  char* base; size_t cap; size_t off = 0; bool ok = true;
  Carver(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <class T> T* take(size_t n) {
    size_t start = align_up(off, 256);
    off = start + n * sizeof(T);
    if (off > cap) ok = false;
    return reinterpret_cast<T*>(base + start);
  }
};
template <class T> inline void size_only(size_t& off, size_t n) {
  off = align_up(off, 256) + n * sizeof(T);
}

// ---- Philox4x32-10 (oracle/philox.py restates this bit for bit) -----------
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox(uint64_t index, uint32_t slot,
                                        uint32_t generation, uint64_t seed) {
  uint32_t c0 = (uint32_t)index, c1 = (uint32_t)(index >> 32), c2 = slot,
           c3 = generation;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

// u32 -> (0,1), exact in fp32: ((x >> 9) + 0.5) * 2^-23
__device__ __forceinline__ double uniform01(uint32_t x) {
  return ((double)(x >> 9) + 0.5) * 1.1920928955078125e-07;
}
// numpy random_double: 53-bit [0,1)
__device__ __forceinline__ double uniform53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) *
         (1.0 / 9007199254740992.0);
}
// Box-Muller in fp64 (the same formula as oracle.philox.normal_pairs).
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, double& n0,
                                           double& n1) {
  double u1 = uniform01(a), u2 = uniform01(b);
  double r = sqrt(-2.0 * log(u1));
  double s, c;
  sincospi(2.0 * u2, &s, &c);
  n0 = r * c; n1 = r * s;
}

// ---- wave helpers (wave64) ---------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace abc
