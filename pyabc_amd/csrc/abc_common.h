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
void profile_start(hipStream_t s, int channel = ABC_PROF_DENSITY);
void profile_stop(hipStream_t s, int channel = ABC_PROF_DENSITY);

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
// Copy of BM_TAB in LDS (every thread of the block calls it; synchronises).
}  // namespace abc
#include "abc_bm_tables.h"
namespace abc {
__device__ __forceinline__ void stage_bm_tab(double* lds) {
  for (int k = threadIdx.x; k < BM_TAB_SIZE; k += blockDim.x) lds[k] = BM_TAB[k];
  __syncthreads();
}

// Box-Muller in fp64: n0 = R cos(2 pi u2), n1 = R sin(2 pi u2),
// R = sqrt(-2 ln u1), u = uniform01 (the formula of oracle.philox.normal_pairs).
// The uniforms carry 24 significant bits (u = m 2^-24, m odd), so the
// transform is table-driven instead of calling the general fp64 log /
// sincospi / sqrt (~200 VALU instructions per pair, most of the candidate
// kernels' work):
//   ln: m = 2^e f, f in [1, 2); with c = 1 + (i + 1/2)/256 for the top 8
//     fraction bits i, ln f = -ln(INV_C[i]) + log1p(f INV_C[i] - 1), the
//     table value a double-double and log1p a degree-7 series on
//     |r| < 2^-8; -ln u1 = (24 - e) ln2 - ln f, where the leading
//     difference is exact when it cancels (Sterbenz), so the result is good to
//     ~1 ulp even for u1 -> 1;
//   sqrt: v_rsq_f64 seed + two Newton steps + one residual correction;
//   sin/cos: angle = pi i / 128 + pi j 2^-23 (i, j = high 8 / low 16 bits of
//     m2): table sin/cos of the first + degree-7/8 series of the second,
//     combined by the angle-addition formulas.
// Agrees with the libm formula to a few ulp (the oracle tests' 1e-12).

// tab: BM_TAB or a copy of it in LDS (the hot kernels stage one per block:
// three random-index table reads per pair from global memory cost more
// latency than the arithmetic they save)
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, double& n0,
                                           double& n1, const double* tab = BM_TAB) {
  constexpr double LN2_HI = 0x1.62e42fefa3800p-1;   // 42 significant bits
  constexpr double LN2_LO = 0x1.ef35793c76730p-45;  // ln 2 - LN2_HI
  // ---- R = sqrt(-2 ln u1), u1 = m1 2^-24
  const uint32_t m1 = ((a >> 9) << 1) | 1u;
  const int e = 31 - __clz((int)m1);                // floor(log2 m1), 0..23
  const uint32_t t = m1 << (31 - e);                // leading one at bit 31
  const int i = (int)((t >> 23) & 255u);
  const double f = (double)(t >> 8) * 0x1p-23;      // m1 / 2^e in [1, 2), exact
  const double ic = tab[BM_TAB_LOG + 2 * i], lh = tab[BM_TAB_LOG + 2 * i + 1];
  const double ll = tab[BM_TAB_LO + i];
  const double r = fma(f, ic, -1.0);
  double q = fma(r, 1.0 / 7.0, -1.0 / 6.0);
  q = fma(r, q, 1.0 / 5.0);
  q = fma(r, q, -1.0 / 4.0);
  q = fma(r, q, 1.0 / 3.0);
  q = fma(r, q, -0.5);
  const double p = fma(r * r, q, r);                // log1p(r)
  const double k = (double)(24 - e);
  double v = fma(k, LN2_HI, -lh) + (fma(k, LN2_LO, -ll) - p);  // -ln u1
  const uint32_t yi = (1u << 24) - m1;
  if (yi < (1u << 15)) {
    // u1 > 1 - 2^-9: -ln u1 cancels to |v| >= 2^-24 above; the series of
    // -ln(1 - y), y = 1 - u1 exact, keeps it to an ulp (rare: a branch)
    const double yy = (double)yi * 0x1p-24;
    double z = fma(yy, 1.0 / 7.0, 1.0 / 6.0);
    z = fma(yy, z, 1.0 / 5.0);
    z = fma(yy, z, 1.0 / 4.0);
    z = fma(yy, z, 1.0 / 3.0);
    z = fma(yy, z, 0.5);
    v = fma(yy * yy, z, yy);
  }
  const double x = 2.0 * v;
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  double c = fma(-hx * y, y, 0.5);
  y = fma(y, c, y);
  c = fma(-hx * y, y, 0.5);
  y = fma(y, c, y);
  double R = x * y;
  R = fma(fma(-R, R, x), 0.5 * y, R);
  // ---- (cos, sin)(pi m2 2^-23), m2 = 2 (b >> 9) + 1
  const uint32_t m2 = ((b >> 9) << 1) | 1u;
  const int ia = (int)(m2 >> 16);
  const double ang = (double)(m2 & 0xFFFFu) * 0x1.921fb54442d18p-22;  // pi 2^-23 j
  const double a2 = ang * ang;
  double ps = fma(a2, -1.0 / 5040.0, 1.0 / 120.0);
  ps = fma(a2, ps, -1.0 / 6.0);
  const double sb = fma(ang * a2, ps, ang);
  double pc = fma(a2, 1.0 / 40320.0, -1.0 / 720.0);
  pc = fma(a2, pc, 1.0 / 24.0);
  pc = fma(a2, pc, -0.5);
  const double cb = fma(a2, pc, 1.0);
  const double sa = tab[BM_TAB_SC + 2 * ia], ca = tab[BM_TAB_SC + 2 * ia + 1];
  const double sn = fma(sa, cb, ca * sb);
  const double cs = fma(ca, cb, -(sa * sb));
  n0 = R * cs;
  n1 = R * sn;
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
