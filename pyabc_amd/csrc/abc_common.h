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

// Resident blocks of a kernel on the current device: the occupancy query x
// CUs, cached per kernel and device (grids of ticket-scheduled kernels).
template <class K>
int resident_blocks(K kernel, int block, int fallback = 1024) {
  struct Entry { const void* k; int dev; int n; };
  static Entry cache[64];
  static int ncache = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fallback;
  for (int i = 0; i < ncache; ++i)
    if (cache[i].k == (const void*)kernel && cache[i].dev == dev) return cache[i].n;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      per_cu < 1 || cus < 1)
    return fallback;
  const int n = per_cu * cus;
  if (ncache < 64) cache[ncache++] = Entry{(const void*)kernel, dev, n};
  return n;
}

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
  // what is left after the pieces taken so far (256-byte aligned)
  void* rest() const { return base + align_up(off, 256); }
  size_t rest_bytes() const { return align_up(off, 256) < cap ? cap - align_up(off, 256) : 0; }
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
    // three-way xors as single v_bitop3_b32 (0x96 = a ^ b ^ c)
    uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
    uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
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
// Correctly rounded fp32 sqrt of a positive normal v: v_sqrt_f32 (within one
// ulp) and the one-ulp fix-up by the signs of the fma residuals of its
// neighbours (the sequence LLVM emits for IEEE sqrtf, without the denormal
// and special-value scaling v never needs).  Checked against
// (float)sqrt((double)v) on every fp32 in [2^-26, 128):
// tools/probes/sqrt_check.hip.
__device__ __forceinline__ float sqrt_rn(float v) {
  const float s = __builtin_amdgcn_sqrtf(v);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float em = __builtin_fmaf(-sm, s, v);
  const float ep = __builtin_fmaf(-sp, s, v);
  const float r = em <= 0.0f ? sm : s;
  return ep > 0.0f ? sp : r;
}

// Copy of BM_TAB in LDS (every thread of the block calls it; synchronises).
}  // namespace abc
#include "abc_bm_tables.h"
namespace abc {
__device__ __forceinline__ void stage_bm_tab(float* lds) {
  for (int k = threadIdx.x; k < BM_TAB_SIZE; k += blockDim.x) lds[k] = BM_TAB[k];
  __syncthreads();
}

// Box-Muller: n0 = R cos(2 pi u2), n1 = R sin(2 pi u2), R = sqrt(-2 ln u1),
// u1 = m1 2^-32 with m1 the whole 32-bit word a made odd, u2 = m2 2^-24 (m2
// odd, the top 23 bits of b: the angle).  Below 2^-23 (a < 2^9) u1 takes
// the 9 low bits of b, which the angle leaves unused, as 9 more bits: u1 =
// m1' 2^-41, m1' = (a << 9 | b & 511) made odd.  So u1 >= 2^-41 and R <=
// sqrt(82 ln 2) = 7.54: P(R > 7.54) = 2^-41, a normal's cut mass ~5e-14
// (32 bits alone cut at 6.66, mass 2.7e-11).  The
// transform is evaluated in fp32 with only correctly rounded operations in a
// fixed order (no contraction; sqrt_rn; 4 KB of tables), so that
// oracle/philox.py normal_pairs replays it bit for bit in numpy float32:
//   ln: m1 = 2^e f, f = c_i + delta with c_i = 1 + i/128 for the top 7
//     fraction bits i (delta, the next 24 bits, exact in fp32); ln f = ln c_i
//     + log1p(delta / c_i), the table value an fp32 pair and log1p a degree-4
//     series on [0, 2^-7); -ln u1 = (32 - e) ln2 - ln f, whose leading
//     difference is exact where it cancels; for u1 > 1 - 2^-8 the series of
//     -ln(1 - y), y = 1 - u1 exact (a rare branch);
//   sin/cos: angle = pi i / 128 + pi j 2^-23 (i, j = high 8 / low 16 bits of
//     m2): table sin/cos of the first, degree-3/4 series of the second,
//     combined by the angle-addition formulas.
// Within ~4 fp32 ulp of R of the exact transform (tests/test_gpu_fused.py).
// tab: BM_TAB or a copy of it in LDS (the hot kernels stage one per block).
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, double& n0,
                                           double& n1, const float* tab = BM_TAB) {
#pragma clang fp contract(off)
  constexpr float LN2_HI = 0x1.62e4p-1f;      // 17 significant bits
  constexpr float LN2_LO = 0x1.7f7d1cp-20f;   // ln 2 - LN2_HI
  constexpr float C3 = 0x1.555556p-2f, C5 = 0x1.99999ap-3f;  // 1/3, 1/5
  constexpr float C6 = 0x1.555556p-3f, C24 = 0x1.555556p-5f;  // 1/6, 1/24
  constexpr float PI_2M23 = 0x1.921fb6p-22f;  // pi 2^-23
  // ---- v = -ln u1, u1 = m1 2^-32
  const uint32_t m1 = a | 1u;
  const uint32_t yi = 0u - m1;                       // 2^32 - m1
  float v;
  if (yi < (1u << 24)) {
    const float y = (float)yi * 0x1p-32f;
    float z = y * C5 + 0.25f;
    z = z * y + C3;
    z = z * y + 0.5f;
    z = z * y + 1.0f;
    v = z * y;
  } else {
    // u1 < 2^-23: 41 bits, the 9 low bits of b below a's (m1' < 2^18)
    const bool ext = a < 512u;
    const uint32_t mt = ext ? ((a << 9) | (b & 511u) | 1u) : m1;
    const int e = 31 - __clz((int)mt);               // floor(log2 m), 0..31
    const uint32_t t = mt << (31 - e);               // leading one at bit 31
    const int i = (int)((t >> 24) & 127u);
    const float delta = (float)(t & 0xFFFFFFu) * 0x1p-31f;
    const float* lg = tab + BM_TAB_LOG + 4 * i;      // (INV_C, LN_HI, LN_LO, 0)
    const float r = delta * lg[0];
    float p = r * -0.25f + C3;
    p = p * r - 0.5f;
    p = p * r + 1.0f;
    p = p * r;                                       // log1p(r)
    const float k = (float)((ext ? 41 : 32) - e);    // k LN2_HI exact (<= 23 bits)
    v = (k * LN2_HI - lg[1]) + ((k * LN2_LO - lg[2]) - p);
  }
  const float R = sqrt_rn(2.0f * v);
  // ---- (cos, sin)(pi m2 2^-23), m2 = 2 (b >> 9) + 1
  const uint32_t m2 = ((b >> 9) << 1) | 1u;
  const float* sc = tab + BM_TAB_SC + 2 * (int)(m2 >> 16);
  const float bb = (float)(m2 & 0xFFFFu) * PI_2M23;
  const float b2 = bb * bb;
  const float sb = bb - (bb * b2) * C6;
  const float cb = 1.0f - b2 * (0.5f - b2 * C24);
  const float sa = sc[0], ca = sc[1];
  const float sn = sa * cb + ca * sb;
  const float cs = ca * cb - sa * sb;
  n0 = (double)(R * cs);
  n1 = (double)(R * sn);
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
