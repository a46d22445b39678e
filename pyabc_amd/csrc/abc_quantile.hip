// QuantileEpsilon's weighted quantile as a weighted MSD select: no sort of
// the N points.
//
// Reference: pyabc/weighted_statistics.py:27-43 via QuantileEpsilon._update
// (pyabc/epsilon/epsilon.py:202-228):
//   sorted = argsort(points); cs = cumsum(w[sorted]); xp = (cs - w/2) / cs[-1]
//   q = np.interp(alpha, xp, points[sorted])
// np.interp only reads the two knots around alpha, so only the points whose
// cumulative weight lies near alpha * total need ordering.
//
// Keys are the order-preserving u64 images of the points (-0.0 == +0.0, ties
// broken by index like the stable sort).  Weights enter the search as 62-bit
// fixed-point integers (w * 2^(62 - ceil log2 N) / max w, truncated), so the
// histograms' sums are exact integers, independent of any order -- the search
// is deterministic -- and each bin's cumulative weight is known to within N
// units.  Four kernels (the control block is left zeroed for the next
// call, no memset); each
// single-block step runs in the last block of the multi-block kernel before
// it (device-scope fence + counter), so there is no one-block launch:
//   1. range: min / max key and max weight (integer max atomics);
//   2. hist (level 1): 2048 bins linear in the key span, counts and
//      fixed-point weight sums per bin (LDS atomics, integer); its last
//      block picks the bins that can hold the knots j, j + 1 (every bin whose
//      cumulative weight interval, widened by the fixed-point error, reaches
//      alpha * total, plus one bin on each side that certainly lies below /
//      above it) -> a key segment [lo, hi];
//   3. hist + pick (level 2) inside that segment when it holds more than
//      WQ_REFINE points (every block exits at once otherwise); level 1 uses
//      2048 bins (half the global atomics), level 2 4096;
//   4. gather: the segment's points (key, index, w) into a list, and the
//      fp64 sums of the weights below the segment and of all weights (fixed
//      per-thread order + fixed tree: deterministic); its last block sorts
//      the list by (key, index) in LDS (rank sort: every point counts the
//      points before it), forms the cumulative weights from the
//      sum below, xp and np.interp's rules (quantile_pick semantics: clamps,
//      exact knot hit, NaN fallbacks).
// Up to 2^20 points (c3's population) the same stages run in ONE launch on a
// resident grid, the points held in registers and the stages handed on by
// counters and flags instead of kernel boundaries (wq_onepass_kernel below:
// 0.045 vs 0.069 ms at 1e6).
// A segment that still holds more than WQ_CAP points after level 2 (ties by
// the thousand at the knots, e.g. discrete distances) is not decided here:
// *q = NaN, and the host (gpu.weighted_quantile's readers) reruns the exact
// sort-based abc_weighted_quantile_sorted on the same inputs.
#include <type_traits>

#include "abc_common.h"

namespace abc {
namespace {

constexpr int WQ_T = 1024;
constexpr int WQ_BITS = 12, WQ_NB = 1 << WQ_BITS;   // level 2 (and the buffers)
constexpr int WQ_BITS1 = 11;                        // level 1: half the global atomics
constexpr int WQ_REFINE = 256;   // level 1's segment is refined above this many points
constexpr int WQ_CAP = 2048;     // list capacity (level 2's segment; ties)
constexpr int WQ_U = 4;          // loads in flight per thread in the streaming loops
constexpr int WQ_MAXB = 256;
constexpr int WQ_FT = WQ_T;  // the final runs in the last gather block
static_assert(WQ_MAXB <= WQ_FT, "the final sums one gather block per thread");
static_assert(WQ_CAP % WQ_FT == 0 && WQ_FT % WQ_REFINE == 0, "rank sort layout");

typedef unsigned long long u64;

__device__ __forceinline__ u64 qkey(double v) {
  if (v == 0.0) v = 0.0;
  const u64 b = (u64)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double qval(u64 k) {
  const u64 b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

// per-call control block, zero when a call starts (the workspace is zeroed
// once; the gather's last block resets it): the global
// key range (kmin stored complemented, so zero is the identity of the max
// atomics), the last-block counters of the three multi-block stages (the
// one-launch path: done[0] its arrival counter, done[1] its hand-off flag),
// the fixed-point total and the list counter; pad != 0 marks a one-launch
// call whose wait timed out
struct WqCtl {
  u64 nkmin, kmax, wmax;
  unsigned int done[4];
  u64 tot;
  unsigned int list_n, pad;
};
struct WqDesc {
  u64 lo, hi;          // key segment [lo, hi] (inclusive)
  u64 base_w;          // fixed-point weight below lo
  long long count;     // points in [lo, hi]
  long long below;     // points below lo
  int ok;              // segment fits WQ_CAP
  int done;            // (level 2) nothing more to refine
};

__device__ __forceinline__ int lg_ceil(int64_t N) {
  return N <= 1 ? 0 : 64 - __clzll((u64)(N - 1));
}
// fixed-point weight (non-negative, finite weights; anything else counts 0)
__device__ __forceinline__ u64 wfix(double w, double S) {
  return (w > 0.0 && w < INFINITY) ? (u64)(w * S) : 0ull;
}
__device__ __forceinline__ double wval(double w) { return (w > 0.0 && w < INFINITY) ? w : 0.0; }

// block-wide min / max / sum helpers (WQ_T threads)
template <class T, class Op>
__device__ __forceinline__ T block_reduce(T v, T* sh, Op op) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  T r = sh[0];
  for (int i = 1; i < WQ_T / 64; ++i) r = op(r, sh[i]);
  __syncthreads();
  return r;
}

struct Range { u64 kmin, kmax; double S; };
__device__ __forceinline__ Range wq_global_range(const WqCtl* ctl, int64_t N) {
  Range r{~ctl->nkmin, ctl->kmax, 0.0};
  const double wmax = __longlong_as_double((long long)ctl->wmax);
  r.S = wmax > 0.0 ? ldexp(1.0, 62 - lg_ceil(N)) / wmax : 0.0;
  return r;
}

template <int BITS = WQ_BITS>
__device__ __forceinline__ int span_shift(u64 lo, u64 hi) {
  const u64 span = hi - lo;
  const int L = span ? 64 - __clzll(span) : 0;
  return L > BITS ? L - BITS : 0;
}

// ---- 1. range ----------------------------------------------------------------
__global__ __launch_bounds__(WQ_T) void wq_range_kernel(const double* __restrict__ x,
                                                        const double* __restrict__ w,
                                                        int64_t N, int64_t chunk,
                                                        WqCtl* __restrict__ ctl,
                                                        unsigned int* __restrict__ ghc,
                                                        u64* __restrict__ ghw) {
  __shared__ u64 sh[WQ_T / 64];
  // zero both levels' global histograms (the hist kernels add into them)
  for (int64_t e = (int64_t)blockIdx.x * WQ_T + threadIdx.x; e < 2 * WQ_NB;
       e += (int64_t)gridDim.x * WQ_T) {
    ghc[e] = 0u;
    ghw[e] = 0ull;
  }
  const int64_t b0 = (int64_t)blockIdx.x * chunk;
  const int64_t b1 = b0 + chunk < N ? b0 + chunk : N;
  u64 mn = ~0ull, mx = 0ull, wm = 0ull;
  for (int64_t i0 = b0 + threadIdx.x; i0 < b1; i0 += WQ_U * WQ_T) {
    double xv[WQ_U], wv[WQ_U];
#pragma unroll
    for (int u = 0; u < WQ_U; ++u) {
      const int64_t i = i0 + (int64_t)u * WQ_T;
      xv[u] = i < b1 ? x[i] : x[i0];
      wv[u] = i < b1 ? w[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < WQ_U; ++u) {
      const u64 k = qkey(xv[u]);
      mn = k < mn ? k : mn;
      mx = k > mx ? k : mx;
      const u64 wb = (u64)__double_as_longlong(wval(wv[u]));  // >= 0: bits order like values
      wm = wb > wm ? wb : wm;
    }
  }
  auto umin = [](u64 a, u64 b) { return a < b ? a : b; };
  auto umax = [](u64 a, u64 b) { return a > b ? a : b; };
  mn = block_reduce(mn, sh, umin);
  mx = block_reduce(mx, sh, umax);
  wm = block_reduce(wm, sh, umax);
  // one global range: integer max atomics (order-free) on the zeroed control
  // block, the minimum as the max of the complement
  if (threadIdx.x == 0) {
    atomicMax(reinterpret_cast<unsigned long long*>(&ctl->nkmin), (unsigned long long)~mn);
    atomicMax(reinterpret_cast<unsigned long long*>(&ctl->kmax), (unsigned long long)mx);
    atomicMax(reinterpret_cast<unsigned long long*>(&ctl->wmax), (unsigned long long)wm);
  }
}

template <class T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Last-block hand-over.  Everything one stage hands to its last block is
// written by agent-scope atomics (histogram adds, list / partial-sum stores
// through __hip_atomic_store) and read there by agent-scope atomic loads, so
// no L2 write-back is needed per block: each wave waits for its own memory
// operations to complete, the block's counter is bumped once, and the block
// that brings it to the grid size runs the stage's tail (pick / final) after
// one acquire fence.  The single-block kernels and their launch gaps go.
// The counter's bump is a release (one per block: the block's writes,
// ordered before it by the barrier, happen-before the last block's reads)
// and the last block's acquire pairs with it, as the HIP / LLVM memory model
// requires on a multi-XCD part.
__device__ __forceinline__ bool wq_last_block(unsigned int* done) {
  __shared__ int s_last;
  __builtin_amdgcn_s_waitcnt(0);   // this wave's atomics / stores completed
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
             gridDim.x - 1;
  __syncthreads();
  if (!s_last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// the control block back to zero for the next call (the gather's last block,
// after every stage has read it): no memset per call
__device__ __forceinline__ void wq_reset(WqCtl* ctl) {
  if (threadIdx.x == 0) {
    st_agent(&ctl->nkmin, 0ull);
    st_agent(&ctl->kmax, 0ull);
    st_agent(&ctl->wmax, 0ull);
    st_agent(&ctl->tot, 0ull);
    st_agent(&ctl->list_n, 0u);
#pragma unroll
    for (int i = 0; i < 4; ++i) st_agent(&ctl->done[i], 0u);
  }
}

__device__ __forceinline__ void seg_keys(u64 lo, u64 hi, int sh, int b1, int b2, u64& slo,
                                         u64& shi) {
  slo = lo + ((u64)b1 << sh);
  const u64 off = ((u64)b2 << sh) + ((1ull << sh) - 1ull);
  shi = off >= hi - lo ? hi : lo + off;
}

// ---- pick the segment of one level (the last histogram block) --------------
// Per-bin totals from the level's global histogram (integers), exclusive
// prefixes by a block scan held in registers (4 bins per thread), and the
// segment: from the last non-empty bin whose whole weight interval lies
// certainly below the target to the first whose interval lies certainly
// above it (the knots j and j + 1 lie between them, inclusive).  Block
// reductions by wave shuffles (no same-address LDS atomics).
// The level-1 pick also returns the input's fixed-point total (tot_out),
// which level 2 takes as tot_in.
template <int BITS>
__device__ void wq_pick_block(int64_t N, double alpha, const unsigned int* ghc,
                              const u64* ghw, u64 lo, u64 hi, u64 base_w, long long base_c,
                              bool level1, double tot_in, u64* tot_out, WqDesc* out) {
  constexpr int NB = 1 << BITS, PER = NB >= WQ_T ? NB / WQ_T : 1;
  __shared__ u64 s_w[WQ_T / 64];
  __shared__ long long s_c[WQ_T / 64];
  __shared__ int s_i[4][WQ_T / 64];
  __shared__ u64 s_bw;
  __shared__ long long s_bc, s_ec;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  unsigned int c[PER];
  u64 wsm[PER];
  u64 sw = 0ull;
  long long sc = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const bool has = NB >= WQ_T || t < NB;   // fewer bins than threads: the rest hold 0
    c[i] = has ? ld_agent(&ghc[t * PER + i]) : 0u;
    wsm[i] = has ? ld_agent(&ghw[t * PER + i]) : 0ull;
    sw += wsm[i];
    sc += c[i];
  }
  // inclusive wave scans, then the waves' totals in order
  u64 iw = sw;
  long long ic = sc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u64 a = __shfl_up(iw, o, 64);
    const long long b = __shfl_up(ic, o, 64);
    if (lane >= o) { iw += a; ic += b; }
  }
  if (lane == 63) { s_w[wv] = iw; s_c[wv] = ic; }
  __syncthreads();
  u64 tw = 0ull, ow = iw - sw;
  long long oc = ic - sc;
  for (int i = 0; i < WQ_T / 64; ++i) {
    tw += s_w[i];
    if (i < wv) { ow += s_w[i]; oc += s_c[i]; }
  }
  // the whole input's fixed-point total: summed at level 1 and kept in the
  // control block for level 2
  const double tot_fx = level1 ? (double)tw : tot_in;
  const double target = alpha * tot_fx;
  const double margin = (double)N + ldexp(tot_fx, -48) + 4096.0;
  ow += base_w;
  // b1 = last non-empty bin with pre + W + margin <= target (else the first
  // non-empty bin); b2 = first non-empty bin with pre - margin > target
  // (else the last non-empty bin)
  int cb1 = -1, cb2 = NB, first = NB, last = -1;
  {
    u64 pw = ow;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int b = t * PER + i;
      if (c[i]) {
        first = min(first, b);
        last = max(last, b);
        if ((double)(pw + wsm[i]) + margin <= target) cb1 = max(cb1, b);
        if ((double)pw - margin > target) cb2 = min(cb2, b);
      }
      pw += wsm[i];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cb1 = max(cb1, __shfl_xor(cb1, o, 64));
    cb2 = min(cb2, __shfl_xor(cb2, o, 64));
    first = min(first, __shfl_xor(first, o, 64));
    last = max(last, __shfl_xor(last, o, 64));
  }
  if (lane == 0) { s_i[0][wv] = cb1; s_i[1][wv] = cb2; s_i[2][wv] = first; s_i[3][wv] = last; }
  __syncthreads();
  for (int i = 0; i < WQ_T / 64; ++i) {
    cb1 = max(cb1, s_i[0][i]);
    cb2 = min(cb2, s_i[1][i]);
    first = min(first, s_i[2][i]);
    last = max(last, s_i[3][i]);
  }
  int b1 = cb1 >= 0 ? cb1 : first;
  int b2 = cb2 < NB ? cb2 : last;
  if (b1 >= NB) b1 = 0;      // no point in range (cannot happen: guards)
  if (b2 < b1) b2 = b1;
  {
    u64 pw = ow;
    long long pc = oc;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int b = t * PER + i;
      if (b == b1) { s_bw = pw; s_bc = pc; }
      if (b == b2) s_ec = pc + c[i];
      pw += wsm[i];
      pc += c[i];
    }
  }
  __syncthreads();
  if (t == 0) {
    WqDesc d;
    seg_keys(lo, hi, span_shift<BITS>(lo, hi), b1, b2, d.lo, d.hi);
    d.base_w = s_bw;
    d.below = base_c + s_bc;
    d.count = s_ec - s_bc;
    d.ok = d.count <= (level1 ? WQ_REFINE : WQ_CAP) ? 1 : 0;
    d.done = 0;
    *out = d;
    if (level1) *tot_out = (u64)__double_as_longlong((double)tw);
  }
}

// The same pick by one wave (wave 0 of the block; the other waves do not
// take part) for levels of at most 256 bins (4 per lane): the scans and
// reductions are shuffles only -- no block barrier, no LDS -- and every
// decision is the block version's (same prefix sums, same rules).
template <int BITS>
__device__ void wq_pick_wave(int64_t N, double alpha, const unsigned int* ghc,
                             const u64* ghw, u64 lo, u64 hi, u64 base_w, long long base_c,
                             bool level1, double tot_in, u64* tot_out, WqDesc* out) {
  constexpr int NB = 1 << BITS, PER = NB / 64;
  static_assert(NB % 64 == 0 && PER <= 4, "wave pick: 64 .. 256 bins");
  const int lane = threadIdx.x & 63;
  unsigned int c[PER];
  u64 wsm[PER];
  u64 sw = 0ull;
  long long sc = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    c[i] = ld_agent(&ghc[lane * PER + i]);
    wsm[i] = ld_agent(&ghw[lane * PER + i]);
    sw += wsm[i];
    sc += c[i];
  }
  u64 iw = sw;
  long long ic = sc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u64 a = __shfl_up(iw, o, 64);
    const long long b = __shfl_up(ic, o, 64);
    if (lane >= o) { iw += a; ic += b; }
  }
  const u64 tw = __shfl(iw, 63, 64);
  u64 ow = iw - sw;
  const long long oc = ic - sc;
  const double tot_fx = level1 ? (double)tw : tot_in;
  const double target = alpha * tot_fx;
  const double margin = (double)N + ldexp(tot_fx, -48) + 4096.0;
  ow += base_w;
  int cb1 = -1, cb2 = NB, first = NB, last = -1;
  {
    u64 pw = ow;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int b = lane * PER + i;
      if (c[i]) {
        first = min(first, b);
        last = max(last, b);
        if ((double)(pw + wsm[i]) + margin <= target) cb1 = max(cb1, b);
        if ((double)pw - margin > target) cb2 = min(cb2, b);
      }
      pw += wsm[i];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cb1 = max(cb1, __shfl_xor(cb1, o, 64));
    cb2 = min(cb2, __shfl_xor(cb2, o, 64));
    first = min(first, __shfl_xor(first, o, 64));
    last = max(last, __shfl_xor(last, o, 64));
  }
  int b1 = cb1 >= 0 ? cb1 : first;
  int b2 = cb2 < NB ? cb2 : last;
  if (b1 >= NB) b1 = 0;
  if (b2 < b1) b2 = b1;
  // the prefix at b1 and the end of b2: held by one lane each, summed over
  // the wave (every other lane adds zero)
  u64 bw = 0ull;
  long long bc = 0, ec = 0;
  {
    u64 pw = ow;
    long long pc = oc;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int b = lane * PER + i;
      if (b == b1) { bw = pw; bc = pc; }
      if (b == b2) ec = pc + c[i];
      pw += wsm[i];
      pc += c[i];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    bw += __shfl_xor(bw, o, 64);
    bc += __shfl_xor(bc, o, 64);
    ec += __shfl_xor(ec, o, 64);
  }
  if (lane == 0) {
    WqDesc d;
    seg_keys(lo, hi, span_shift<BITS>(lo, hi), b1, b2, d.lo, d.hi);
    d.base_w = bw;
    d.below = base_c + bc;
    d.count = ec - bc;
    d.ok = d.count <= (level1 ? WQ_REFINE : WQ_CAP) ? 1 : 0;
    d.done = 0;
    *out = d;
    if (level1) *tot_out = (u64)__double_as_longlong((double)tw);
  }
}

// ---- 2./3. histogram of one level + its pick --------------------------------
// level 1: the whole key range; level 2: the level-1 segment (every block
// exits when the level-1 segment fits).  The block's LDS histogram goes into
// the level's global histogram by integer atomics (totals independent of the
// blocks' order); the last block picks the segment.
template <int LEVEL>
__global__ __launch_bounds__(WQ_T) void wq_hist_kernel(
    const double* __restrict__ x, const double* __restrict__ w, int64_t N, int64_t chunk,
    double alpha, WqCtl* __restrict__ ctl, WqDesc* __restrict__ desc,
    unsigned int* __restrict__ ghc, u64* __restrict__ ghw) {
  constexpr int BITS = LEVEL == 1 ? WQ_BITS1 : WQ_BITS, NB = 1 << BITS;
  const WqDesc* prev = LEVEL == 2 ? desc : nullptr;
  if (prev && prev->ok) return;
  __shared__ unsigned int cnt[NB];
  __shared__ u64 ws[NB];
  for (int b = threadIdx.x; b < NB; b += WQ_T) { cnt[b] = 0u; ws[b] = 0ull; }
  const Range R = wq_global_range(ctl, N);
  const u64 lo = prev ? prev->lo : R.kmin, hi = prev ? prev->hi : R.kmax;
  const int sh = span_shift<BITS>(lo, hi);
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * chunk;
  const int64_t b1 = b0 + chunk < N ? b0 + chunk : N;
  for (int64_t i0 = b0 + threadIdx.x; i0 < b1; i0 += WQ_U * WQ_T) {
    u64 kv[WQ_U];
#pragma unroll
    for (int u = 0; u < WQ_U; ++u) {
      const int64_t i = i0 + (int64_t)u * WQ_T;
      kv[u] = i < b1 ? qkey(x[i]) : ~0ull;
    }
#pragma unroll
    for (int u = 0; u < WQ_U; ++u) {
      const int64_t i = i0 + (int64_t)u * WQ_T;
      if (i >= b1 || kv[u] < lo || kv[u] > hi) continue;
      const int bin = (int)((kv[u] - lo) >> sh);
      atomicAdd(&cnt[bin], 1u);
      atomicAdd(&ws[bin], wfix(w[i], R.S));
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < NB; b += WQ_T) {
    if (cnt[b]) {
      atomicAdd(&ghc[b], cnt[b]);
      atomicAdd(reinterpret_cast<unsigned long long*>(&ghw[b]), (unsigned long long)ws[b]);
    }
  }
  if (!wq_last_block(&ctl->done[LEVEL - 1])) return;
  wq_pick_block<BITS>(N, alpha, ghc, ghw, lo, hi, prev ? prev->base_w : 0ull,
                      prev ? prev->below : 0, LEVEL == 1,
                      LEVEL == 1 ? 0.0 : __longlong_as_double((long long)ctl->tot), &ctl->tot,
                      desc + (LEVEL - 1));
}

// ---- 7. final ---------------------------------------------------------------
// np.interp(alpha, xp, fp) on the knots around alpha; k0 = global index of
// the first listed element, n = N
struct Knot { double xp, fp; };
__device__ double interp_rules(double alpha, Knot first, Knot last, bool at_start, bool at_end,
                               const Knot* kn, int m, bool& ok) {
  ok = true;
  if (at_end && alpha > last.xp) return last.fp;
  if (at_start && alpha < first.xp) return first.fp;
  int lo = 0, hi = m;  // first with xp > alpha
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (kn[mid].xp > alpha) hi = mid; else lo = mid + 1;
  }
  const int j = lo - 1;
  if (j < 0 || (j == m - 1 && !at_end)) { ok = false; return NAN; }
  if (j == m - 1) return kn[j].fp;
  const double xj = kn[j].xp, xj1 = kn[j + 1].xp, yj = kn[j].fp, yj1 = kn[j + 1].fp;
  if (xj == alpha) return yj;
  const double slope = (yj1 - yj) / (xj1 - xj);
  double r = slope * (alpha - xj) + yj;
  if (isnan(r)) {
    r = slope * (alpha - xj1) + yj1;
    if (isnan(r) && yj == yj1) r = yj;
  }
  return r;
}

__device__ __forceinline__ bool kless(u64 ka, int ia, u64 kb, int ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// ---- the final (one block) ------------------------------------------------------
// The gather blocks' fp64 sums, the segment's list sorted by (key, index),
// the cumulative weights and np.interp's rules.
struct WqFinalLds {
  u64 skey[WQ_CAP];
  int sidx[WQ_CAP];
  double sw[WQ_CAP];
  Knot kn[WQ_CAP];
  int srank[WQ_CAP];
};

__device__ void wq_final(const WqDesc D, int64_t N, double alpha, int nsum,
                         const double* psum, const u64* gkey, const int* gidx, const double* gw,
                         double* q, WqFinalLds& L) {
  u64* skey = L.skey;
  int* sidx = L.sidx;
  double* sw = L.sw;
  Knot* kn = L.kn;
  __shared__ double dsh[WQ_FT / 64];
  const int t = threadIdx.x;
  if (!D.ok) {   // the knots sit in more than WQ_CAP points (ties): not decided
    if (t == 0) *q = NAN;
    return;
  }
  const int m = (int)D.count;
  // the gather blocks' fp64 sums and the listed points: all loads in flight
  // together, then the sums by a fixed tree (lanes, then waves in order)
  __shared__ double s_bt[2][WQ_FT / 64];
  __shared__ double s_below, s_total;
  {
    double bl = t < nsum ? ld_agent(&psum[2 * t]) : 0.0;
    double al = t < nsum ? ld_agent(&psum[2 * t + 1]) : 0.0;
    constexpr int PT = WQ_CAP / WQ_FT;
    u64 lk[PT];
    int li[PT];
    double lw[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int e = t + q * WQ_FT;
      if (e < m) {
        lk[q] = ld_agent(&gkey[e]);
        li[q] = ld_agent(&gidx[e]);
        lw[q] = ld_agent(&gw[e]);
      }
    }
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int e = t + q * WQ_FT;
      if (e < m) { skey[e] = lk[q]; sidx[e] = li[q]; sw[e] = lw[q]; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      bl += __shfl_xor(bl, o, 64);
      al += __shfl_xor(al, o, 64);
    }
    if ((t & 63) == 0) { s_bt[0][t >> 6] = bl; s_bt[1][t >> 6] = al; }
    __syncthreads();
    if (t == 0) {
      double b2 = 0.0, a2 = 0.0;
      for (int i = 0; i < WQ_FT / 64; ++i) { b2 += s_bt[0][i]; a2 += s_bt[1][i]; }
      s_below = b2;
      s_total = a2;
    }
    __syncthreads();
  }
  const double below = s_below, total = s_total;
  // rank sort by (key, index) -- the stable order of the reference's sort:
  // each listed point counts the points before it (LDS broadcast reads, no
  // dependent stages; up to WQ_REFINE points the count is split over
  // WQ_FT / WQ_REFINE groups of the list and summed by integer LDS atomics),
  // then the list is rewritten in rank order.  The ranks are exact integers,
  // so the order -- and the fixed-order prefix below -- never depends on the
  // list's (atomic) fill order.
  {
    int* srank = L.srank;
    const int G = m <= WQ_REFINE ? WQ_FT / WQ_REFINE : 1;
    const int per_g = WQ_FT / G, g = t / per_g, e0 = t % per_g;
    const int jn = (m + G - 1) / G, jlo = g * jn, jhi = min(m, jlo + jn);
    for (int e = t; e < m; e += WQ_FT) srank[e] = 0;
    __syncthreads();
    for (int e = e0; e < m; e += per_g) {
      const u64 ke = skey[e];
      const int ie = sidx[e];
      int r = 0;
      for (int j = jlo; j < jhi; ++j) r += kless(skey[j], sidx[j], ke, ie) ? 1 : 0;
      if (G == 1) srank[e] = r;
      else atomicAdd(&srank[e], r);
    }
    __syncthreads();
    constexpr int PT = WQ_CAP / WQ_FT;
    u64 k[PT];
    int ix[PT], rk[PT];
    double wv[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int e = t + q * WQ_FT;
      if (e < m) { k[q] = skey[e]; ix[q] = sidx[e]; wv[q] = sw[e]; rk[q] = srank[e]; }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      if (t + q * WQ_FT < m) {
        skey[rk[q]] = k[q];
        sidx[rk[q]] = ix[q];
        sw[rk[q]] = wv[q];
      }
    }
  }
  __syncthreads();
  // cumulative weights: the fp64 sum below + an inclusive prefix in a fixed
  // order (each thread a run of consecutive elements, then the thread sums)
  {
    const int per = (m + WQ_FT - 1) / WQ_FT;
    const int i0 = t * per;
    double sum = 0.0;
    for (int k = 0; k < per && i0 + k < m; ++k) sum += sw[i0 + k];
    const int lane = t & 63, wv = t >> 6;
    double inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double a = __shfl_up(inc, o, 64);
      if (lane >= o) inc += a;
    }
    if (lane == 63) dsh[wv] = inc;
    __syncthreads();
    double run = below + (inc - sum);
    for (int i = 0; i < wv; ++i) run += dsh[i];
    for (int k = 0; k < per && i0 + k < m; ++k) {
      run += sw[i0 + k];
      kn[i0 + k] = Knot{(run - 0.5 * sw[i0 + k]) / total, qval(skey[i0 + k])};
    }
  }
  __syncthreads();
  if (t == 0) {
    bool ok = m > 0;
    double r = NAN;
    if (ok) r = interp_rules(alpha, kn[0], kn[m - 1], D.below == 0, D.below + m == N, kn, m, ok);
    *q = ok ? r : NAN;
  }
}


// ---- 4./5. gather the segment + the fp64 sums, final in the last block -----
__global__ __launch_bounds__(WQ_T) void wq_gather_final_kernel(
    const double* __restrict__ x, const double* __restrict__ w, int64_t N, int64_t chunk,
    double alpha, WqCtl* __restrict__ ctl, const WqDesc* __restrict__ desc,
    u64* __restrict__ gkey, int* __restrict__ gidx, double* __restrict__ gw,
    double* __restrict__ psum, double* __restrict__ q) {
  __shared__ double sh[WQ_T / 64];
  // the level-1 segment when it fits, else level 2's
  const WqDesc D = desc[0].ok ? desc[0] : desc[1];
  {
    const int64_t b0 = (int64_t)blockIdx.x * chunk;
    const int64_t b1 = b0 + chunk < N ? b0 + chunk : N;
    double below = 0.0, all = 0.0;
    for (int64_t i0 = b0 + threadIdx.x; i0 < b1; i0 += WQ_U * WQ_T) {
      double xv[WQ_U], wv[WQ_U];
#pragma unroll
      for (int u = 0; u < WQ_U; ++u) {
        const int64_t i = i0 + (int64_t)u * WQ_T;
        xv[u] = i < b1 ? x[i] : 0.0;
        wv[u] = i < b1 ? w[i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < WQ_U; ++u) {
      const int64_t i = i0 + (int64_t)u * WQ_T;
      if (i >= b1) continue;
      const u64 k = qkey(xv[u]);
      const double wi = wval(wv[u]);
      all += wi;
      if (k < D.lo) below += wi;
      else if (D.ok && k <= D.hi) {
        const unsigned int pos = atomicAdd(&ctl->list_n, 1u);
        if (pos < (unsigned int)WQ_CAP) {
          st_agent(&gkey[pos], k);
          st_agent(&gidx[pos], (int)i);
          st_agent(&gw[pos], wi);
        }
      }
      }
    }
    auto add = [](double a, double b) { return a + b; };
    below = block_reduce(below, sh, add);
    all = block_reduce(all, sh, add);
    if (threadIdx.x == 0) {
      st_agent(&psum[2 * blockIdx.x], below);
      st_agent(&psum[2 * blockIdx.x + 1], all);
    }
  }
  if (!wq_last_block(&ctl->done[2])) return;
  wq_reset(ctl);
  __shared__ WqFinalLds L;
  wq_final(D, N, alpha, (int)gridDim.x, psum, gkey, gidx, gw, q, L);
}

// ---- one launch: every stage in one resident grid ---------------------------
// Up to WQ_ONE_MAX points (c3's 1e6) each thread holds its WQ_U points in
// registers from the first read: the range, both histogram levels and the
// gather run on them, the stages separated by grid-wide hand-offs instead of
// kernel boundaries (the grid -- at most WQ_MAXB blocks, one per CU -- is
// checked against the device's resident capacity before launch, so every
// block runs at once).  A hand-off: every block bumps an arrival counter;
// the block that brings it to the grid size runs the stage's tail alone (the
// level's pick), publishes its result with agent-scope stores and raises a
// flag; the others wait on the flag.  Level 1 bins on 256 bins (not 2048 as
// the four-launch path): the flush of each block's LDS histogram into the
// global one is one integer atomic per non-empty bin and block, and with
// ~250 blocks those atomics on a few KB dominated the level (measured:
// 28 us at 2048 bins, profiles/r06_quantile_onepass.log); level 2 then
// resolves the wider segment (4096 bins over its few thousand points).
// A third level (4096 bins) resolves spans whose points crowd into a tiny
// part of the key range.
// Deterministic (integer histograms, fixed-order fp64 sums); the segment
// differs from the four-launch path's, so the fp64 sum below it -- and q --
// may differ from that path's in the last bits (both within the 1e-12 bar).
constexpr int64_t WQ_ONE_MAX = (int64_t)WQ_MAXB * WQ_U * WQ_T;
constexpr int WQ_BITS1_ONE = 8;
constexpr int WQ_ONE_LEVELS = 3;   // 256 x 4096 x 4096 bins over the key span at most
constexpr unsigned int WQ_SPIN_MAX = 1u << 18;   // 10-300 ms of polls: a hang guard only

union WqOneLds {
  struct { unsigned int cnt[WQ_NB]; u64 ws[WQ_NB]; } h;
  WqFinalLds f;
};

// Hand-off counters and flags (a zeroed workspace region, one 256-B line
// each so that no two share a memory channel's queue): blocks arrive on the
// counter of their group (block index mod 8), the last of a group on the top
// counter, and the last there is the last block; it raises one flag per
// group, which the group's blocks poll.  One counter for every block cost
// ~12 us per hand-off at 245 blocks (the arrivals and polls on one address
// are served one after another), the groups ~3 us.
// The key range and the weight maximum go the same way: one (~key min, key
// max, weight max) slot per group, read by every block after hand-off 1 (the
// same three addresses for every block cost ~5 us more).
constexpr int WQ_HS_STRIDE = 64;                 // u32 per line
constexpr int WQ_HS_TOP = 8, WQ_HS_FLAG = 9;     // line indices
constexpr int WQ_HS_RANGE = 17;                  // 8 lines: u64 ~kmin, kmax, wmax
constexpr int WQ_HS_LINES = WQ_HS_RANGE + 8;

// Arrival k (1, 2, ...): true in the block that arrives last.  Everything a
// stage hands on is written by agent-scope atomics and stores (performed at
// the agent's coherence point, past the XCD's L2), complete (s_waitcnt)
// before the block arrives, and read after the wait with agent-scope loads,
// which the workgroup barrier after the wait keeps behind it.  So the
// counters and flags need no release / acquire of their own: with them
// (acq_rel arrivals, release flags, acquire polls and fence) a call takes
// 0.174 instead of 0.044 ms at 1e6 -- every agent-scope release writes back
// the XCD's L2 and every acquire invalidates it
// (profiles/r06_quantile_release_ab.log).
__device__ bool wq_arrive(unsigned int* hs, unsigned int k) {
  __shared__ int s_last;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int g = blockIdx.x & 7u, ng = (gridDim.x - g + 7u) >> 3;
    const unsigned int groups = gridDim.x < 8u ? gridDim.x : 8u;
    int last = 0;
    if (__hip_atomic_fetch_add(&hs[g * WQ_HS_STRIDE], 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) == k * ng - 1u)
      last = __hip_atomic_fetch_add(&hs[WQ_HS_TOP * WQ_HS_STRIDE], 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) == k * groups - 1u;
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}
// the last block's result is out: raise every group's flag to k
__device__ void wq_release(unsigned int* hs, unsigned int k) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x < (gridDim.x < 8u ? gridDim.x : 8u))
    st_agent(&hs[(WQ_HS_FLAG + threadIdx.x) * WQ_HS_STRIDE], k);
}
// wait for flag k.  A wait that outlasts WQ_SPIN_MAX polls (the grid was not
// resident after all) returns false: the caller leaves q NaN, the host's
// exact path then answers, and the control block stays poisoned for the
// calls after.
__device__ bool wq_wait(unsigned int* hs, unsigned int k) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    const unsigned int* f = &hs[(WQ_HS_FLAG + (blockIdx.x & 7u)) * WQ_HS_STRIDE];
    int ok = 1;
    for (unsigned int it = 0; ld_agent(f) < k; ++it) {
      if (it >= WQ_SPIN_MAX) { ok = 0; break; }
      __builtin_amdgcn_s_sleep(2);
    }
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

__device__ __forceinline__ void wq_poison(WqCtl* ctl, double* q) {
  if (threadIdx.x == 0) {
    st_agent(&ctl->pad, 1u);
    st_agent(q, (double)NAN);
  }
}

__device__ __forceinline__ void st_desc(WqDesc* g, const WqDesc& d) {
  st_agent(&g->lo, d.lo);
  st_agent(&g->hi, d.hi);
  st_agent(&g->base_w, d.base_w);
  st_agent(&g->count, d.count);
  st_agent(&g->below, d.below);
  st_agent(&g->ok, d.ok);
}
__device__ __forceinline__ WqDesc ld_desc(const WqDesc* g) {
  WqDesc d;
  d.lo = ld_agent(&g->lo);
  d.hi = ld_agent(&g->hi);
  d.base_w = ld_agent(&g->base_w);
  d.count = ld_agent(&g->count);
  d.below = ld_agent(&g->below);
  d.ok = ld_agent(&g->ok);
  d.done = 0;
  return d;
}

__global__ __launch_bounds__(WQ_T) void wq_onepass_kernel(
    const double* __restrict__ x, const double* __restrict__ w, int64_t N, int64_t chunk,
    double alpha, WqCtl* __restrict__ ctl, unsigned int* __restrict__ hs,
    WqDesc* __restrict__ gdesc, unsigned int* __restrict__ ghc, u64* __restrict__ ghw,
    u64* __restrict__ gkey,
    int* __restrict__ gidx, double* __restrict__ gw, double* __restrict__ psum,
    double* __restrict__ q) {
  __shared__ WqOneLds L;
  __shared__ double shd[WQ_T / 64];
  __shared__ WqDesc sD;
  __shared__ u64 s_tot;
  if (ld_agent(&ctl->pad)) {   // an earlier call's wait timed out
    if (blockIdx.x == 0 && threadIdx.x == 0) *q = NAN;
    return;
  }
  const int t = threadIdx.x;
  // every level's global histogram to zero (added into after hand-off 1)
  for (int e = blockIdx.x * WQ_T + t; e < WQ_ONE_LEVELS * WQ_NB; e += gridDim.x * WQ_T) {
    st_agent(&ghc[e], 0u);
    st_agent(&ghw[e], 0ull);
  }
  const int64_t b0 = (int64_t)blockIdx.x * chunk;
  const int64_t b1 = b0 + chunk < N ? b0 + chunk : N;
  u64 kv[WQ_U];
  double wv[WQ_U];
  bool in[WQ_U];
  u64 mn = ~0ull, mx = 0ull, wm = 0ull;
  double all = 0.0;
#pragma unroll
  for (int u = 0; u < WQ_U; ++u) {
    const int64_t i = b0 + t + (int64_t)u * WQ_T;
    in[u] = i < b1;
    kv[u] = in[u] ? qkey(x[i]) : ~0ull;
    wv[u] = in[u] ? wval(w[i]) : 0.0;
  }
#pragma unroll
  for (int u = 0; u < WQ_U; ++u) {
    if (!in[u]) continue;
    mn = kv[u] < mn ? kv[u] : mn;
    mx = kv[u] > mx ? kv[u] : mx;
    const u64 wb = (u64)__double_as_longlong(wv[u]);   // >= 0: bits order like values
    wm = wb > wm ? wb : wm;
    all += wv[u];
  }
  auto add = [](double a, double b) { return a + b; };
  {
    // the four block reductions in one pass (~kmin, kmax, wmax by max; the
    // weight sum by the same fixed tree as block_reduce)
    u64 nmn = ~mn;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const u64 a = __shfl_xor(nmn, o, 64), b = __shfl_xor(mx, o, 64),
                c = __shfl_xor(wm, o, 64);
      nmn = a > nmn ? a : nmn;
      mx = b > mx ? b : mx;
      wm = c > wm ? c : wm;
      all += __shfl_xor(all, o, 64);
    }
    __shared__ u64 s_r[3][WQ_T / 64];
    if ((t & 63) == 0) {
      s_r[0][t >> 6] = nmn; s_r[1][t >> 6] = mx; s_r[2][t >> 6] = wm; shd[t >> 6] = all;
    }
    __syncthreads();
    if (t == 0) {
      double a = shd[0];
      for (int i = 1; i < WQ_T / 64; ++i) {
        nmn = s_r[0][i] > nmn ? s_r[0][i] : nmn;
        mx = s_r[1][i] > mx ? s_r[1][i] : mx;
        wm = s_r[2][i] > wm ? s_r[2][i] : wm;
        a += shd[i];
      }
      unsigned long long* r = reinterpret_cast<unsigned long long*>(
          &hs[(WQ_HS_RANGE + (blockIdx.x & 7u)) * WQ_HS_STRIDE]);
      atomicMax(&r[0], (unsigned long long)nmn);
      atomicMax(&r[1], (unsigned long long)mx);
      atomicMax(&r[2], (unsigned long long)wm);
      st_agent(&psum[2 * blockIdx.x + 1], a);
    }
  }
  if (wq_arrive(hs, 1)) wq_release(hs, 1);
  if (!wq_wait(hs, 1)) { wq_poison(ctl, q); return; }

  __shared__ Range s_range;
  if (t < 64) {   // the groups' slots (zero = the identity of the max)
    const unsigned int groups = gridDim.x < 8u ? gridDim.x : 8u;
    const u64* r = reinterpret_cast<const u64*>(&hs[(WQ_HS_RANGE + (t & 7)) * WQ_HS_STRIDE]);
    u64 a = 0ull, b = 0ull, c = 0ull;
    if (t < (int)groups) { a = ld_agent(&r[0]); b = ld_agent(&r[1]); c = ld_agent(&r[2]); }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) {
      const u64 a2 = __shfl_xor(a, o, 64), b2 = __shfl_xor(b, o, 64), c2 = __shfl_xor(c, o, 64);
      a = a2 > a ? a2 : a;
      b = b2 > b ? b2 : b;
      c = c2 > c ? c2 : c;
    }
    if (t == 0) {
      const double wmax = __longlong_as_double((long long)c);
      s_range = Range{~a, b, wmax > 0.0 ? ldexp(1.0, 62 - lg_ceil(N)) / wmax : 0.0};
    }
  }
  __syncthreads();
  const Range R = s_range;
  // one histogram level over [lo, hi] into the level's global bins
  auto level = [&](auto bits_c, u64 lo, u64 hi, unsigned int* gc, u64* gws) {
    constexpr int BITS = decltype(bits_c)::value, NB = 1 << BITS;
    for (int b = t; b < NB; b += WQ_T) { L.h.cnt[b] = 0u; L.h.ws[b] = 0ull; }
    const int sh = span_shift<BITS>(lo, hi);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < WQ_U; ++u) {
      if (!in[u] || kv[u] < lo || kv[u] > hi) continue;
      const int bin = (int)((kv[u] - lo) >> sh);
      atomicAdd(&L.h.cnt[bin], 1u);
      atomicAdd(&L.h.ws[bin], wfix(wv[u], R.S));
    }
    __syncthreads();
    for (int b = t; b < NB; b += WQ_T) {
      if (L.h.cnt[b]) {
        atomicAdd(&gc[b], L.h.cnt[b]);
        atomicAdd(reinterpret_cast<unsigned long long*>(&gws[b]),
                  (unsigned long long)L.h.ws[b]);
      }
    }
  };
  level(std::integral_constant<int, WQ_BITS1_ONE>{}, R.kmin, R.kmax, ghc, ghw);
  unsigned int k = 2;
  if (wq_arrive(hs, k)) {
    if (t < 64)
      wq_pick_wave<WQ_BITS1_ONE>(N, alpha, ghc, ghw, R.kmin, R.kmax, 0ull, 0, true, 0.0,
                                 &s_tot, &sD);
    __syncthreads();
    if (t == 0) {
      st_desc(&gdesc[0], sD);
      st_agent(&ctl->tot, s_tot);
    }
    wq_release(hs, k);
  }
  if (!wq_wait(hs, k)) { wq_poison(ctl, q); return; }
  WqDesc D = ld_desc(&gdesc[0]);
  // levels 2.. on 4096 bins while the segment holds more than WQ_CAP points
  // (the same decision in every block)
  for (int lev = 1; !D.ok && lev < WQ_ONE_LEVELS; ++lev) {
    level(std::integral_constant<int, WQ_BITS>{}, D.lo, D.hi, ghc + lev * WQ_NB,
          ghw + lev * WQ_NB);
    ++k;
    if (wq_arrive(hs, k)) {
      wq_pick_block<WQ_BITS>(N, alpha, ghc + lev * WQ_NB, ghw + lev * WQ_NB, D.lo, D.hi,
                             D.base_w, D.below, false,
                             __longlong_as_double((long long)ld_agent(&ctl->tot)), nullptr, &sD);
      __syncthreads();
      if (t == 0) st_desc(&gdesc[lev & 1], sD);
      wq_release(hs, k);
    }
    if (!wq_wait(hs, k)) { wq_poison(ctl, q); return; }
    D = ld_desc(&gdesc[lev & 1]);
  }
  // gather: the segment's points into the list, the fp64 sum below it
  double below = 0.0;
#pragma unroll
  for (int u = 0; u < WQ_U; ++u) {
    if (!in[u]) continue;
    if (kv[u] < D.lo) below += wv[u];
    else if (D.ok && kv[u] <= D.hi) {
      const unsigned int pos = atomicAdd(&ctl->list_n, 1u);
      if (pos < (unsigned int)WQ_CAP) {
        st_agent(&gkey[pos], kv[u]);
        st_agent(&gidx[pos], (int)(b0 + t + (int64_t)u * WQ_T));
        st_agent(&gw[pos], wv[u]);
      }
    }
  }
  below = block_reduce(below, shd, add);
  if (t == 0) st_agent(&psum[2 * blockIdx.x], below);
  if (!wq_arrive(hs, k + 1)) return;
  // every block is past its last wait: the counters and flags back to zero
  wq_reset(ctl);
  if (t < WQ_HS_LINES * 8) st_agent(&hs[(t >> 3) * WQ_HS_STRIDE + (t & 7)], 0u);
  wq_final(D, N, alpha, (int)gridDim.x, psum, gkey, gidx, gw, q, L.f);
}

int wq_blocks(int64_t N) {
  const int64_t b = ceil_div(N, 4096);
  return (int)(b < 1 ? 1 : (b > WQ_MAXB ? WQ_MAXB : b));
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" size_t abc_weighted_quantile_workspace(int64_t N) {
  const int nb = wq_blocks(N > 0 ? N : 1);
  size_t off = 0;
  size_only<WqCtl>(off, 1);
  size_only<unsigned int>(off, (size_t)WQ_HS_LINES * WQ_HS_STRIDE);
  size_only<unsigned int>(off, (size_t)WQ_ONE_LEVELS * WQ_NB);
  size_only<u64>(off, (size_t)WQ_ONE_LEVELS * WQ_NB);
  size_only<WqDesc>(off, 2);
  size_only<u64>(off, WQ_CAP);
  size_only<int>(off, WQ_CAP);
  size_only<double>(off, WQ_CAP);
  size_only<double>(off, (size_t)2 * nb);
  return off + 256;
}

// Launches: range, level-1 histogram (its
// last block picks), level-2 histogram (exits at once when level 1 fits; its
// last block picks), gather (its last block sorts the list and
// interpolates).  No single-block kernel.
extern "C" int abc_weighted_quantile(const double* points, const double* w, int64_t N,
                                     double alpha, double* q, void* ws, size_t ws_bytes,
                                     void* stream) {
  ABC_CHECK_ARG(N >= 1 && N < (1ll << 31), "quantile: bad N");
  ABC_CHECK_ARG(points && w && q && ws, "quantile: null pointer");
  if (ws_bytes < abc_weighted_quantile_workspace(N))
    return set_error(ABC_ERR_WORKSPACE, "quantile: workspace too small");
  hipStream_t s = as_stream(stream);
  const int nb = wq_blocks(N);
  const int64_t chunk = ceil_div(N, nb);
  Carver cv(ws, ws_bytes);
  WqCtl* ctl = cv.take<WqCtl>(1);
  unsigned int* hs = cv.take<unsigned int>((size_t)WQ_HS_LINES * WQ_HS_STRIDE);
  // levels 1 | 2 (| 3: the one-launch path)
  unsigned int* ghc = cv.take<unsigned int>((size_t)WQ_ONE_LEVELS * WQ_NB);
  u64* ghw = cv.take<u64>((size_t)WQ_ONE_LEVELS * WQ_NB);
  WqDesc* desc = cv.take<WqDesc>(2);
  u64* lkey = cv.take<u64>(WQ_CAP);
  int* lidx = cv.take<int>(WQ_CAP);
  double* lw = cv.take<double>(WQ_CAP);
  double* psum = cv.take<double>((size_t)2 * nb);
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "quantile: carve");
  if (N <= WQ_ONE_MAX && nb <= resident_blocks(wq_onepass_kernel, WQ_T, 0)) {
    hipLaunchKernelGGL(wq_onepass_kernel, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk,
                       alpha, ctl, hs, desc, ghc, ghw, lkey, lidx, lw, psum, q);
    ABC_LAUNCHED();
    return ABC_OK;
  }
  hipLaunchKernelGGL(wq_range_kernel, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk, ctl,
                     ghc, ghw);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_hist_kernel<1>, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk,
                     alpha, ctl, desc, ghc, ghw);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_hist_kernel<2>, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk,
                     alpha, ctl, desc, ghc + WQ_NB, ghw + WQ_NB);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_gather_final_kernel, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk,
                     alpha, ctl, (const WqDesc*)desc, lkey, lidx, lw, psum, q);
  ABC_LAUNCHED();
  return ABC_OK;
}
