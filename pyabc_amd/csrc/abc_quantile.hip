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
// units.  Launches:
//   1. range: per-block min / max key and max weight;
//   2. hist (level 1): 4096 bins linear in the key span, counts and
//      fixed-point weight sums per bin (LDS atomics, integer);
//   3. pick (level 1, one block): the bins that can hold the knots j, j + 1
//      (every bin whose cumulative weight interval, widened by the
//      fixed-point error, reaches alpha * total, plus one bin on each side
//      that certainly lies below / above it) -> a key segment [lo, hi];
//   4./5. hist + pick (level 2) inside that segment when it holds more than
//      WQ_CAP points (both exit at once otherwise);
//   6. gather: the segment's points (key, index, w) into a list, and the
//      fp64 sums of the weights below the segment and of all weights (fixed
//      per-thread order + fixed tree: deterministic);
//   7. final (one block): the list sorted by (key, index) in LDS, cumulative
//      weights from the sum below, xp and np.interp's rules
//      (quantile_pick semantics: clamps, exact knot hit, NaN fallbacks).
// A segment that still holds more than WQ_CAP points after level 2 (ties by
// the thousand at the knots, e.g. discrete distances) is not decided here:
// *q = NaN, and the host (gpu.weighted_quantile's readers) reruns the exact
// sort-based abc_weighted_quantile_sorted on the same inputs.
#include "abc_common.h"

namespace abc {
namespace {

constexpr int WQ_T = 1024;
constexpr int WQ_BITS = 12, WQ_NB = 1 << WQ_BITS;
constexpr int WQ_CAP = 2048;
constexpr int WQ_MAXB = 256;
constexpr int WQ_FT = 1024;  // threads of the final (single-block) kernel (256: 54 vs 35 us)
static_assert(WQ_MAXB <= WQ_FT, "wq_final_kernel sums one gather block per thread");

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

struct WqPart { u64 kmin, kmax, wmax; };
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
__device__ __forceinline__ Range wq_global_range(const WqPart* part, int nblk, int64_t N) {
  Range r{~0ull, 0ull, 0.0};
  u64 wm = 0ull;
  for (int b = 0; b < nblk; ++b) {
    r.kmin = part[b].kmin < r.kmin ? part[b].kmin : r.kmin;
    r.kmax = part[b].kmax > r.kmax ? part[b].kmax : r.kmax;
    wm = part[b].wmax > wm ? part[b].wmax : wm;
  }
  const double wmax = __longlong_as_double((long long)wm);
  r.S = wmax > 0.0 ? ldexp(1.0, 62 - lg_ceil(N)) / wmax : 0.0;
  return r;
}

__device__ __forceinline__ int span_shift(u64 lo, u64 hi) {
  const u64 span = hi - lo;
  const int L = span ? 64 - __clzll(span) : 0;
  return L > WQ_BITS ? L - WQ_BITS : 0;
}

// ---- 1. range ----------------------------------------------------------------
__global__ __launch_bounds__(WQ_T) void wq_range_kernel(const double* __restrict__ x,
                                                        const double* __restrict__ w,
                                                        int64_t N, int64_t chunk,
                                                        WqPart* __restrict__ part,
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
  for (int64_t i = b0 + threadIdx.x; i < b1; i += WQ_T) {
    const u64 k = qkey(x[i]);
    mn = k < mn ? k : mn;
    mx = k > mx ? k : mx;
    const u64 wb = (u64)__double_as_longlong(wval(w[i]));  // >= 0: bits order like values
    wm = wb > wm ? wb : wm;
  }
  auto umin = [](u64 a, u64 b) { return a < b ? a : b; };
  auto umax = [](u64 a, u64 b) { return a > b ? a : b; };
  mn = block_reduce(mn, sh, umin);
  mx = block_reduce(mx, sh, umax);
  wm = block_reduce(wm, sh, umax);
  // one global range: integer min / max atomics (order-free), initialised
  // by the launcher's memsets
  if (threadIdx.x == 0) {
    atomicMin(reinterpret_cast<unsigned long long*>(&part->kmin), (unsigned long long)mn);
    atomicMax(reinterpret_cast<unsigned long long*>(&part->kmax), (unsigned long long)mx);
    atomicMax(reinterpret_cast<unsigned long long*>(&part->wmax), (unsigned long long)wm);
  }
}

// ---- 2. histogram of one level ----------------------------------------------
// level 1: the whole key range; level 2: the level-1 segment (exits when the
// level-1 segment fits)
__global__ __launch_bounds__(WQ_T) void wq_hist_kernel(
    const double* __restrict__ x, const double* __restrict__ w, int64_t N, int64_t chunk,
    const WqPart* __restrict__ part, int nblk, const WqDesc* __restrict__ prev,
    unsigned int* __restrict__ ghc, u64* __restrict__ ghw) {
  if (prev && prev->ok) return;
  __shared__ unsigned int cnt[WQ_NB];
  __shared__ u64 ws[WQ_NB];
  for (int b = threadIdx.x; b < WQ_NB; b += WQ_T) { cnt[b] = 0u; ws[b] = 0ull; }
  const Range R = wq_global_range(part, nblk, N);
  const u64 lo = prev ? prev->lo : R.kmin, hi = prev ? prev->hi : R.kmax;
  const int sh = span_shift(lo, hi);
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * chunk;
  const int64_t b1 = b0 + chunk < N ? b0 + chunk : N;
  for (int64_t i = b0 + threadIdx.x; i < b1; i += WQ_T) {
    const u64 k = qkey(x[i]);
    if (k < lo || k > hi) continue;
    const int bin = (int)((k - lo) >> sh);
    atomicAdd(&cnt[bin], 1u);
    atomicAdd(&ws[bin], wfix(w[i], R.S));
  }
  __syncthreads();
  // into the level's global histogram: integer atomics, so the totals do
  // not depend on the blocks' order
  for (int b = threadIdx.x; b < WQ_NB; b += WQ_T) {
    if (cnt[b]) {
      atomicAdd(&ghc[b], cnt[b]);
      atomicAdd(reinterpret_cast<unsigned long long*>(&ghw[b]), (unsigned long long)ws[b]);
    }
  }
}

// ---- 3. pick the segment of one level ------------------------------------------
// Per-bin totals (fixed order over blocks; integers), exclusive prefixes, and
// the segment: from the last non-empty bin whose whole weight interval lies
// certainly below the target to the first whose interval lies certainly
// above it (the knots j and j + 1 lie between them, inclusive).  Shared by
// the multi-block path (cnt / wsum summed from the block histograms) and the
// final block's slow refinement.
struct Pick { int b1, b2; };
__device__ void wq_pick_bins(const unsigned int* cnt, const u64* wsum, u64* pre_w,
                             long long* pre_c, u64 base_w, double target, double margin,
                             Pick& pk, u64* s_sh) {
  // exclusive prefixes: 4 bins per thread, then a block scan of the thread sums
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  constexpr int PER = WQ_NB / WQ_T;
  u64 sw = 0ull;
  long long sc = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) { sw += wsum[t * PER + i]; sc += cnt[t * PER + i]; }
  u64 iw = sw;
  long long ic = sc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u64 a = __shfl_up(iw, o, 64);
    const long long c = __shfl_up(ic, o, 64);
    if (lane >= o) { iw += a; ic += c; }
  }
  __shared__ long long s_c[WQ_T / 64];
  if (lane == 63) { s_sh[wv] = iw; s_c[wv] = ic; }
  __syncthreads();
  u64 ow = base_w + iw - sw;
  long long oc = ic - sc;
  for (int i = 0; i < wv; ++i) { ow += s_sh[i]; oc += s_c[i]; }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    pre_w[t * PER + i] = ow;
    pre_c[t * PER + i] = oc;
    ow += wsum[t * PER + i];
    oc += cnt[t * PER + i];
  }
  __syncthreads();
  // b1 = last non-empty bin with pre + W + margin <= target (else the first
  // non-empty bin); b2 = first non-empty bin with pre - margin > target
  // (else the last non-empty bin)
  __shared__ int s_b1, s_b2, s_first, s_last;
  if (t == 0) { s_b1 = -1; s_b2 = WQ_NB; s_first = WQ_NB; s_last = -1; }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int b = t * PER + i;
    if (cnt[b] == 0u) continue;
    atomicMin(&s_first, b);
    atomicMax(&s_last, b);
    if ((double)(pre_w[b] + wsum[b]) + margin <= target) atomicMax(&s_b1, b);
    if ((double)pre_w[b] - margin > target) atomicMin(&s_b2, b);
  }
  __syncthreads();
  pk.b1 = s_b1 >= 0 ? s_b1 : s_first;
  pk.b2 = s_b2 < WQ_NB ? s_b2 : s_last;
  if (pk.b2 < pk.b1) pk.b2 = pk.b1;
  __syncthreads();
}

__device__ __forceinline__ void seg_keys(u64 lo, u64 hi, int sh, int b1, int b2, u64& slo,
                                         u64& shi) {
  slo = lo + ((u64)b1 << sh);
  const u64 off = ((u64)b2 << sh) + ((1ull << sh) - 1ull);
  shi = off >= hi - lo ? hi : lo + off;
}

__global__ __launch_bounds__(WQ_T) void wq_pick_kernel(
    int64_t N, double alpha, const WqPart* __restrict__ part, int nblk,
    const unsigned int* __restrict__ ghc, const u64* __restrict__ ghw, int nhb,
    const WqDesc* __restrict__ prev, WqDesc* __restrict__ out, unsigned int* __restrict__ list_n) {
  (void)nhb;   // one global histogram per level (integer atomics in wq_hist_kernel)
  if (prev && prev->ok) {
    if (threadIdx.x == 0) *out = *prev;
    return;
  }
  __shared__ unsigned int cnt[WQ_NB];
  __shared__ u64 wsum[WQ_NB], pre_w[WQ_NB];
  __shared__ long long pre_c[WQ_NB];
  __shared__ u64 s_sh[WQ_T / 64];
  const Range R = wq_global_range(part, nblk, N);
  u64 tw = 0ull;
  for (int b = threadIdx.x; b < WQ_NB; b += WQ_T) {
    const unsigned int c = ghc[b];
    const u64 sm = ghw[b];
    cnt[b] = c;
    wsum[b] = sm;
    tw += sm;
  }
  auto add = [](u64 a, u64 b) { return a + b; };
  tw = block_reduce(tw, s_sh, add);
  // the whole input's fixed-point total: summed at level 1 and kept next to
  // the list counter for level 2 and the final block
  long long* tot_slot = reinterpret_cast<long long*>(list_n + 2);
  const double tot_fx = prev ? __longlong_as_double(*tot_slot) : (double)tw;
  const u64 lo = prev ? prev->lo : R.kmin, hi = prev ? prev->hi : R.kmax;
  const u64 base_w = prev ? prev->base_w : 0ull;
  const long long base_c = prev ? prev->below : 0;
  const double target = alpha * tot_fx;
  const double margin = (double)N + ldexp(tot_fx, -48) + 4096.0;
  Pick pk;
  wq_pick_bins(cnt, wsum, pre_w, pre_c, base_w, target, margin, pk, s_sh);
  if (threadIdx.x == 0) {
    WqDesc d;
    seg_keys(lo, hi, span_shift(lo, hi), pk.b1, pk.b2, d.lo, d.hi);
    d.base_w = pre_w[pk.b1];
    d.below = base_c + pre_c[pk.b1];
    long long c = 0;
    for (int b = pk.b1; b <= pk.b2; ++b) c += cnt[b];
    d.count = c;
    d.ok = c <= WQ_CAP ? 1 : 0;
    d.done = 0;
    *out = d;
    if (!prev) {
      list_n[0] = 0u;
      *tot_slot = __double_as_longlong((double)tw);
    }
  }
}

// ---- 6. gather the segment + the fp64 sums ----------------------------------
__global__ __launch_bounds__(WQ_T) void wq_gather_kernel(
    const double* __restrict__ x, const double* __restrict__ w, int64_t N, int64_t chunk,
    const WqDesc* __restrict__ desc, u64* __restrict__ lkey, int* __restrict__ lidx,
    double* __restrict__ lw, unsigned int* __restrict__ list_n, double* __restrict__ psum) {
  __shared__ double sh[WQ_T / 64];
  const WqDesc D = *desc;
  const int64_t b0 = (int64_t)blockIdx.x * chunk;
  const int64_t b1 = b0 + chunk < N ? b0 + chunk : N;
  double below = 0.0, all = 0.0;
  for (int64_t i = b0 + threadIdx.x; i < b1; i += WQ_T) {
    const u64 k = qkey(x[i]);
    const double wi = wval(w[i]);
    all += wi;
    if (k < D.lo) below += wi;
    else if (D.ok && k <= D.hi) {
      const unsigned int pos = atomicAdd(list_n, 1u);
      if (pos < (unsigned int)WQ_CAP) { lkey[pos] = k; lidx[pos] = (int)i; lw[pos] = wi; }
    }
  }
  auto add = [](double a, double b) { return a + b; };
  below = block_reduce(below, sh, add);
  all = block_reduce(all, sh, add);
  if (threadIdx.x == 0) { psum[2 * blockIdx.x] = below; psum[2 * blockIdx.x + 1] = all; }
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

__global__ __launch_bounds__(WQ_FT) void wq_final_kernel(
    int64_t N, double alpha, const WqDesc* __restrict__ desc,
    const u64* __restrict__ gkey, const int* __restrict__ gidx, const double* __restrict__ gw,
    const double* __restrict__ psum, int nsum, double* __restrict__ q) {
  __shared__ u64 skey[WQ_CAP];
  __shared__ int sidx[WQ_CAP];
  __shared__ double sw[WQ_CAP];
  __shared__ Knot kn[WQ_CAP];
  __shared__ double dsh[WQ_FT / 64];
  const int t = threadIdx.x;
  const WqDesc D = *desc;
  if (!D.ok) {   // the knots sit in more than WQ_CAP points (ties): not decided
    if (t == 0) *q = NAN;
    return;
  }
  // the gather blocks' fp64 sums: a fixed tree (lanes, then waves in order)
  __shared__ double s_bt[2][WQ_FT / 64];
  __shared__ double s_below, s_total;
  {
    double bl = t < nsum ? psum[2 * t] : 0.0, al = t < nsum ? psum[2 * t + 1] : 0.0;
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
  const int m = (int)D.count;
  int M = 1;
  while (M < m) M <<= 1;
  for (int i = t; i < M; i += WQ_FT) {
    const bool in = i < m;
    skey[i] = in ? gkey[i] : ~0ull;
    sidx[i] = in ? gidx[i] : 0x7FFFFFFF;
    sw[i] = in ? gw[i] : 0.0;
  }
  __syncthreads();
  // bitonic sort by (key, index): the stable order of the reference's sort
  for (int size = 2; size <= M; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < M; i += WQ_FT) {
        const int jx = i ^ stride;
        if (jx > i) {
          const bool asc = (i & size) == 0;
          if (kless(skey[jx], sidx[jx], skey[i], sidx[i]) == asc) {
            const u64 a = skey[i]; skey[i] = skey[jx]; skey[jx] = a;
            const int b = sidx[i]; sidx[i] = sidx[jx]; sidx[jx] = b;
            const double c = sw[i]; sw[i] = sw[jx]; sw[jx] = c;
          }
        }
      }
      __syncthreads();
    }
  }
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
  size_only<WqPart>(off, 1);
  size_only<unsigned int>(off, (size_t)2 * WQ_NB);
  size_only<u64>(off, (size_t)2 * WQ_NB);
  size_only<WqDesc>(off, 2);
  size_only<u64>(off, WQ_CAP);
  size_only<int>(off, WQ_CAP);
  size_only<double>(off, WQ_CAP);
  size_only<unsigned int>(off, 4);
  size_only<double>(off, (size_t)2 * nb);
  return off + 256;
}

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
  WqPart* part = cv.take<WqPart>(1);
  unsigned int* ghc = cv.take<unsigned int>((size_t)2 * WQ_NB);   // level 1 | level 2
  u64* ghw = cv.take<u64>((size_t)2 * WQ_NB);
  WqDesc* desc = cv.take<WqDesc>(2);
  u64* lkey = cv.take<u64>(WQ_CAP);
  int* lidx = cv.take<int>(WQ_CAP);
  double* lw = cv.take<double>(WQ_CAP);
  unsigned int* list_n = cv.take<unsigned int>(4);   // [0]: count; [2..3]: total (fixed)
  double* psum = cv.take<double>((size_t)2 * nb);
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "quantile: carve");
  ABC_HIP(hipMemsetAsync(&part->kmin, 0xFF, sizeof(u64), s));
  ABC_HIP(hipMemsetAsync(&part->kmax, 0, 2 * sizeof(u64), s));
  hipLaunchKernelGGL(wq_range_kernel, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk, part,
                     ghc, ghw);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_hist_kernel, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk, part, 1,
                     (const WqDesc*)nullptr, ghc, ghw);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_pick_kernel, dim3(1), dim3(WQ_T), 0, s, N, alpha, part, 1, ghc, ghw, 1,
                     (const WqDesc*)nullptr, desc, list_n);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_hist_kernel, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk, part, 1,
                     (const WqDesc*)desc, ghc + WQ_NB, ghw + WQ_NB);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_pick_kernel, dim3(1), dim3(WQ_T), 0, s, N, alpha, part, 1,
                     ghc + WQ_NB, ghw + WQ_NB, 1, (const WqDesc*)desc, desc + 1, list_n);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_gather_kernel, dim3(nb), dim3(WQ_T), 0, s, points, w, N, chunk,
                     (const WqDesc*)(desc + 1), lkey, lidx, lw, list_n, psum);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wq_final_kernel, dim3(1), dim3(WQ_FT), 0, s, N, alpha,
                     (const WqDesc*)(desc + 1), lkey, lidx, lw, psum, nb, q);
  ABC_LAUNCHED();
  return ABC_OK;
}
