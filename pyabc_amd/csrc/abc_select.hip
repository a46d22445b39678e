// Per-column exact order statistics by radix select, for the
// AdaptivePNormDistance scale update with median_absolute_deviation.
//
// Reference: pyabc/distance/scale.py:38-47
//   median_absolute_deviation(data) = np.median(np.abs(data - np.median(data)))
// over the recorded summary statistics of one key (distance.py:263-307), i.e.
// per column of the recorded [R x S] matrix.  np.median: the middle order
// statistic for odd R, the mean (a + b) / 2 of the two middle ones for even R.
//
// Layout: the row-major [R x S] fp64 matrix is transposed once (LDS tiles)
// into column-major order-preserving u64 keys Kc[S][R].  One 1024-thread
// workgroup per column then selects the rank-k key with 12-bit MSD digits:
//   level 0: histogram of bits 63..52 over the column (LDS atomics), pick the
//            bin holding rank k;
//   level l: one pass over the surviving set that compacts the keys of the
//            picked bin into scratch (in place from level 2 on, chunk-wise
//            behind a barrier) and histograms their next digit.
// The surviving set shrinks by ~the bin count per level.  Long columns are
// first bracketed by a sorted sample (see BR_MARG): one streaming pass keeps
// the ~12% of keys around the wanted rank, so a select costs ~1 full read of
// the column instead of ~2.  For even R the (k+1)-th statistic is tracked along:
// while it falls in the same bin it survives with rank k; once it falls in
// the next non-empty bin it is the minimum of that bin, taken in the next
// pass (LDS 64-bit atomic min).  Results are exact and bitwise deterministic
// (the selection is order independent).
#include "abc_common.h"

namespace abc {
namespace {

constexpr int SEL_T = 1024;
constexpr int SEL_BITS = 12, SEL_BINS = 1 << SEL_BITS;
constexpr int TP = 64;  // transpose tile

__device__ __forceinline__ uint64_t f2key_s(double v) {
  if (v == 0.0) v = 0.0;  // -0.0 ties with +0.0
  uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key2f_s(uint64_t k) {
  uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

// X [R x S] row-major fp64 -> Kc [S][R] keys; 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void transpose_keys_kernel(
    const double* __restrict__ X, int64_t R, int S, uint64_t* __restrict__ Kc) {
  __shared__ uint64_t tile[TP][TP + 1];
  const int64_t r0 = (int64_t)blockIdx.x * TP;
  const int c0 = blockIdx.y * TP;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  for (int i = ty; i < TP; i += 4) {
    const int64_t r = r0 + i;
    const int c = c0 + tx;
    if (r < R && c < S) tile[i][tx] = f2key_s(X[r * S + c]);
  }
  __syncthreads();
  for (int i = ty; i < TP; i += 4) {
    const int c = c0 + i;
    const int64_t r = r0 + tx;
    if (r < R && c < S) Kc[(int64_t)c * R + r] = tile[tx][i];
  }
}

// sample bracketing: columns with R >= BR_MIN first take SMP evenly spaced
// keys, sort them in LDS and keep only the keys between the sample order
// statistics BR_MARG places either side of the wanted rank(s) (5.7 sigma of
// the sample rank at the median).  One streaming pass counts the keys below
// the window and compacts the window into scratch; the radix levels then run
// on ~12% of the column.  When the rank is not inside the window (a sample
// that misrepresents the column) the full radix select runs instead.
constexpr int SMP = 2 * SEL_T;
constexpr int BR_MARG = 128;
constexpr int64_t BR_MIN = 4 * SMP;
constexpr int BR_U = 8;  // keys in flight per thread in the bracket pass

struct SelShared {
  uint32_t hist[SEL_BINS];
  uint64_t smp[SMP];
  uint32_t wsum[SEL_T / 64];
  unsigned long long vmin;
  unsigned long long below;
  uint64_t lo, hi;
  uint32_t cnt;
  int b1, b2;
  int64_t below1;
};

// ascending bitonic sort of sh.smp (SMP = 2 x blockDim keys)
__device__ void sort_sample(SelShared& sh) {
  const int t = threadIdx.x;
  for (int size = 2; size <= SMP; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int i = 2 * t - (t & (stride - 1));
      const int j = i + stride;
      const bool asc = (i & size) == 0;
      const uint64_t a = sh.smp[i], b = sh.smp[j];
      if ((a > b) == asc) { sh.smp[i] = b; sh.smp[j] = a; }
      __syncthreads();
    }
  }
}

// exclusive-prefix search over the histogram: bin holding rank k (and k+1)
__device__ void find_bins(SelShared& sh, int64_t k, bool want2) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  constexpr int PER = SEL_BINS / SEL_T;  // 4 bins per thread
  uint32_t loc[PER];
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) { loc[q] = sh.hist[t * PER + q]; s += loc[q]; }
  // inclusive scan of s over the block
  uint32_t v = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  if (lane == 63) sh.wsum[wv] = v;
  __syncthreads();
  uint32_t wbase = 0;
  for (int w = 0; w < wv; ++w) wbase += sh.wsum[w];
  int64_t run = (int64_t)wbase + v - s;  // exclusive prefix of this thread
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int64_t nxt = run + loc[q];
    if (k >= run && k < nxt) { sh.b1 = t * PER + q; sh.below1 = run; }
    if (want2 && k + 1 >= run && k + 1 < nxt) sh.b2 = t * PER + q;
    run = nxt;
  }
  __syncthreads();
}

// DEV: keys are f2key(|key2f(Kc) - med[c]|) (the MAD deviations)
template <bool DEV>
__global__ __launch_bounds__(SEL_T) void col_select_kernel(
    const uint64_t* __restrict__ Kc, int64_t R, const double* __restrict__ med,
    uint64_t* __restrict__ scratch, double* __restrict__ out) {
  __shared__ SelShared sh;
  const int c = blockIdx.x;
  const int t = threadIdx.x;
  const uint64_t* col = Kc + (int64_t)c * R;
  uint64_t* sc = scratch + (int64_t)c * R;
  const double m = DEV ? med[c] : 0.0;
  auto keyof = [&](uint64_t k) -> uint64_t {
    if (!DEV) return k;
    return f2key_s(fabs(key2f_s(k) - m));
  };
  int64_t k = (R & 1) ? (R - 1) / 2 : R / 2 - 1;
  bool want2 = (R & 1) == 0;     // still tracking rank k+1 inside the set
  bool have2 = false;            // rank k+1 resolved as a bin minimum
  uint64_t v2 = 0;
  int64_t n = R;
  bool in_scratch = false;
  const int lane = t & 63;
  if (R >= BR_MIN) {
    // ---- sample bracketing (see BR_MARG): one pass instead of two
    for (int q = t; q < SMP; q += SEL_T)
      sh.smp[q] = keyof(col[((2 * (int64_t)q + 1) * R) / (2 * SMP)]);
    if (t == 0) { sh.cnt = 0; sh.below = 0; }
    __syncthreads();
    sort_sample(sh);
    if (t == 0) {
      const int64_t j1 = (k * SMP) / R - BR_MARG;
      const int64_t j2 = ((k + (want2 ? 1 : 0)) * SMP) / R + BR_MARG;
      sh.lo = j1 < 0 ? 0ull : sh.smp[j1];
      sh.hi = j2 >= SMP ? ~0ull : sh.smp[j2];
    }
    __syncthreads();
    const uint64_t lo = sh.lo, hi = sh.hi;
    uint64_t below = 0;
    for (int64_t base = 0; base < R; base += (int64_t)SEL_T * BR_U) {
      uint64_t kv[BR_U];
      bool keep[BR_U];
      uint64_t bal[BR_U];
#pragma unroll
      for (int u = 0; u < BR_U; ++u) {
        const int64_t i = base + (int64_t)u * SEL_T + t;
        kv[u] = i < R ? col[i] : 0;
      }
      uint32_t tot = 0;
#pragma unroll
      for (int u = 0; u < BR_U; ++u) {
        const int64_t i = base + (int64_t)u * SEL_T + t;
        const uint64_t key = keyof(kv[u]);
        kv[u] = key;
        below += (i < R && key < lo) ? 1 : 0;
        keep[u] = i < R && key >= lo && key <= hi;
        bal[u] = __ballot(keep[u]);
        tot += (uint32_t)__popcll(bal[u]);
      }
      uint32_t wpos = 0;
      if (lane == 0 && tot) wpos = atomicAdd(&sh.cnt, tot);
      wpos = __shfl(wpos, 0, 64);
      const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
      for (int u = 0; u < BR_U; ++u) {
        if (keep[u]) sc[wpos + __popcll(bal[u] & lt)] = kv[u];
        wpos += (uint32_t)__popcll(bal[u]);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) below += __shfl_down(below, o, 64);
    if (lane == 0 && below) atomicAdd(&sh.below, (unsigned long long)below);
    __syncthreads();
    const int64_t nin = sh.cnt, bel = (int64_t)sh.below;
    if (bel <= k && k + (want2 ? 1 : 0) < bel + nin) {  // uniform
      k -= bel;
      n = nin;
      in_scratch = true;
    }
    // else: the full select below, from the column
  }
  // ---- level 0: histogram of the top digit over the (bracketed) set
  for (int i = t; i < SEL_BINS; i += SEL_T) sh.hist[i] = 0;
  if (t == 0) sh.b2 = -1;
  __syncthreads();
  int shift = 64 - SEL_BITS;
  for (int64_t base = 0; base < n; base += (int64_t)SEL_T * BR_U) {
    uint64_t kv[BR_U];
#pragma unroll
    for (int u = 0; u < BR_U; ++u) {
      const int64_t i = base + (int64_t)u * SEL_T + t;
      kv[u] = i < n ? (in_scratch ? sc[i] : col[i]) : 0;
    }
#pragma unroll
    for (int u = 0; u < BR_U; ++u) {
      const int64_t i = base + (int64_t)u * SEL_T + t;
      if (i < n) {
        const uint64_t key = in_scratch ? kv[u] : keyof(kv[u]);
        atomicAdd(&sh.hist[(key >> shift) & (SEL_BINS - 1)], 1u);
      }
    }
  }
  __syncthreads();
  find_bins(sh, k, want2);
  uint64_t prefix = 0, pmask = 0;
  while (true) {
    const int b1 = sh.b1, b2 = sh.b2;
    k -= sh.below1;
    const bool track_min = want2 && b2 != b1;  // k+1 = min of bin b2
    if (track_min) want2 = false;
    prefix |= (uint64_t)b1 << shift;
    pmask |= (uint64_t)(SEL_BINS - 1) << shift;
    if (shift == 0) {  // every bit decided: the key is `prefix`
      // last digit: each bin is one key value, rank k+1's is higher | b2
      if (track_min) { have2 = true; v2 = (prefix ^ (uint64_t)b1) | (uint64_t)b2; }
      break;
    }
    const int nshift = shift >= SEL_BITS ? shift - SEL_BITS : 0;
    const int nbits = shift - nshift;
    const uint64_t nmask = (1ull << nbits) - 1;
    __syncthreads();
    for (int i = t; i < SEL_BINS; i += SEL_T) sh.hist[i] = 0;
    if (t == 0) { sh.cnt = 0; sh.vmin = ~0ull; sh.b2 = -1; }
    __syncthreads();
    // compaction pass: keep the keys of bin b1, histogram their next digit;
    // in place (chunk-wise behind a barrier) once the set lives in scratch
    const uint64_t* src = in_scratch ? sc : col;
    for (int64_t base = 0; base < n; base += SEL_T * 4) {
      uint64_t kv[4];
      bool keep[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = base + (int64_t)u * SEL_T + t;
        keep[u] = false;
        if (i < n) {
          kv[u] = in_scratch ? src[i] : keyof(src[i]);
          const uint64_t hi = (kv[u] & pmask) ^ prefix;  // 0 iff in bin b1
          keep[u] = hi == 0;
          if (track_min && ((kv[u] >> shift) & (SEL_BINS - 1)) == (uint64_t)b2 &&
              ((kv[u] >> shift) >> SEL_BITS) == (prefix >> shift >> SEL_BITS))
            atomicMin(&sh.vmin, (unsigned long long)kv[u]);
        }
      }
      if (in_scratch) __syncthreads();  // all reads of the chunk done
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (keep[u]) {
          const uint32_t pos = atomicAdd(&sh.cnt, 1u);
          sc[pos] = kv[u];
          atomicAdd(&sh.hist[(kv[u] >> nshift) & nmask], 1u);
        }
      }
      if (in_scratch) __syncthreads();
    }
    __syncthreads();
    if (track_min) { have2 = true; v2 = sh.vmin; }
    n = sh.cnt;
    in_scratch = true;
    shift = nshift;
    // next digit is only nbits wide: bins above nmask stay empty
    find_bins(sh, k, want2);
  }
  if (t == 0) {
    const double v1 = key2f_s(prefix);
    double r = v1;
    if ((R & 1) == 0) {
      const double w2 = have2 ? key2f_s(v2) : v1;  // same final bin: equal keys
      r = (v1 + w2) / 2.0;
    }
    out[c] = r;
  }
}

}  // namespace

size_t select_ws_bytes(int64_t R, int S) {
  size_t off = 0;
  size_only<uint64_t>(off, (size_t)R * S);  // keys
  size_only<uint64_t>(off, (size_t)R * S);  // scratch
  size_only<double>(off, (size_t)S);        // medians
  return off + 256;
}

// out[c] = median_c(|X[:, c] - median_c(X[:, c])|)
int column_mad_select(const double* X, int64_t R, int S, double* out, void* ws,
                      size_t ws_bytes, hipStream_t s) {
  Carver cv(ws, ws_bytes);
  uint64_t* Kc = cv.take<uint64_t>((size_t)R * S);
  uint64_t* scratch = cv.take<uint64_t>((size_t)R * S);
  double* med = cv.take<double>((size_t)S);
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "column_mad: workspace carve");
  hipLaunchKernelGGL(transpose_keys_kernel,
                     dim3((unsigned)ceil_div(R, TP), (unsigned)ceil_div(S, TP)),
                     dim3(256), 0, s, X, R, S, Kc);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(col_select_kernel<false>, dim3((unsigned)S), dim3(SEL_T), 0, s,
                     (const uint64_t*)Kc, R, (const double*)nullptr, scratch, med);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(col_select_kernel<true>, dim3((unsigned)S), dim3(SEL_T), 0, s,
                     (const uint64_t*)Kc, R, (const double*)med, scratch, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

}  // namespace abc
