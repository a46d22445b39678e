// Per-column exact order statistics by radix select, for the
// AdaptivePNormDistance scale update with median_absolute_deviation.
//
// Reference: pyabc/distance/scale.py:38-47
//   median_absolute_deviation(data) = np.median(np.abs(data - np.median(data)))
// over the recorded summary statistics of one key (distance.py:263-307), i.e.
// per column of the recorded [R x S] matrix.  np.median: the middle order
// statistic for odd R, the mean (a + b) / 2 of the two middle ones for even R.
//
// Layout: the recorded matrix stays row-major [R x S] fp64 (no transposed
// copy).  Per pass (the median, then the median of |x - median|):
//   col_sample_kernel   one workgroup per column sorts SMP evenly spaced
//                       keys and brackets the wanted rank(s) by the sample
//                       order statistics BR_MARG places either side;
//   col_bracket_kernel  one streaming, coalesced read of the whole matrix
//                       (each thread owns one column of a row band) counts
//                       the keys below each column's window and compacts
//                       the window (~9% of the column) into scratch;
//   col_select_kernel   one 1024-thread workgroup per column selects the
//                       rank-k key inside the window with 12-bit MSD digits:
//     level 0: histogram of bits 63..52 (LDS atomics), pick the bin holding
//              rank k;
//     level l: one pass over the surviving set that compacts the keys of the
//              picked bin in place (chunk-wise behind a barrier) and
//              histograms their next digit.
// When a column's rank is not inside its window (a sample that
// misrepresents the column) the select runs over the whole column, read
// strided from X.  For even R the (k+1)-th statistic is tracked along: while
// it falls in the same bin it survives with rank k; once it falls in the
// next non-empty bin it is the minimum of that bin, taken in the next pass
// (LDS 64-bit atomic min).  Results are exact and bitwise deterministic (the
// selection does not depend on the order of the compacted keys).
#include "abc_common.h"

namespace abc {
namespace {

constexpr int SEL_T = 1024;
constexpr int SEL_BITS = 12, SEL_BINS = 1 << SEL_BITS;

__device__ __forceinline__ uint64_t f2key_s(double v) {
  if (v == 0.0) v = 0.0;  // -0.0 ties with +0.0
  uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key2f_s(uint64_t k) {
  uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

// sample bracketing: columns with R >= BR_MIN first take SMP evenly spaced
// keys, sort them in LDS and keep only the keys between the sample order
// statistics BR_MARG places either side of the wanted rank(s) (5.75 sigma of
// the sample rank at the median).  One streaming pass counts the keys below
// the window and compacts the window into scratch; the radix levels then run
// on ~9% of the column.  When the rank is not inside the window (a sample
// that misrepresents the column) the full radix select runs instead.
constexpr int SMP = 4 * SEL_T;
constexpr int BR_MARG = 184;
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

// ascending bitonic sort of sh.smp (SMP keys, SMP / 2 compare-exchange
// pairs per stage spread over the block)
__device__ void sort_sample(SelShared& sh) {
  static_assert(SMP % (2 * SEL_T) == 0, "whole pair sets per thread");
  for (int size = 2; size <= SMP; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int pidx = threadIdx.x; pidx < SMP / 2; pidx += SEL_T) {
        const int i = 2 * pidx - (pidx & (stride - 1));
        const int j = i + stride;
        const bool asc = (i & size) == 0;
        const uint64_t a = sh.smp[i], b = sh.smp[j];
        if ((a > b) == asc) { sh.smp[i] = b; sh.smp[j] = a; }
      }
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

// key of element i of column c (DEV: of |x - med|, the MAD deviations)
template <bool DEV>
__device__ __forceinline__ uint64_t col_key(const double* __restrict__ X, int S, int c,
                                            int64_t i, double m) {
  const double v = X[i * S + c];
  return DEV ? f2key_s(fabs(v - m)) : f2key_s(v);
}
// the rank(s) the median needs: k (and k + 1 for even R)
__host__ __device__ inline int64_t med_rank(int64_t R) { return (R & 1) ? (R - 1) / 2 : R / 2 - 1; }

// Per column: sample SMP keys, sort them and store the key window [lo, hi]
// that brackets the wanted rank(s); columns shorter than BR_MIN get the
// whole key range (their "window" is the column).
template <bool DEV>
__global__ __launch_bounds__(SEL_T) void col_sample_kernel(
    const double* __restrict__ X, int64_t R, int S, const double* __restrict__ med,
    uint64_t* __restrict__ win, unsigned long long* __restrict__ cnt) {
  __shared__ SelShared sh;
  const int c = blockIdx.x, t = threadIdx.x;
  if (t == 0) { cnt[2 * c] = 0ull; cnt[2 * c + 1] = 0ull; }  // in window, below
  if (R < BR_MIN) {
    if (t == 0) { win[2 * c] = 0ull; win[2 * c + 1] = ~0ull; }
    return;
  }
  const double m = DEV ? med[c] : 0.0;
  for (int q = t; q < SMP; q += SEL_T)
    sh.smp[q] = col_key<DEV>(X, S, c, ((2 * (int64_t)q + 1) * R) / (2 * SMP), m);
  __syncthreads();
  sort_sample(sh);
  if (t == 0) {
    const int64_t k = med_rank(R);
    const int64_t j1 = (k * SMP) / R - BR_MARG;
    const int64_t j2 = ((k + ((R & 1) ? 0 : 1)) * SMP) / R + BR_MARG;
    win[2 * c] = j1 < 0 ? 0ull : sh.smp[j1];
    win[2 * c + 1] = j2 >= SMP ? ~0ull : sh.smp[j2];
  }
}

// One coalesced read of X: thread t of a block owns column c0 + t % CB of
// the rows r = t / CB (mod RPI) of the block's band of BK_ROWS rows.  Keys
// below a column's window are counted in registers; keys inside it go to an
// LDS pool of (key, column) pairs (LDS atomics only).  After the band, one
// global atomic per column reserves room in the column's scratch segment and
// the pool is scattered there.  A band whose window keys overflow the pool
// (heavy ties: a constant column is all window) sends the rest straight to
// scratch, one returning global atomic per key.  The order of the compacted
// keys is not deterministic; the selection does not depend on it.
constexpr int BK_T = 256, BK_U = 16, BK_ROWS = 160, BK_CAP = 4096;
template <bool DEV>
__global__ __launch_bounds__(BK_T) void col_bracket_kernel(
    const double* __restrict__ X, int64_t R, int S, const double* __restrict__ med,
    const uint64_t* __restrict__ win, int64_t rows_per_block,
    unsigned long long* __restrict__ cnt, uint64_t* __restrict__ scratch) {
  __shared__ uint64_t pool[BK_CAP];
  __shared__ uint16_t pool_c[BK_CAP];
  __shared__ uint32_t pool_n;
  __shared__ uint32_t col_n[BK_T];                 // pool keys per local column
  __shared__ unsigned long long col_base[BK_T];    // their scratch offsets
  const int t = threadIdx.x;
  const int CB = S < BK_T ? S : BK_T;              // columns per block
  const int RPI = BK_T / CB;                       // rows per iteration
  const int cl = t % CB;
  const int c = blockIdx.y * CB + cl;
  const int rsub = t / CB;
  const bool active = rsub < RPI && c < S;
  if (t == 0) pool_n = 0;
  col_n[t] = 0;
  __syncthreads();
  const double m = (DEV && active) ? med[c] : 0.0;
  const uint64_t lo = active ? win[2 * c] : 0ull, hi = active ? win[2 * c + 1] : 0ull;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < R ? r0 + rows_per_block : R;
  uint64_t* sc = scratch + (int64_t)c * R;
  unsigned long long below = 0;
  auto take = [&](uint64_t key) {
    below += key < lo ? 1ull : 0ull;
    if (key >= lo && key <= hi) {
      const uint32_t pos = atomicAdd(&pool_n, 1u);
      if (pos < (uint32_t)BK_CAP) {
        pool[pos] = key;
        pool_c[pos] = (uint16_t)cl;
        atomicAdd(&col_n[cl], 1u);
      } else {  // overflow: straight to scratch
        sc[atomicAdd(&cnt[2 * c], 1ull)] = key;
      }
    }
  };
  if (active) {
    int64_t r = r0 + rsub;
    for (; r + (BK_U - 1) * RPI < r1; r += BK_U * RPI) {
      uint64_t k4[BK_U];
#pragma unroll
      for (int u = 0; u < BK_U; ++u) k4[u] = col_key<DEV>(X, S, c, r + u * RPI, m);
#pragma unroll
      for (int u = 0; u < BK_U; ++u) take(k4[u]);
    }
    for (; r < r1; r += RPI) take(col_key<DEV>(X, S, c, r, m));
    if (below) atomicAdd(&cnt[2 * c + 1], below);
  }
  __syncthreads();
  // one reservation per column, then the pool in place (col_n counts down)
  if (t < CB && blockIdx.y * CB + t < S && col_n[t])
    col_base[t] = atomicAdd(&cnt[2 * (blockIdx.y * CB + t)], (unsigned long long)col_n[t]);
  __syncthreads();
  const uint32_t np = pool_n < (uint32_t)BK_CAP ? pool_n : (uint32_t)BK_CAP;
  for (uint32_t e = t; e < np; e += BK_T) {
    const int q = pool_c[e];
    const uint32_t slot = atomicSub(&col_n[q], 1u) - 1u;
    scratch[(int64_t)(blockIdx.y * CB + q) * R + col_base[q] + slot] = pool[e];
  }
}

// Rank-k select of column c from its compacted window (cnt[2c] keys in
// scratch, cnt[2c + 1] keys below it), or from the whole column when the
// rank is outside the window.
template <bool DEV>
__global__ __launch_bounds__(SEL_T) void col_select_kernel(
    const double* __restrict__ X, int64_t R, int S, const double* __restrict__ med,
    const unsigned long long* __restrict__ cnt, const uint64_t* __restrict__ win,
    uint64_t* __restrict__ scratch, double* __restrict__ out) {
  __shared__ SelShared sh;
  const int c = blockIdx.x;
  const int t = threadIdx.x;
  uint64_t* sc = scratch + (int64_t)c * R;
  const double m = DEV ? med[c] : 0.0;
  auto colkey = [&](int64_t i) -> uint64_t { return col_key<DEV>(X, S, c, i, m); };
  int64_t k = med_rank(R);
  bool want2 = (R & 1) == 0;     // still tracking rank k+1 inside the set
  bool have2 = false;            // rank k+1 resolved as a bin minimum
  uint64_t v2 = 0;
  int64_t n = R;
  bool in_scratch = false;
  int top = 64;                  // bits below which the candidate keys differ
  {
    const int64_t nin = (int64_t)cnt[2 * c], bel = (int64_t)cnt[2 * c + 1];
    if (bel <= k && k + (want2 ? 1 : 0) < bel + nin) {  // uniform
      k -= bel;
      n = nin;
      in_scratch = true;
      // every window key lies in [lo, hi], so shares their common high bits:
      // the digits start below them (no pass over a constant digit)
      const uint64_t d = win[2 * c] ^ win[2 * c + 1];
      top = d ? 64 - __clzll((long long)d) : 0;
    }
    // else: the full select below, from the column
  }
  const uint64_t low = top >= 64 ? ~0ull : ((1ull << top) - 1);
  // ---- level 0: histogram of the top digit over the (bracketed) set
  for (int i = t; i < SEL_BINS; i += SEL_T) sh.hist[i] = 0;
  if (t == 0) sh.b2 = -1;
  __syncthreads();
  int shift = top > SEL_BITS ? top - SEL_BITS : 0;
  for (int64_t base = 0; base < n; base += (int64_t)SEL_T * BR_U) {
    uint64_t kv[BR_U];
#pragma unroll
    for (int u = 0; u < BR_U; ++u) {
      const int64_t i = base + (int64_t)u * SEL_T + t;
      kv[u] = i < n ? (in_scratch ? sc[i] : colkey(i)) : 0;
    }
#pragma unroll
    for (int u = 0; u < BR_U; ++u) {
      const int64_t i = base + (int64_t)u * SEL_T + t;
      if (i < n) {
        atomicAdd(&sh.hist[(kv[u] >> shift) & (SEL_BINS - 1)], 1u);
      }
    }
  }
  __syncthreads();
  find_bins(sh, k, want2);
  uint64_t pmask = ~low, prefix = in_scratch ? (win[2 * c] & pmask) : 0ull;
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
    for (int64_t base = 0; base < n; base += SEL_T * 4) {
      uint64_t kv[4];
      bool keep[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = base + (int64_t)u * SEL_T + t;
        keep[u] = false;
        if (i < n) {
          kv[u] = in_scratch ? sc[i] : colkey(i);
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
  size_only<uint64_t>(off, (size_t)R * S);             // window keys (worst case: all)
  size_only<uint64_t>(off, (size_t)2 * S);             // windows [lo, hi]
  size_only<unsigned long long>(off, (size_t)2 * S);   // in-window / below counts
  size_only<double>(off, (size_t)S);                   // medians
  return off + 256;
}

// out[c] = median_c(|X[:, c] - median_c(X[:, c])|)
int column_mad_select(const double* X, int64_t R, int S, double* out, void* ws,
                      size_t ws_bytes, hipStream_t s) {
  Carver cv(ws, ws_bytes);
  uint64_t* scratch = cv.take<uint64_t>((size_t)R * S);
  uint64_t* win = cv.take<uint64_t>((size_t)2 * S);
  unsigned long long* cnt = cv.take<unsigned long long>((size_t)2 * S);
  double* med = cv.take<double>((size_t)S);
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "column_mad: workspace carve");
  const int CB = S < BK_T ? S : BK_T;
  const int ctiles = (int)ceil_div(S, CB);
  // expected window keys per band 2 BR_MARG / SMP = 9% x 160 x 256 = 3680 <
  // BK_CAP.  Measured at c4 (same box, tools/ab.sh mad): SMP 2048 / 96 rows /
  // 8 loads in flight 1.12 ms per MAD; 16 in flight 1.12; SMP 4096 / 128 rows
  // 1.05; SMP 4096 / 160 rows / 16 in flight 1.03.  Without the compaction
  // the bracket pass streams at 253 us (the colsum rate); with it 367 us.
  // Per-column LDS segments flushed 64 keys a store over 64-column tiles
  // were slower (470 us: a block then reads 512-B pieces of 512 rows
  // instead of whole 2-KB rows)
  const int64_t rpb = BK_ROWS;
  const unsigned nb = (unsigned)ceil_div(R, rpb);
  for (int pass = 0; pass < 2; ++pass) {
    const bool dev = pass == 1;
    double* dst = dev ? out : med;
    if (!dev) {
      hipLaunchKernelGGL(col_sample_kernel<false>, dim3((unsigned)S), dim3(SEL_T), 0, s, X, R, S,
                         (const double*)med, win, cnt);
    } else {
      hipLaunchKernelGGL(col_sample_kernel<true>, dim3((unsigned)S), dim3(SEL_T), 0, s, X, R, S,
                         (const double*)med, win, cnt);
    }
    ABC_LAUNCHED();
    if (!dev) {
      hipLaunchKernelGGL(col_bracket_kernel<false>, dim3(nb, (unsigned)ctiles), dim3(BK_T), 0, s,
                         X, R, S, (const double*)med, (const uint64_t*)win, rpb, cnt, scratch);
    } else {
      hipLaunchKernelGGL(col_bracket_kernel<true>, dim3(nb, (unsigned)ctiles), dim3(BK_T), 0, s,
                         X, R, S, (const double*)med, (const uint64_t*)win, rpb, cnt, scratch);
    }
    ABC_LAUNCHED();
    if (!dev) {
      hipLaunchKernelGGL(col_select_kernel<false>, dim3((unsigned)S), dim3(SEL_T), 0, s, X, R, S,
                         (const double*)med, (const unsigned long long*)cnt, (const uint64_t*)win,
                         scratch, dst);
    } else {
      hipLaunchKernelGGL(col_select_kernel<true>, dim3((unsigned)S), dim3(SEL_T), 0, s, X, R, S,
                         (const double*)med, (const unsigned long long*)cnt, (const uint64_t*)win,
                         scratch, dst);
    }
    ABC_LAUNCHED();
  }
  return ABC_OK;
}

}  // namespace abc
