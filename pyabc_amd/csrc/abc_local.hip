// LocalTransition on CDNA4: per-particle k-NN covariance fit, density, rvs.
//
// Reference: pyabc/transition/local_transition.py
//   fit   :77-96   cKDTree.query(X, k+1) per particle, then a Python loop of
//                  _cov_and_inv (:112-123) / _cov (:125-139) per particle
//   pdf   :98-110  np.average(exp(-d^T inv_j d / 2) / norm_j, weights=w)
//   rvs   :141-145 j ~ Cat(w); theta ~ N(X_j, cov_j)  (abc_local_propose in
//                  abc_sampler.hip uses the Cholesky factors written here)
//
// fit: workgroups of 8 particles find the k+1 nearest particles in
// (squared distance, index) order by an exact select on the fp64 bits of the
// squared distances (sample-bracketed window, MSD radix passes as fallback,
// the rank's bucket selected in LDS); then one particle per lane accumulates
// the weighted moments of the neighbour offsets over wave-uniform rows (ties
// at the k-th distance taken by index, rank 0 dropped like the reference's
// indices[n, 1:]), and a finishing kernel applies the reference's fix-ups
// (diag(|X[0]|) for an all-zero covariance, scaling, "while det <= 0: cov +=
// EPS I") and writes cov, inverse (Gauss-Jordan with partial pivoting), det
// (LU), Cholesky and log normalisation.
#include "abc_common.h"

namespace abc {
namespace {

constexpr double LOG_2PI = 1.8378770664093454836;
constexpr double LOG2E_L = 1.4426950408889634074;
constexpr double LN2_L = 0.69314718055994530942;

// squared distance with explicit fma: the select and accumulate kernels must
// produce bit-identical keys
template <int D>
__device__ __forceinline__ double dist2v(const double (&xj)[D], const double* xn) {
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < D; ++q) { const double t = xj[q] - xn[q]; s = __builtin_fma(t, t, s); }
  return s;
}
template <int D>
__device__ __forceinline__ double dist2(const double* __restrict__ X, int64_t j,
                                        const double (&xn)[D]) {
  double xj[D];
#pragma unroll
  for (int q = 0; q < D; ++q) xj[q] = X[j * D + q];
  return dist2v<D>(xj, xn);
}

// ---- fp32 prefilter of the fp64 squared distances ---------------------------
// The moments sweep compares s = |x_j - x_n|^2 (the fp64 fma chain of
// dist2v) with the particle's k-th key v*.  The same chain in fp32 on fp32
// copies of X, s32, decides most comparisons at twice the fp64 rate (k = 50
// at c5: 7.1 -> 3.3 ms; in the selection sweeps the extra registers cost
// more occupancy and branching than the fp32 arithmetic saved: 15.9 ms
// fp64 vs 31.1 ms prefiltered with 8 particles per block, 23.5 ms with 4,
// so they stay fp64): with u = 2^-24, M = max |x| over the population and
// the exact
// s (and every fp32/fp64 rounding of the copies, the differences and the
// fma chain accounted for)
//   |s32 - s64| <= B(s) = 1.01 (4 u M sqrt(D s) + (D + 2) u s
//                               + D u^2 (2 M + sqrt(s))^2) + 2^-1000,
// B increasing and s - B(s) increasing above the tiny floor handled below,
// so s32 < V - B(V) implies s64 < V and s32 > V + B(V) implies s64 > V.
// Pairs between the two cuts, and s32 == 0 (exact duplicates, the rank-0
// index), take the fp64 path.  The cuts are rounded outward to fp32.
template <int D>
__device__ __forceinline__ float dist2f(const float (&xj)[D], const float (&xn)[D]) {
  float s = 0.0f;
#pragma unroll
  for (int q = 0; q < D; ++q) { const float t = xj[q] - xn[q]; s = __builtin_fmaf(t, t, s); }
  return s;
}
template <int D>
__device__ __forceinline__ double f32_bound(double V, double M) {
  constexpr double u = 5.9604644775390625e-08;  // 2^-24
  const double r = sqrt(V);
  return 1.01 * (4.0 * u * M * sqrt((double)D) * r + (D + 2) * u * V +
                 D * u * u * (2.0 * M + r) * (2.0 * M + r)) + 1e-300;
}
// fp32 c with c <= V - B(V) (-1 when that is not positive: no fast "below")
template <int D>
__device__ __forceinline__ float f32_cut_below(double V, double M) {
  const double t = V - f32_bound<D>(V, M);
  if (!(t > 0.0)) return -1.0f;
  float c = (float)t;
  if ((double)c > t) c = __uint_as_float(__float_as_uint(c) - 1u);  // c > t > 0
  return c;
}
// fp32 c with c >= V + B(V) (+inf when V is not finite)
template <int D>
__device__ __forceinline__ float f32_cut_above(double V, double M) {
  const double t = V + f32_bound<D>(V, M);
  if (!(t < 3.0e38)) return INFINITY;
  float c = (float)t;
  if ((double)c < t) c = __uint_as_float(__float_as_uint(c) + 1u);  // 0 < c < t
  return c;
}
__device__ __forceinline__ double key_val(unsigned long long k) {
  return __longlong_as_double((long long)k);
}

// X32 = (float)X and M = max |X| (bits of a non-negative double, block-reduced
// atomic max; a NaN orders above +inf and disables every fast path)
__global__ __launch_bounds__(256) void local_prep_kernel(const double* __restrict__ X, int64_t n,
                                                         float* __restrict__ X32,
                                                         unsigned long long* __restrict__ mbits) {
  __shared__ unsigned long long wm[4];
  unsigned long long a = 0ull;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const double v = X[e];
    X32[e] = (float)v;
    const unsigned long long b = (unsigned long long)__double_as_longlong(fabs(v));
    a = b > a ? b : a;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long b = __shfl_xor(a, o, 64);
    a = b > a ? b : a;
  }
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0ull;
    for (int w = 0; w < 4; ++w) m = wm[w] > m ? wm[w] : m;
    atomicMax(mbits, m);
  }
}

#include "abc_local_knn.h"

// LU with partial pivoting (getrf order: pivot = first max |a[r][c]|,
// multipliers l = a[r][c] * (1 / pivot)); returns det and keeps the factors
// in a, the row permutation in perm.  The determinant and the inverse come
// from the same factors, as la.det and la.inv (getrf + getri) do in the
// reference: with two independently rounded factorisations a nearly
// singular covariance could pass "det > 0" while its inverse is indefinite.
template <int D>
__device__ double lu_factor(double (&a)[D][D], int (&perm)[D]) {
  double det = 1.0;
  for (int i = 0; i < D; ++i) perm[i] = i;
  for (int c = 0; c < D; ++c) {
    int p = c;
    double best = fabs(a[c][c]);
    for (int r = c + 1; r < D; ++r)
      if (fabs(a[r][c]) > best) { best = fabs(a[r][c]); p = r; }
    if (a[p][c] == 0.0) return 0.0;
    if (p != c) {
      for (int j = 0; j < D; ++j) { double t = a[c][j]; a[c][j] = a[p][j]; a[p][j] = t; }
      const int t = perm[c]; perm[c] = perm[p]; perm[p] = t;
      det = -det;
    }
    det *= a[c][c];
    const double rp = 1.0 / a[c][c];
    for (int r = c + 1; r < D; ++r) {
      const double f = a[r][c] * rp;
      a[r][c] = f;
      for (int j = c + 1; j < D; ++j) a[r][j] -= f * a[c][j];
    }
  }
  return det;
}

// inverse from the factors of lu_factor (det != 0): column j of A^-1 solves
// L U x = P e_j
template <int D>
__device__ void lu_inverse(const double (&lu)[D][D], const int (&perm)[D],
                           double (&inv)[D][D]) {
  for (int j = 0; j < D; ++j) {
    double x[D];
    for (int i = 0; i < D; ++i) {
      double v = perm[i] == j ? 1.0 : 0.0;
      for (int k = 0; k < i; ++k) v -= lu[i][k] * x[k];
      x[i] = v;
    }
    for (int i = D - 1; i >= 0; --i) {
      double v = x[i];
      for (int k = i + 1; k < D; ++k) v -= lu[i][k] * x[k];
      x[i] = v / lu[i][i];
    }
    for (int i = 0; i < D; ++i) inv[i][j] = x[i];
  }
}

// Cholesky; on a non-positive pivot fall back to sqrt(|diag|) (the reference
// samples such covariances through an SVD; not a case the fits produce after
// the det > 0 loop unless the matrix is indefinite).
template <int D>
__device__ void cholesky(const double (&a)[D][D], double (&L)[D][D]) {
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) L[i][j] = 0.0;
  bool ok = true;
  for (int j = 0; j < D && ok; ++j) {
    double s = a[j][j];
    for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
    if (!(s > 0.0)) { ok = false; break; }
    L[j][j] = sqrt(s);
    for (int i = j + 1; i < D; ++i) {
      double t = a[i][j];
      for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
      L[i][j] = t / L[j][j];
    }
  }
  if (!ok)
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) L[i][j] = (i == j) ? sqrt(fabs(a[i][i])) : 0.0;
}

constexpr int SEL_CAP = 256;  // LDS list of the rank bucket
constexpr int BR_SK = 512;    // k-NN sample rows per block (sample bracketing)
constexpr int BR_NB = 520;    // window histogram bins (offsets 0..512 used)
constexpr int BR_PER = (BR_NB + 31) / 32;

// Collect the (key, index) pairs of each particle's rank bucket -- keys with
// (key >> s_sh[p]) == s_prefix[p] -- into LDS in one sweep and select rank
// s_rank[p] by (key, index) order.  Writes v*, the index cutoff of the ties
// and the rank-0 index.
template <int D, int PB>
__device__ __forceinline__ void collect_select(
    const double* __restrict__ X, int64_t N, int64_t n0, const double (&xr)[PB][D],
    const int* s_sh, const unsigned long long* s_prefix, const long long* s_rank,
    const unsigned long long* s_rank0, unsigned long long (*s_lkey)[2 * SEL_CAP],
    int* s_lcnt, unsigned long long* __restrict__ sel_v,
    long long* __restrict__ sel_jcut, long long* __restrict__ sel_rank0) {
  const int tid = threadIdx.x;
  if (tid < PB) s_lcnt[tid] = 0;
  __syncthreads();
  int sh[PB];
  unsigned long long pre[PB];
#pragma unroll
  for (int q = 0; q < PB; ++q) { sh[q] = s_sh[q]; pre[q] = s_prefix[q]; }
  for (int64_t j = tid; j < N; j += 256) {
    double xj[D];
#pragma unroll
    for (int q = 0; q < D; ++q) xj[q] = X[j * D + q];
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const unsigned long long key =
          (unsigned long long)__double_as_longlong(dist2v<D>(xj, xr[q]));
      if ((key >> sh[q]) == pre[q]) {
        const int slot = atomicAdd(&s_lcnt[q], 1);
        s_lkey[q][slot] = key;
        s_lkey[q][SEL_CAP + slot] = (unsigned long long)j;
      }
    }
  }
  __syncthreads();
  for (int q = 0; q < PB; ++q) {
    const int cnt = s_lcnt[q];
    const long long r = s_rank[q];
    for (int e = tid; e < cnt; e += 256) {
      const unsigned long long ke = s_lkey[q][e];
      const long long je = (long long)s_lkey[q][SEL_CAP + e];
      int less = 0;
      for (int f = 0; f < cnt; ++f) {
        const unsigned long long kf = s_lkey[q][f];
        less += (kf < ke) || (kf == ke && (long long)s_lkey[q][SEL_CAP + f] < je);
      }
      if (less == r && n0 + q < N) {
        sel_v[n0 + q] = ke;
        sel_jcut[n0 + q] = je + 1;      // (key, j) <= (v*, j*) are in
        sel_rank0[n0 + q] = (long long)s_rank0[q];
      }
    }
  }
}

// k-NN selection for PB particles per block: MSD radix select (8 passes of
// 8 bits; usually 2 passes + one collecting sweep) of the rank nq-1 squared
// distance, every streamed row X[j] shared by
// the block's PB particles (PB x less L2 traffic than one particle per block).
// Writes, per particle, the key v* of rank nq-1, how many keys equal to v*
// are inside the k+1 nearest (ties taken by index), and the rank-0 index (the
// smallest index at distance 0, dropped like indices[n, 1:] in the reference).
template <int D, int PB>
__global__ __launch_bounds__(256) void local_select_kernel(
    const double* __restrict__ X, int64_t N, int64_t nq,
    unsigned long long* __restrict__ sel_v, long long* __restrict__ sel_jcut,
    long long* __restrict__ sel_rank0, const int* __restrict__ need) {
  __shared__ unsigned hist[PB][BR_NB];
  __shared__ long long s_tot[PB];
  __shared__ int s_cnt[4];
  __shared__ double xn[PB][D];
  __shared__ unsigned long long s_prefix[PB], s_rank0[PB];
  __shared__ long long s_rank[PB];
  // the rank bucket's (key, index) list; before the passes the same LDS holds
  // the sorted distance sample of each particle
  __shared__ unsigned long long s_buf[PB][2 * SEL_CAP];
  __shared__ int s_lcnt[PB];
  __shared__ int s_sh[PB];
  __shared__ unsigned long long s_below[PB];
  __shared__ int s_fail;
  unsigned long long (*s_lkey)[2 * SEL_CAP] = s_buf;
  const int tid = threadIdx.x;
  const int64_t n0 = (int64_t)blockIdx.x * PB;
  if (need) {
    // re-selection of the particles knn_select_kernel flagged: blocks
    // without one exit at once
    bool any = false;
    for (int p = 0; p < PB && n0 + p < N; ++p) any = any || need[n0 + p] != 0;
    if (!any) return;
  }
  for (int e = tid; e < PB * D; e += 256) {
    const int p = e / D, q = e % D;
    const int64_t n = n0 + p < N ? n0 + p : N - 1;  // pad: duplicate, not written
    xn[p][q] = X[n * D + q];
  }
  if (tid < PB) { s_rank0[tid] = (unsigned long long)N; }
  if (tid == 0) s_fail = 0;
  __syncthreads();
  double xr[PB][D];  // the block's particles in registers (no LDS reads per pair)
#pragma unroll
  for (int p = 0; p < PB; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) xr[p][q] = xn[p][q];
  if (N >= 4 * BR_SK) {
    // ---- sample bracketing: BR_SK evenly spaced rows give each particle a
    // sorted distance sample; the sample order statistics BR_M places either
    // side of the rank bound a key window [lo, hi].  ONE sweep then counts the
    // keys below the window and histograms the window on the ~9 bits below
    // the top bit of hi - lo (BR_NB bins, offsets from lo); the bin holding
    // the rank is collected in a second sweep and selected in LDS.  Two
    // sweeps instead of 3-4 radix sweeps; the histogram atomics see only the
    // window.  If the rank is outside the window or its bin overflows the
    // LDS list, the full radix select below runs instead.
    for (int q = tid; q < BR_SK; q += 256) {
      const int64_t j = ((2 * (int64_t)q + 1) * N) / (2 * BR_SK);
      double xj[D];
#pragma unroll
      for (int c = 0; c < D; ++c) xj[c] = X[j * D + c];
#pragma unroll
      for (int p = 0; p < PB; ++p)
        s_buf[p][q] = (unsigned long long)__double_as_longlong(dist2v<D>(xj, xr[p]));
    }
    __syncthreads();
    for (int size = 2; size <= BR_SK; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int e = tid; e < PB * (BR_SK / 2); e += 256) {
          const int p = e / (BR_SK / 2), t = e % (BR_SK / 2);
          const int i = 2 * t - (t & (stride - 1)), j = i + stride;
          const bool asc = (i & size) == 0;
          const unsigned long long a = s_buf[p][i], b = s_buf[p][j];
          if ((a > b) == asc) { s_buf[p][i] = b; s_buf[p][j] = a; }
        }
        __syncthreads();
      }
    const double pf = (double)(nq - 1) / (double)N;
    const int64_t mrg = 8 + (int64_t)(5.0 * sqrt(BR_SK * pf * (1.0 - pf)));
    const int64_t jk = ((nq - 1) * BR_SK) / N;
    unsigned long long lo_r[PB];
    int sh_r[PB];
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      // a rank below the sample's reach (small k): the window starts 2^-12 x
      // the smallest sampled distance (squared distances are >= 0, so key
      // minus 12 << 52 divides by 4096), not at 0 -- starting at 0 would
      // bin the window by exponent only and overflow the bucket list
      const unsigned long long s0 = s_buf[p][0];
      const unsigned long long lo =
          jk - mrg >= 0 ? s_buf[p][jk - mrg]
                        : (s0 > (12ull << 52) ? s0 - (12ull << 52) : 0ull);
      const unsigned long long hi = jk + mrg >= BR_SK ? ~0ull : s_buf[p][jk + mrg];
      const int L = hi > lo ? 64 - __builtin_clzll(hi - lo) : 0;
      sh_r[p] = L > 9 ? L - 9 : 0;   // (hi >> sh) - (lo >> sh) <= 512 < BR_NB
      lo_r[p] = lo >> sh_r[p];
    }
    __syncthreads();  // sample reads done; s_buf becomes the bucket list
    for (int e = tid; e < PB * BR_NB; e += 256) (&hist[0][0])[e] = 0u;
    if (tid < PB) { s_below[tid] = 0ull; s_sh[tid] = sh_r[tid]; }
    __syncthreads();
    unsigned below[PB];
#pragma unroll
    for (int p = 0; p < PB; ++p) below[p] = 0u;
    for (int64_t j = tid; j < N; j += 256) {
      double xj[D];
#pragma unroll
      for (int q = 0; q < D; ++q) xj[q] = X[j * D + q];
#pragma unroll
      for (int p = 0; p < PB; ++p) {
        const unsigned long long key =
            (unsigned long long)__double_as_longlong(dist2v<D>(xj, xr[p]));
        const unsigned long long top = key >> sh_r[p];
        if (top < lo_r[p]) ++below[p];
        else if (top - lo_r[p] < (unsigned long long)BR_NB)
          atomicAdd(&hist[p][top - lo_r[p]], 1u);
        if (key == 0ull) atomicMin(&s_rank0[p], (unsigned long long)j);
      }
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      unsigned v = below[p];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
      if ((tid & 63) == 0 && v) atomicAdd(&s_below[p], (unsigned long long)v);
    }
    __syncthreads();
    {
      // bin holding the rank: 32 lanes per particle, BR_PER bins per lane
      const int p = tid >> 5, l = tid & 31;
      if (p < PB) {
        const long long r = nq - 1 - (long long)s_below[p];
        long long v = 0;
        for (int b = l * BR_PER; b < (l + 1) * BR_PER && b < BR_NB; ++b) v += hist[p][b];
        long long inc = v;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const long long u = __shfl_up(inc, o, 32);
          if (l >= o) inc += u;
        }
        const long long tot = __shfl(inc, 31, 32);
        if (r < 0 || r >= tot) {
          if (l == 0) s_fail = 1;
        } else if (r >= inc - v && r < inc) {
          long long run = inc - v;
          int b = l * BR_PER;
          for (; b < BR_NB; ++b) {
            if (r < run + (long long)hist[p][b]) break;
            run += hist[p][b];
          }
          if (hist[p][b] > (unsigned)SEL_CAP) s_fail = 1;
          s_prefix[p] = lo_r[p] + (unsigned long long)b;
          s_rank[p] = r - run;
        }
      }
    }
    __syncthreads();
    if (!s_fail) {
      collect_select<D, PB>(X, N, n0, xr, s_sh, s_prefix, s_rank, s_rank0, s_lkey,
                            s_lcnt, sel_v, sel_jcut, sel_rank0);
      return;
    }
    __syncthreads();
  }
  if (tid < PB) { s_prefix[tid] = 0ull; s_rank[tid] = nq - 1; s_rank0[tid] = (unsigned long long)N; }
  __syncthreads();
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    for (int e = tid; e < PB * BR_NB; e += 256) (&hist[0][0])[e] = 0u;
    unsigned long long pre[PB];
#pragma unroll
    for (int p = 0; p < PB; ++p) pre[p] = s_prefix[p];
    __syncthreads();
    for (int64_t j = tid; j < N; j += 256) {
      double xj[D];
#pragma unroll
      for (int q = 0; q < D; ++q) xj[q] = X[j * D + q];
#pragma unroll
      for (int p = 0; p < PB; ++p) {
        const unsigned long long key =
            (unsigned long long)__double_as_longlong(dist2v<D>(xj, xr[p]));
        const bool match = (pass == 0) || ((key >> (shift + 8)) == pre[p]);
        if (match) atomicAdd(&hist[p][(key >> shift) & 255ull], 1u);
        if (pass == 0 && key == 0ull) atomicMin(&s_rank0[p], (unsigned long long)j);
      }
    }
    __syncthreads();
    if (tid < PB) {
      long long r = s_rank[tid];
      int b = 0;
      for (; b < 256; ++b) {
        if (r < (long long)hist[tid][b]) break;
        r -= hist[tid][b];
      }
      s_rank[tid] = r;
      s_prefix[tid] = (pre[tid] << 8) | (unsigned long long)b;
      s_tot[tid] = hist[tid][b];  // last pass: number of keys equal to v*
    }
    __syncthreads();
    if (pass >= 1 && pass < 7) {
      // Once the bucket holding rank nq-1 is small (its size is s_tot; after
      // 16 bits for small k, 24 bits for k = N/4), collect its (key, j) pairs
      // in one more sweep and select the rank by (key, index) order in LDS:
      // 3-4 sweeps instead of 8.  Larger buckets take another radix pass.
      bool fits = true;
#pragma unroll
      for (int q = 0; q < PB; ++q) fits = fits && (s_tot[q] <= SEL_CAP);
      if (fits) {
        if (tid < PB) s_sh[tid] = shift;
        __syncthreads();
        collect_select<D, PB>(X, N, n0, xr, s_sh, s_prefix, s_rank, s_rank0, s_lkey,
                              s_lcnt, sel_v, sel_jcut, sel_rank0);
        return;
      }
    }
  }
  // keys equal to v* enter in index order: ties_in = s_rank + 1 of s_tot.  If
  // not all of them do, find the index cutoff with an ordered sweep (rare:
  // only duplicated distances)
  for (int p = 0; p < PB; ++p) {
    const long long ties_in = s_rank[p] + 1;
    long long jcut = N;
    if (ties_in < s_tot[p]) {
      const unsigned long long vs = s_prefix[p];
      long long seen = 0;
      jcut = -1;
      for (int64_t c0 = 0; c0 < N && jcut < 0; c0 += 256) {
        const int64_t j = c0 + tid;
        double xj[D];
#pragma unroll
        for (int q = 0; q < D; ++q) xj[q] = j < N ? X[j * D + q] : 0.0;
        const bool tie = j < N &&
            (unsigned long long)__double_as_longlong(dist2v<D>(xj, xn[p])) == vs;
        const unsigned long long bal = __ballot(tie);
        const int lane = tid & 63, wv = tid >> 6;
        if (lane == 0) s_cnt[wv] = __popcll(bal);
        __syncthreads();
        int before = __popcll(bal & ((1ull << lane) - 1ull)), total = 0;
        for (int t = 0; t < 4; ++t) { const int v = s_cnt[t]; if (t < wv) before += v; total += v; }
        // the ties_in-th tie (0-based ties_in - 1) sets the cutoff
        if (tie && seen + before == ties_in - 1) s_rank[p] = j + 1;
        __syncthreads();
        seen += total;
        if (seen >= ties_in) jcut = s_rank[p];
        __syncthreads();
      }
    }
    if (tid == 0 && n0 + p < N) {
      sel_v[n0 + p] = s_prefix[p];
      sel_jcut[n0 + p] = jcut;
      sel_rank0[n0 + p] = (long long)s_rank0[p];
    }
  }
}

// Covariance of the selected neighbours, one particle per lane: every row
// X[j] is wave-uniform (scalar loads, shared by the wave's 64 particles), the
// per-pair work is the distance, the membership test (key < v*, or key == v*
// and j < jcut; the rank-0 index excluded) and, for members, the moments
// (sum a, sum a^2, sum a d, upper triangle of sum a d d^T with a the
// neighbour's weight) in the lane's registers.  The rows are split into RS
// chunks (grid.y) for occupancy; the partial moments go to part[RS][NM][N]
// and local_finish_kernel adds them in chunk order (deterministic).  Above
// d = 8 the NM moments no longer fit one lane's registers: the kernel is
// instantiated per slice SL of MSLICE moments (the distance and membership
// test are recomputed per slice; the same bits).
constexpr int MSLICE = 48;
template <int D> constexpr int local_nm() { return 2 + D + D * (D + 1) / 2; }
template <int D> constexpr int local_nslices() { return (local_nm<D>() + MSLICE - 1) / MSLICE; }

template <int D, int SL>
__global__ __launch_bounds__(256) void local_moments_kernel(
    const double* __restrict__ X, const float* __restrict__ X32,
    const double* __restrict__ Mp, const double* __restrict__ w, int64_t N,
    const unsigned long long* __restrict__ sel_v,
    const long long* __restrict__ sel_jcut,
    const long long* __restrict__ sel_rank0, double* __restrict__ part,
    const int* __restrict__ done) {
  constexpr int NM = local_nm<D>();
  constexpr int C0 = SL * MSLICE;
  constexpr int C1 = C0 + MSLICE < NM ? C0 + MSLICE : NM;
  constexpr int NS = C1 - C0;
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t ne = n < N ? n : N - 1;
  // particles whose moments knn_select_kernel already summed (list mode):
  // a wave with none left exits
  if (done && __builtin_amdgcn_ballot_w64(n < N && !done[ne]) == 0ull) return;
  const int RS = gridDim.y;
  const int64_t j0 = (N * (int64_t)blockIdx.y) / RS, j1 = (N * ((int64_t)blockIdx.y + 1)) / RS;
  double xp[D];
#pragma unroll
  for (int q = 0; q < D; ++q) xp[q] = X[ne * D + q];
  const unsigned long long vs = sel_v[ne];
  const long long jcut = sel_jcut[ne], r0 = sel_rank0[ne];
  float xp32[D];
#pragma unroll
  for (int q = 0; q < D; ++q) xp32[q] = X32[ne * D + q];
  // fp32 prefilter of the membership test key <= v* (see f32_bound)
  const double M = *Mp;
  const float cut_in = f32_cut_below<D>(key_val(vs), M);   // s32 < cut_in: member
  const float cut_out = f32_cut_above<D>(key_val(vs), M);  // s32 > cut_out: not one
  double m[NS];
#pragma unroll
  for (int t = 0; t < NS; ++t) m[t] = 0.0;
  auto row = [&](int64_t j, const float (&xj32)[D]) {
    const float s32 = dist2f<D>(xj32, xp32);
    if (s32 > cut_out) return;
    bool member;
    double xj[D];
#pragma unroll
    for (int q = 0; q < D; ++q) xj[q] = X[j * D + q];
    if (s32 < cut_in && s32 > 0.0f) {
      member = true;
    } else {
      const unsigned long long key = (unsigned long long)__double_as_longlong(dist2v<D>(xj, xp));
      member = key < vs || (key == vs && j < jcut);
    }
    if (member && j != r0) {
      const double lw = w[j];
      double dj[D];
#pragma unroll
      for (int q = 0; q < D; ++q) dj[q] = xj[q] - xp[q];
      if (0 >= C0 && 0 < C1) m[0 - C0] += lw;
      if (1 >= C0 && 1 < C1) m[1 - C0] += lw * lw;
      int c = 2 + D;
#pragma unroll
      for (int a = 0; a < D; ++a) {
        if (2 + a >= C0 && 2 + a < C1) m[2 + a - C0] += lw * dj[a];
#pragma unroll
        for (int b = a; b < D; ++b) {
          if (c >= C0 && c < C1) m[c - C0] += lw * dj[a] * dj[b];
          ++c;
        }
      }
    }
  };
  // 8 rows per step: their (scalar) fp32 loads issue together, then the
  // pairs; the fp64 row is loaded only for pairs the prefilter leaves open
  constexpr int RU = D <= 8 ? 8 : 4;
  int64_t j = j0;
  for (; j + RU <= j1; j += RU) {
    float xa[RU][D];
#pragma unroll
    for (int u = 0; u < RU; ++u)
#pragma unroll
      for (int q = 0; q < D; ++q) xa[u][q] = X32[(j + u) * D + q];
#pragma unroll
    for (int u = 0; u < RU; ++u) row(j + u, xa[u]);
  }
  for (; j < j1; ++j) {
    float xj[D];
#pragma unroll
    for (int q = 0; q < D; ++q) xj[q] = X32[j * D + q];
    row(j, xj);
  }
  if (n < N) {
#pragma unroll
    for (int t = 0; t < NS; ++t) part[((int64_t)blockIdx.y * NM + C0 + t) * N + n] = m[t];
  }
}

// Per particle: the moments (partials added in chunk order), then the
// reference's fix-ups and factorisations (local_transition.py:112-139).
template <int D>
__global__ __launch_bounds__(256) void local_finish_kernel(
    const double* __restrict__ X, int64_t N, int64_t nq, double scaling, double eps,
    const double* __restrict__ part, int RS, double* __restrict__ covs,
    double* __restrict__ invs, double* __restrict__ dets,
    double* __restrict__ chol, double* __restrict__ lnorm,
    const int* __restrict__ done, const double* __restrict__ lmom) {
  constexpr int NM = local_nm<D>();
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const bool listed = done && done[n];   // moments summed by knn_select_kernel
  double cov[D][D];
  if (N == 1) {
    // indices is 1-D -> deltas = |X|, one sample -> diag(|X[0]|)
    for (int a = 0; a < D; ++a)
      for (int b = 0; b < D; ++b) cov[a][b] = (a == b) ? fabs(X[a]) : 0.0;
  } else {
    double M[NM];
    for (int t = 0; t < NM; ++t) {
      double v = 0.0;
      if (listed) v = lmom[(int64_t)t * N + n];
      else
        for (int y = 0; y < RS; ++y) v += part[((int64_t)y * NM + t) * N + n];
      M[t] = v;
    }
    double S2[D][D];
    {
      int c = 2 + D;
      for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) { S2[a][b] = M[c]; S2[b][a] = M[c]; ++c; }
    }
    const long long nnb = nq - 1;
    if (nnb == 1) {
      // one neighbour: smart_cov -> diag(|delta|); delta = sum lw d / lw
      for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) cov[a][b] = (a == b) ? fabs(M[2 + a] / M[0]) : 0.0;
    } else {
      // np.cov(deltas, aweights=a), a = lw / sum lw:
      // sum a (d - dbar)(d - dbar)^T / (1 - sum a^2)
      const double sw = M[0];
      const double sa2 = M[1] / (sw * sw);
      double mean[D];
      for (int a = 0; a < D; ++a) mean[a] = M[2 + a] / sw;
      for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b)
          cov[a][b] = (S2[a][b] / sw - mean[a] * mean[b]) / (1.0 - sa2);
    }
  }
  double csum = 0.0;
  for (int a = 0; a < D; ++a)
    for (int b = 0; b < D; ++b) csum += cov[a][b];
  if (fabs(csum) == 0.0)
    for (int a = 0; a < D; ++a) cov[a][a] = fabs(X[a]);  // X[0, a]
  for (int a = 0; a < D; ++a)
    for (int b = 0; b < D; ++b) cov[a][b] *= scaling;
  double lu[D][D];
  int perm[D];
  double det;
  for (int it = 0;; ++it) {
    for (int a = 0; a < D; ++a)
      for (int b = 0; b < D; ++b) lu[a][b] = cov[a][b];
    det = lu_factor<D>(lu, perm);
    if (!(det <= 0.0) || it >= 1000000) break;  // NaN exits, as "while det <= 0" does
    for (int a = 0; a < D; ++a) cov[a][a] += eps;
  }
  double inv[D][D], L[D][D];
  lu_inverse<D>(lu, perm, inv);
  cholesky<D>(cov, L);
  for (int a = 0; a < D; ++a)
    for (int b = 0; b < D; ++b) {
      covs[n * D * D + a * D + b] = cov[a][b];
      invs[n * D * D + a * D + b] = inv[a][b];
      chol[n * D * D + a * D + b] = L[a][b];
    }
  dets[n] = det;
  lnorm[n] = 0.5 * (D * LOG_2PI + log(det));
}

// row chunks of the moments kernel: ~8 waves per SIMD, >= 64 rows a chunk
inline int moments_chunks(int64_t N) {
  const int64_t waves = (N + 63) / 64;
  int64_t rs = (8192 + waves - 1) / waves;
  const int64_t cap = N / 64 > 1 ? N / 64 : 1;
  if (rs > cap) rs = cap;
  if (rs > 32) rs = 32;
  return (int)(rs < 1 ? 1 : rs);
}

// ---- dense neighbourhoods: the moments on f16 MFMA with exact limbs --------
// At k a sizeable fraction of N (the default k = N/4) a quarter of all pairs
// are members and local_moments_kernel runs its fp64 update for every row
// (some lane of the wave is always a member).  Here the raw sums
//   S_n,f = sum_j m_nj F_j,f,  F_j = [w, w^2, w Y_a, w Y_a Y_b (a <= b)],
//   Y = X - X_0,  m the 0/1 membership of local_moments_kernel (same fp32
//   prefilter and exact fp64 test)
// are a [particles x rows] x [rows x features] product.  Each feature column
// f is split into ML_NL = 5 limbs of 11 bits on a block exponent e_f (|F_f| <
// 2^e_f from the population's max w and max |Y_a|): F = sum_l L_l 2^(e_f -
// 11 (l + 1)), L_l integers with |L_l| <= 2048, exact f16.  Products m L are
// exact and f32 sums of at most 8192 of them stay below 2^24, so the MFMA's
// f32 accumulation is exact; every 256 steps (8192 rows) the sums are added
// into fp64 partials (integers, exact).  The only rounding is the last
// limb's (2^(e_f - 56) per term) and the fp64 re-centring at X_n
// (mm_finish_kernel), whose error bound is checked per particle against the
// local variance: a particle that fails it sends the whole fit back to the
// VALU kernel (a device flag read by the host; never seen on the tests'
// populations).
constexpr int ML_NL = 5;
template <int D> constexpr int mm_nc() { return local_nm<D>() * ML_NL; }
template <int D> constexpr int mm_nt() { return (mm_nc<D>() + 15) / 16; }
constexpr double MM_EPS = 2.220446049250313e-16;  // fp64 epsilon
constexpr int MM_FLUSH = 256;   // 32-row steps between fp64 flushes (8192 rows)
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// feature f of a row with weight lw and offsets y (local_nm order)
template <int D>
__device__ __forceinline__ double mm_feature(int f, double lw, const double (&y)[D]) {
  if (f == 0) return lw;
  if (f == 1) return lw * lw;
  if (f < 2 + D) return lw * y[f - 2];
  int c = 2 + D;
#pragma unroll
  for (int a = 0; a < D; ++a)
#pragma unroll
    for (int b = a; b < D; ++b) {
      if (c == f) return lw * y[a] * y[b];
      ++c;
    }
  return 0.0;
}

// block exponent of feature f: |F_f| <= bound < 2^e (bnd = [max w, max |Y_a|])
template <int D>
__device__ __forceinline__ int mm_fexp(int f, const double* bnd) {
  double y[D];
#pragma unroll
  for (int a = 0; a < D; ++a) y[a] = bnd[1 + a];
  const double b = mm_feature<D>(f, bnd[0], y);
  if (!(b > 0.0)) return 0;
  int e;
  frexp(b, &e);
  return e;
}

// limb l of v on the block exponent e (integer-valued, |.| <= 2048)
__device__ __forceinline__ double mm_limb(double v, int e, int l) {
  double r = ldexp(v, 11 - e);
  double L = rint(r);
  for (int q = 0; q < l; ++q) {
    r = ldexp(r - L, 11);
    L = rint(r);
  }
  return L;
}

// bnd[0] = max w, bnd[1 + a] = max |X_a - X_0a| (bit patterns of non-negative
// doubles are monotone: atomicMax on them; bnd zeroed by the caller)
template <int D>
__global__ __launch_bounds__(256) void mm_bounds_kernel(const double* __restrict__ X,
                                                        const double* __restrict__ w,
                                                        int64_t N,
                                                        unsigned long long* __restrict__ bnd) {
  double m[1 + D];
#pragma unroll
  for (int a = 0; a <= D; ++a) m[a] = 0.0;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < N;
       j += (int64_t)gridDim.x * 256) {
    m[0] = fmax(m[0], fabs(w[j]));
#pragma unroll
    for (int a = 0; a < D; ++a) m[1 + a] = fmax(m[1 + a], fabs(X[j * D + a] - X[a]));
  }
#pragma unroll
  for (int a = 0; a <= D; ++a) {
    const double v = wave_max(m[a]);
    if ((threadIdx.x & 63) == 0 && v > 0.0)
      atomicMax(bnd + a, (unsigned long long)__double_as_longlong(v));
  }
}

// B operand image [step][tile][lane][8 halves]: lane l of tile t holds rows
// 32 s + 8 (l >> 4) + 0..7 of column 16 t + (l & 15) = f * ML_NL + limb
template <int D>
__global__ __launch_bounds__(256) void mm_bimg_kernel(const double* __restrict__ X,
                                                      const double* __restrict__ w,
                                                      int64_t N, int64_t nsteps,
                                                      const double* __restrict__ bnd,
                                                      half8* __restrict__ img) {
  constexpr int NT = mm_nt<D>(), NC = mm_nc<D>();
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= nsteps * NT * 64) return;
  const int lane = (int)(g & 63);
  const int64_t st = g >> 6;
  const int t = (int)(st % NT);
  const int64_t s = st / NT;
  const int c = 16 * t + (lane & 15);
  half8 h;
  if (c >= NC) {
#pragma unroll
    for (int u = 0; u < 8; ++u) h[u] = (_Float16)0.0f;
  } else {
    const int f = c / ML_NL, l = c % ML_NL;
    const int e = mm_fexp<D>(f, bnd);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t j = 32 * s + 8 * (lane >> 4) + u;
      double v = 0.0;
      if (j < N) {
        double y[D];
#pragma unroll
        for (int a = 0; a < D; ++a) y[a] = X[j * D + a] - X[a];
        v = mm_limb(mm_feature<D>(f, w[j], y), e, l);
      }
      h[u] = (_Float16)(float)v;
    }
  }
  img[g] = h;
}

// Block = 8 waves x MM_G particle tiles of 16 (256 particles); a wave's tiles
// share each B fragment, and the block stages MM_SB steps of the B image and
// of the rows' fp32 coordinates in LDS (the image is ~14x the bytes of the
// rows: every particle group re-reads it).  grid (ceil(N / 256), RS row
// chunks of whole 32-row steps); part [RS][16 NT][N] (exact integer sums).
constexpr int MM_G = 2, MM_W = 8, MM_SB = 4;
constexpr int MM_T = MM_W * 64;          // threads per block
constexpr int MM_PB = MM_W * MM_G * 16;   // particles per block
template <int D>
__global__ __launch_bounds__(MM_T) void mm_moments_kernel(
    const double* __restrict__ X, const float* __restrict__ X32,
    const double* __restrict__ Mp, const half8* __restrict__ img, int64_t N,
    int64_t nsteps, const unsigned long long* __restrict__ sel_v,
    const long long* __restrict__ sel_jcut, const long long* __restrict__ sel_rank0,
    double* __restrict__ part) {
  constexpr int NT = mm_nt<D>(), NCP = 16 * NT;
  __shared__ half8 bs[MM_SB * NT * 64];
  __shared__ float xs[MM_SB * 32 * D];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int RS = gridDim.y;
  const int64_t s0 = (nsteps * (int64_t)blockIdx.y) / RS;
  const int64_t s1 = (nsteps * ((int64_t)blockIdx.y + 1)) / RS;
  const int64_t p0 = ((int64_t)blockIdx.x * MM_W + wv) * (MM_G * 16);
  const int kq = lane >> 4;
  const double M = *Mp;
  float xp32[MM_G][D];
  unsigned long long vs[MM_G];
  long long jcut[MM_G], r0[MM_G];
  float cut_in[MM_G], cut_out[MM_G];
#pragma unroll
  for (int g = 0; g < MM_G; ++g) {
    const int64_t pn = p0 + 16 * g + (lane & 15);
    const int64_t pe = pn < N ? pn : N - 1;
#pragma unroll
    for (int q = 0; q < D; ++q) xp32[g][q] = X32[pe * D + q];
    vs[g] = sel_v[pe];
    jcut[g] = sel_jcut[pe];
    r0[g] = sel_rank0[pe];
    cut_in[g] = f32_cut_below<D>(key_val(vs[g]), M);
    cut_out[g] = f32_cut_above<D>(key_val(vs[g]), M);
  }
  static_assert(MM_G == 2, "packed distances pair the two tiles");
  f32x2 xp2[D];
#pragma unroll
  for (int q = 0; q < D; ++q) xp2[q] = f32x2{xp32[0][q], xp32[1][q]};
  f32x4 acc[MM_G][NT];
#pragma unroll
  for (int g = 0; g < MM_G; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool first = true;
  int since = 0;
  auto flush = [&]() {
#pragma unroll
    for (int g = 0; g < MM_G; ++g)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int c = 16 * t + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t n = p0 + 16 * g + 4 * kq + r;
          if (n < N) {
            double* dst = part + ((int64_t)blockIdx.y * NCP + c) * N + n;
            *dst = (first ? 0.0 : *dst) + (double)acc[g][t][r];
          }
        }
        acc[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    first = false;
    since = 0;
  };
  // The next stage's B fragments and rows are loaded into registers while
  // the current one computes (one block per CU at this register count, so a
  // synchronous stage would idle the CU for a full HBM/L2 round trip).
  constexpr int PF = (MM_SB * NT * 64 + MM_T - 1) / MM_T, PFX = (MM_SB * 32 * D + MM_T - 1) / MM_T;
  half8 pf[PF];
  float pfx[PFX];
  auto fetch = [&](int64_t sb) {
    const int nk = (int)((s1 - sb) < MM_SB ? (s1 - sb) : MM_SB);
    const int64_t jb = 32 * sb;
    const int64_t cnt = ((N - jb) < MM_SB * 32 ? (N - jb) : MM_SB * 32) * D;
#pragma unroll
    for (int i = 0; i < PFX; ++i) {
      const int e = threadIdx.x + MM_T * i;
      pfx[i] = e < cnt ? X32[jb * D + e] : 0.0f;
    }
    const half8* src = img + sb * NT * 64;
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = threadIdx.x + MM_T * i;
      if (e < nk * NT * 64) pf[i] = src[e];
    }
  };
  if (s0 < s1) fetch(s0);
  for (int64_t sb = s0; sb < s1; sb += MM_SB) {
    const int nk = (int)((s1 - sb) < MM_SB ? (s1 - sb) : MM_SB);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PFX; ++i) {
      const int e = threadIdx.x + MM_T * i;
      if (e < MM_SB * 32 * D) xs[e] = pfx[i];
    }
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = threadIdx.x + MM_T * i;
      if (e < nk * NT * 64) bs[e] = pf[i];
    }
    __syncthreads();
    if (sb + MM_SB < s1) fetch(sb + MM_SB);
    for (int k = 0; k < nk; ++k) {
      // fp32 prefilter of the 8 x MM_G pairs without branches; pairs between
      // the cuts (and distance 0: duplicates, the particle itself) go to the
      // exact fp64 test below, entered when any lane of the wave has one
      // (rows past N have zero features, so their bits do not matter; the
      // excluded rank-0 row has distance 0 and always takes the exact test).
      // The two tiles' distances run as packed f32 pairs (the same sub / fma
      // per element as dist2f, so the same bits).
      half8 a[MM_G];
      bool anyopen = false;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rl = 32 * k + 8 * kq + u;
        const bool inN = 32 * sb + rl < N;
        f32x2 s2 = f32x2{0.f, 0.f};
#pragma unroll
        for (int q = 0; q < D; ++q) {
          const float xq = xs[rl * D + q];
          const f32x2 t = f32x2{xq, xq} - xp2[q];
          s2 = __builtin_elementwise_fma(t, t, s2);
        }
#pragma unroll
        for (int g = 0; g < MM_G; ++g) {
          const float s32 = s2[g];
          const bool in = s32 < cut_in[g] && s32 > 0.0f;
          anyopen |= !in && !(s32 > cut_out[g]) && inN;
          a[g][u] = in ? (_Float16)1.0f : (_Float16)0.0f;
        }
      }
      if (__ballot(anyopen)) {
        // rare: redo the prefilter per pair and settle the open ones in fp64
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int rl = 32 * k + 8 * kq + u;
          const int64_t j = 32 * sb + rl;
#pragma unroll
          for (int g = 0; g < MM_G; ++g) {
            float xj32[D];
#pragma unroll
            for (int q = 0; q < D; ++q) xj32[q] = xs[rl * D + q];
            const float s32 = dist2f<D>(xj32, xp32[g]);
            const bool in = s32 < cut_in[g] && s32 > 0.0f;
            if (!in && !(s32 > cut_out[g]) && j < N) {
              const int64_t pn = p0 + 16 * g + (lane & 15);
              const int64_t pe = pn < N ? pn : N - 1;
              double xj[D], xp[D];
#pragma unroll
              for (int q = 0; q < D; ++q) { xj[q] = X[j * D + q]; xp[q] = X[pe * D + q]; }
              const unsigned long long key =
                  (unsigned long long)__double_as_longlong(dist2v<D>(xj, xp));
              const bool member = key < vs[g] || (key == vs[g] && j < jcut[g]);
              a[g][u] = (member && j != r0[g]) ? (_Float16)1.0f : (_Float16)0.0f;
            }
          }
        }
      }
      const half8* b = bs + k * NT * 64 + lane;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const half8 bt = b[t * 64];
#pragma unroll
        for (int g = 0; g < MM_G; ++g)
          acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[g], bt, acc[g][t], 0, 0, 0);
      }
      if (++since == MM_FLUSH) flush();
    }
  }
  if (since > 0 || first) flush();
}

// limbs + chunks -> raw sums -> moments centred at X_n in local_finish's
// layout [NM][N]; flags a particle whose rounding bound is not far below its
// local variance
template <int D>
__global__ __launch_bounds__(256) void mm_finish_kernel(const double* __restrict__ X, int64_t N,
                                                        int64_t nq,
                                                        const double* __restrict__ part,
                                                        int RS, const double* __restrict__ bnd,
                                                        double* __restrict__ out,
                                                        int* __restrict__ flag,
                                                        const double* __restrict__ extra) {
  constexpr int NM = local_nm<D>(), NCP = 16 * mm_nt<D>();
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  double S[NM], E[NM];
  for (int f = 0; f < NM; ++f) {
    const int e = mm_fexp<D>(f, bnd);
    double v = 0.0;
    for (int l = ML_NL - 1; l >= 0; --l) {   // smallest limb first
      double c = 0.0;
      for (int y = 0; y < RS; ++y) c += part[((int64_t)y * NCP + f * ML_NL + l) * N + n];
      v += ldexp(c, e - 11 * (l + 1));
    }
    double eq = 0.0;
    if (extra) {   // deferred collect: the queued members' fp64 sum and its bound
      v += extra[(int64_t)f * N + n];
      eq = MM_EPS * extra[(int64_t)(NM + f) * N + n];
    }
    S[f] = v;
    // last-limb rounding per member + the limb sum's own rounding (+ the
    // queued members' sum)
    E[f] = (double)nq * ldexp(1.0, e - 11 * ML_NL - 1) + 4.0 * MM_EPS * fabs(v) + eq;
  }
  double yn[D];
  for (int a = 0; a < D; ++a) yn[a] = X[n * D + a] - X[a];
  const double S0 = S[0];
  out[0 * N + n] = S0;
  out[1 * N + n] = S[1];
  double m1[D];
  for (int a = 0; a < D; ++a) {
    m1[a] = S[2 + a] - S0 * yn[a];
    out[(int64_t)(2 + a) * N + n] = m1[a];
  }
  bool bad = !(S0 > 0.0);
  int c = 2 + D;
  for (int a = 0; a < D; ++a)
    for (int b = a; b < D; ++b, ++c) {
      const double t1 = S[2 + a] * yn[b], t2 = S[2 + b] * yn[a], t3 = S0 * yn[a] * yn[b];
      const double v = ((S[c] - t1) - t2) + t3;
      out[(int64_t)c * N + n] = v;
      if (a == b) {
        // error of v (absolute) against the local variance about the mean
        const double err = E[c] + E[2 + a] * fabs(yn[b]) + E[2 + b] * fabs(yn[a]) +
                           E[0] * fabs(yn[a] * yn[b]) +
                           8.0 * MM_EPS * (fabs(S[c]) + fabs(t1) + fabs(t2) + fabs(t3));
        const double var = v - m1[a] * m1[a] / S0;
        if (!(err <= 1e-11 * var)) bad = true;
      }
    }
  if (bad) atomicOr(flag, 1);
}

#include "abc_local_dense.h"

inline int mm_chunks(int64_t N, int64_t nsteps) {
  const int64_t nblk = (N + MM_PB - 1) / MM_PB;
  int64_t rs = (1024 + nblk - 1) / nblk;
  if (rs > 8) rs = 8;
  if (rs > nsteps) rs = nsteps;
  return (int)(rs < 1 ? 1 : rs);
}

// particles per selection block (their coordinates in registers)
template <int D> constexpr int sel_pb() { return D <= 8 ? 8 : 4; }

template <int D, int SL>
void launch_moments(const double* X, const float* X32, const double* M, const double* w,
                    int64_t N, const unsigned long long* sel_v, const long long* sel_ties,
                    const long long* sel_rank0, double* part, int RS, hipStream_t s,
                    const int* done = nullptr) {
  hipLaunchKernelGGL((local_moments_kernel<D, SL>), dim3((unsigned)ceil_div(N, 256), (unsigned)RS),
                     dim3(256), 0, s, X, X32, M, w, N, sel_v, sel_ties, sel_rank0, part, done);
  if constexpr (SL + 1 < local_nslices<D>())
    launch_moments<D, SL + 1>(X, X32, M, w, N, sel_v, sel_ties, sel_rank0, part, RS, s, done);
}

template <int D>
int launch_fit(const double* X, const double* w, int64_t N, int64_t nq,
               double scaling, double eps, double* covs, double* inv,
               double* dets, double* chol, double* lnorm, void* ws,
               size_t ws_bytes, hipStream_t s) {
  Carver cv(ws, ws_bytes);
  unsigned long long* sel_v = cv.take<unsigned long long>((size_t)N);
  long long* sel_ties = cv.take<long long>((size_t)N);  // index cutoff of the ties
  long long* sel_rank0 = cv.take<long long>((size_t)N);
  float* X32 = cv.take<float>((size_t)N * D);              // fp32 prefilter copy
  double* Mx = cv.take<double>(1);                          // max |X|
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "local_fit: workspace too small");
  ABC_HIP(hipMemsetAsync(Mx, 0, sizeof(double), s));
  {
    const int64_t nx = N * D;
    const int64_t pb = ceil_div(nx, 256) < 512 ? ceil_div(nx, 256) : 512;
    hipLaunchKernelGGL(local_prep_kernel, dim3((unsigned)pb), dim3(256), 0, s, X, nx, X32,
                       reinterpret_cast<unsigned long long*>(Mx));
    ABC_LAUNCHED();
  }
  constexpr int NM = local_nm<D>();
  // k-NN selection on fp32 MFMA keys (abc_local_knn.h) for N >= KN_MIN_N;
  // small k sums the moments in the same kernel (list mode)
  const bool knn = N >= KN_MIN_N;
  const bool list_ok = knn && kn_list_capable<D>() && nq + KN_MARGIN <= KN_CAP;
  // dense neighbourhoods (k > N / 16, d <= 5; above, the kernel's registers
  // spill): the moments on f16 MFMA
  bool dense = D <= 5 && N >= 64 && nq * 16 > N;
  // dense k after the k-NN select's count sweep: the moments sweep does the
  // collect (deferred collect, abc_local_dense.h) -- one sweep less
  const bool defer = knn && !list_ok && dense;
  int* done = nullptr;
  double* lmom = nullptr;
  double* cen = nullptr;
  unsigned long long* r2 = nullptr;
  int h_cnt[2] = {0, 0};
  int* knn_need = nullptr;
  int* knn_cnt = nullptr;
  float* knn_img = nullptr;
  if (knn) {
    const int64_t nt = ceil_div(N, 16) + KN_PAD;   // + prefetch padding
    cen = cv.take<double>(D);
    float* img = cv.take<float>((size_t)nt * kn_kb<D>() * 64);
    r2 = cv.take<unsigned long long>(1);
    int* need = cv.take<int>((size_t)N);
    done = cv.take<int>((size_t)N);
    int* cnt = cv.take<int>(2);
    lmom = cv.take<double>(kn_list_capable<D>() ? (size_t)NM * N : 1);
    if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "local_fit: workspace too small");
    ABC_HIP(hipMemsetAsync(r2, 0, sizeof(unsigned long long), s));
    ABC_HIP(hipMemsetAsync(cnt, 0, 2 * sizeof(int), s));
    hipLaunchKernelGGL((knn_center_kernel<D>), dim3(1), dim3(1024), 0, s, X, N, cen);
    ABC_LAUNCHED();
    hipLaunchKernelGGL((knn_prep_kernel<D>), dim3((unsigned)ceil_div(nt * 16, 256)), dim3(256), 0,
                       s, X, N, (const double*)cen, img, r2);
    ABC_LAUNCHED();
    knn_need = need;
    knn_img = img;
    knn_cnt = cnt;
    hipLaunchKernelGGL((knn_select_kernel<D>), dim3((unsigned)ceil_div(N, KN_PB)), dim3(256), 0,
                       s, X, w, N, nq, (const double*)cen, (const float*)img,
                       (const double*)r2, (int)list_ok, (int)defer, sel_v, sel_ties, sel_rank0,
                       need, done, lmom, cnt);
    ABC_LAUNCHED();
    // particles whose window missed the rank or whose list overflowed: the
    // fp64 radix select (blocks without such a particle exit at once)
    if (!defer) {
      hipLaunchKernelGGL((local_select_kernel<D, sel_pb<D>()>),
                         dim3((unsigned)ceil_div(N, sel_pb<D>())), dim3(256), 0, s, X, N, nq,
                         sel_v, sel_ties, sel_rank0, (const int*)need);
      ABC_LAUNCHED();
    }
    if (list_ok) {
      // one 8-byte read decides whether any particle still needs a sweep
      ABC_HIP(hipMemcpyAsync(h_cnt, cnt, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
      ABC_HIP(hipStreamSynchronize(s));
    }
  } else if (N > 1) {
    hipLaunchKernelGGL((local_select_kernel<D, sel_pb<D>()>), dim3((unsigned)ceil_div(N, sel_pb<D>())),
                       dim3(256), 0, s, X, N, nq, sel_v, sel_ties, sel_rank0, (const int*)nullptr);
    ABC_LAUNCHED();
  }
  const bool all_listed = list_ok && h_cnt[1] == N;
  const int RS = N > 1 ? moments_chunks(N) : 1;
  // (>= 2 NM N: the dense path's deferred collect keeps its member sums and
  // their rounding bounds there)
  double* part = cv.take<double>(all_listed ? 1 : (size_t)(RS < 2 ? 2 : RS) * NM * (size_t)N);
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "local_fit: workspace too small");
  const double* mom = part;
  int mom_rs = RS;
  if constexpr (D <= 5) if (dense) {
    const int64_t nsteps = ceil_div(N, 32);
    const int RS16 = mm_chunks(N, nsteps);
    unsigned long long* bnd = cv.take<unsigned long long>(1 + D);
    int* flag = cv.take<int>(2);            // [rounding bound missed, deferred-collect failures]
    int* qcnt = cv.take<int>((size_t)N);
    int* cbelow = cv.take<int>((size_t)N);
    int* qidx = cv.take<int>((size_t)N * KN_QCAP);
    // (+ DM_SB steps: knn_dense_kernel's stage loads past the last step)
    half8* img = cv.take<half8>((size_t)(nsteps + DM_SB) * mm_nt<D>() * 64);
    double* part16 = cv.take<double>((size_t)RS16 * 16 * mm_nt<D>() * (size_t)N);
    double* cenm = cv.take<double>((size_t)NM * N);
    float* drows = cv.take<float>((size_t)(nsteps + DM_SB) * dm_rstep<D>());
    if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "local_fit: workspace too small");
    ABC_HIP(hipMemsetAsync(bnd, 0, sizeof(unsigned long long) * (1 + D), s));
    ABC_HIP(hipMemsetAsync(flag, 0, 2 * sizeof(int), s));
    const int64_t bb = ceil_div(N, 256) < 256 ? ceil_div(N, 256) : 256;
    hipLaunchKernelGGL((mm_bounds_kernel<D>), dim3((unsigned)bb), dim3(256), 0, s, X, w, N, bnd);
    ABC_LAUNCHED();
    hipLaunchKernelGGL((mm_bimg_kernel<D>), dim3((unsigned)ceil_div(nsteps * mm_nt<D>() * 64, 256)),
                       dim3(256), 0, s, X, w, N, nsteps, (const double*)bnd, img);
    ABC_LAUNCHED();
    int h_flag = 0;
    bool finished = false;   // mm_finish ran already (deferred collect)
    if (knn) {
      // membership from the centred fp32 keys of the k-NN select
      const int64_t nrows = (nsteps + DM_SB) * 32;
      hipLaunchKernelGGL((knn_rows_kernel<D>), dim3((unsigned)ceil_div(nrows, 256)), dim3(256), 0,
                         s, X, N, nrows, (const double*)cen, drows);
      ABC_LAUNCHED();
      bool plain = !defer;
      if (defer) {
        ABC_HIP(hipMemsetAsync(qcnt, 0, sizeof(int) * N, s));
        ABC_HIP(hipMemsetAsync(cbelow, 0, sizeof(int) * N, s));
        hipLaunchKernelGGL((knn_dense_kernel<D, true>), dim3((unsigned)ceil_div(N, DM_PB), (unsigned)RS16),
                           dim3(DM_T), 0, s, X, (const double*)cen, (const double*)r2,
                           (const float*)drows, (const half8*)img, N, nsteps,
                           (const unsigned long long*)sel_v, (const long long*)sel_ties,
                           (const long long*)sel_rank0, part16, qcnt, qidx, cbelow);
        ABC_LAUNCHED();
        hipLaunchKernelGGL((knn_resolve_kernel<D>), dim3((unsigned)ceil_div(N, 4)), dim3(256), 0, s,
                           X, w, N, nq, (const int*)knn_need, sel_v, sel_ties, sel_rank0,
                           (const int*)qcnt, (const int*)qidx, (const int*)cbelow,
                           (const double*)bnd, part16, part, flag + 1);
        ABC_LAUNCHED();
        hipLaunchKernelGGL((mm_finish_kernel<D>), dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, s,
                           X, N, nq, (const double*)part16, RS16, (const double*)bnd, cenm, flag,
                           (const double*)part);
        ABC_LAUNCHED();
        int h_f[2] = {0, 0};
        ABC_HIP(hipMemcpyAsync(h_f, flag, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
        ABC_HIP(hipStreamSynchronize(s));
        if (h_f[1]) {
          // some particle's bracket or queue failed: the select with its own
          // collect sweep (and the fp64 radix select behind it), then the
          // plain moments sweep
          ABC_HIP(hipMemsetAsync(knn_cnt, 0, 2 * sizeof(int), s));
          ABC_HIP(hipMemsetAsync(flag, 0, 2 * sizeof(int), s));
          hipLaunchKernelGGL((knn_select_kernel<D>), dim3((unsigned)ceil_div(N, KN_PB)), dim3(256),
                             0, s, X, w, N, nq, (const double*)cen, (const float*)knn_img,
                             (const double*)r2, 0, 0, sel_v, sel_ties, sel_rank0, knn_need,
                             done, lmom, knn_cnt);
          ABC_LAUNCHED();
          hipLaunchKernelGGL((local_select_kernel<D, sel_pb<D>()>),
                             dim3((unsigned)ceil_div(N, sel_pb<D>())), dim3(256), 0, s, X, N, nq,
                             sel_v, sel_ties, sel_rank0, (const int*)knn_need);
          ABC_LAUNCHED();
          plain = true;
        } else {
          h_flag = h_f[0];
          finished = true;
        }
      }
      if (plain) {
        hipLaunchKernelGGL((knn_dense_kernel<D, false>), dim3((unsigned)ceil_div(N, DM_PB), (unsigned)RS16),
                           dim3(DM_T), 0, s, X, (const double*)cen, (const double*)r2,
                           (const float*)drows, (const half8*)img, N, nsteps,
                           (const unsigned long long*)sel_v, (const long long*)sel_ties,
                           (const long long*)sel_rank0, part16, nullptr, nullptr, nullptr);
        ABC_LAUNCHED();
      }
    } else {
      hipLaunchKernelGGL((mm_moments_kernel<D>), dim3((unsigned)ceil_div(N, MM_PB), (unsigned)RS16),
                         dim3(MM_T), 0, s, X, (const float*)X32, (const double*)Mx,
                         (const half8*)img, N, nsteps, (const unsigned long long*)sel_v,
                         (const long long*)sel_ties, (const long long*)sel_rank0, part16);
      ABC_LAUNCHED();
    }
    if (!finished) {
      hipLaunchKernelGGL((mm_finish_kernel<D>), dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, s,
                         X, N, nq, (const double*)part16, RS16, (const double*)bnd, cenm, flag,
                         (const double*)nullptr);
      ABC_LAUNCHED();
      ABC_HIP(hipMemcpyAsync(&h_flag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
      ABC_HIP(hipStreamSynchronize(s));
    }
    if (h_flag) {
      dense = false;   // rounding bound not met somewhere: the VALU kernel
    } else {
      mom = cenm;
      mom_rs = 1;
    }
  }
  if (N > 1 && !dense && !all_listed) {
    // (after a partly listed select only the remaining particles' waves run)
    launch_moments<D, 0>(X, X32, Mx, w, N, sel_v, sel_ties, sel_rank0, part, RS, s,
                         list_ok ? (const int*)done : nullptr);
    ABC_LAUNCHED();
  }
  hipLaunchKernelGGL((local_finish_kernel<D>), dim3((unsigned)ceil_div(N, 256)), dim3(256),
                     0, s, X, N, nq, scaling, eps, mom, mom_rs, covs, inv,
                     dets, chol, lnorm, (const int*)(list_ok ? done : nullptr),
                     (const double*)lmom);
  ABC_LAUNCHED();
  return ABC_OK;
}


// ---- density on fp64 MFMA ----------------------------------------------------
// s_ij = log2 of w_j N(x_i; X_j, cov_j) = log2e (c_j - q_ij / 2), c_j =
// log w_j - lnorm_j, q_ij = (X_j - x_i)^T A_j (X_j - x_i), A_j = inv_j.  In
// coordinates centred at X_0 (y = x - X_0, Y_j = X_j - X_0), q is linear in the
// quadratic features of the candidate,
//   phi(y) = [y_a y_b (a <= b), y_a, 1, 0-padding]        (K = 4 * KB)
// with population coefficients
//   psi_j  = log2e * [-(A_ab + A_ba)/2 (a < b) | -A_aa/2,
//                     ((A + A^T) Y_j)_a / 2, c_j - Y_j^T A Y_j / 2]
// so s = psi_j . phi(y_i): a [N x K] x [K x M] GEMM on v_mfma_f64_16x16x4_f64
// (population rows = A operand, candidate columns = B operand), followed by
// the running max / exp2 / sum over j of each candidate column (exp2 on the
// f32 unit, 1e-7 per term).
template <int D>
struct LocalFeat {
  static constexpr int K0 = D * (D + 1) / 2 + D + 1;
  static constexpr int KB = (K0 + 3) / 4;          // MFMA k-blocks of 4
  static constexpr int NT = KB <= 6 ? 4 : (KB <= 16 ? 2 : 1);  // candidate tiles per wave
};

// feature k of centred candidate y (order: a <= b pairs, linear, constant)
template <int D>
__device__ __forceinline__ double local_phi(const double (&y)[D], int k) {
  int q = 0;
#pragma unroll
  for (int a = 0; a < D; ++a)
#pragma unroll
    for (int b = a; b < D; ++b, ++q)
      if (k == q) return y[a] * y[b];
#pragma unroll
  for (int a = 0; a < D; ++a, ++q)
    if (k == q) return y[a];
  return (k == q) ? 1.0 : 0.0;
}

// psi in fragment order [N/16 tiles][KB][64 lanes]: lane l of k-block kb
// holds psi[tile*16 + (l & 15)][4 kb + (l >> 4)] (the A operand of one MFMA).
// Rows j >= N get -inf in the constant slot (they add nothing).
template <int D>
__global__ __launch_bounds__(256) void local_pack_kernel(
    const double* __restrict__ X, const double* __restrict__ w,
    const double* __restrict__ invs, const double* __restrict__ lnorm,
    int64_t N, int64_t ntiles, double* __restrict__ psi) {
  constexpr int KB = LocalFeat<D>::KB;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= ntiles * KB * 64) return;
  const int lane = (int)(e & 63);
  const int kb = (int)((e >> 6) % KB);
  const int64_t tile = (e >> 6) / KB;
  const int64_t j = tile * 16 + (lane & 15);
  const int k = 4 * kb + (lane >> 4);
  double v = 0.0;
  const int K0 = LocalFeat<D>::K0;
  if (j >= N) {
    v = (k == K0 - 1) ? -INFINITY : 0.0;
  } else if (k < K0) {
    const double* A = invs + j * D * D;
    double y[D];
#pragma unroll
    for (int a = 0; a < D; ++a) y[a] = X[j * D + a] - X[a];
    int q = 0;
    bool done = false;
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
      for (int b = a; b < D; ++b, ++q)
        if (k == q) {
          v = (a == b) ? -0.5 * A[a * D + a] : -0.5 * (A[a * D + b] + A[b * D + a]);
          done = true;
        }
    if (!done) {
#pragma unroll
      for (int a = 0; a < D; ++a, ++q)
        if (k == q) {
          double t = 0.0;
#pragma unroll
          for (int b = 0; b < D; ++b) t += (A[a * D + b] + A[b * D + a]) * y[b];
          v = 0.5 * t;
          done = true;
        }
    }
    if (!done) {                      // constant slot
      double qf = 0.0;
#pragma unroll
      for (int a = 0; a < D; ++a) {
        double t = 0.0;
#pragma unroll
        for (int b = 0; b < D; ++b) t += A[a * D + b] * y[b];
        qf += y[a] * t;
      }
      const double wj = w[j];
      const double c = (wj > 0.0) ? log(wj) - lnorm[j] : -INFINITY;
      v = c - 0.5 * qf;
    }
    v *= LOG2E_L;
  }
  psi[e] = v;
}

typedef double f64x4 __attribute__((ext_vector_type(4)));

// grid (candidate blocks of 4 waves x NT x 16, population chunks); each wave
// keeps NT candidate tiles' features in registers and streams its chunk of
// population tiles; writes the (max, sum) partial of each candidate.
template <int D>
__global__ __launch_bounds__(256) void local_mfma_kernel(
    const double* __restrict__ x, int64_t M, const double* __restrict__ X,
    const double* __restrict__ psi, int64_t ntiles, int64_t tiles_per_chunk,
    double2* __restrict__ part) {
  constexpr int KB = LocalFeat<D>::KB, NT = LocalFeat<D>::NT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c0 = ((int64_t)blockIdx.x * 4 + wv) * (NT * 16);
  double phi[NT][KB];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int64_t i = c0 + t * 16 + (lane & 15);
    double y[D];
#pragma unroll
    for (int a = 0; a < D; ++a) y[a] = (i < M) ? x[i * D + a] - X[a] : 0.0;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) phi[t][kb] = local_phi<D>(y, 4 * kb + (lane >> 4));
  }
  double m[NT], l[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) { m[t] = -INFINITY; l[t] = 0.0; }
  const int64_t p0 = (int64_t)blockIdx.y * tiles_per_chunk;
  const int64_t p1 = (p0 + tiles_per_chunk < ntiles) ? p0 + tiles_per_chunk : ntiles;
  for (int64_t pt = p0; pt < p1; ++pt) {
    double a[KB];
    const double* src = psi + pt * (KB * 64) + lane;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) a[kb] = src[kb * 64];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kb], phi[t][kb], acc, 0, 0, 0);
      const double mx = fmax(fmax(acc[0], acc[1]), fmax(acc[2], acc[3]));
      if (mx > m[t]) {
        l[t] *= (double)__builtin_amdgcn_exp2f((float)(m[t] - mx));
        m[t] = mx;
      }
      if (m[t] > -INFINITY) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          l[t] += (double)__builtin_amdgcn_exp2f((float)(acc[r] - m[t]));
      }
    }
  }
  // merge the 4 row groups (lanes l, l^16, l^32, l^48 share a candidate)
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      const double mo = __shfl_xor(m[t], o, 64), lo = __shfl_xor(l[t], o, 64);
      const double mn = fmax(m[t], mo);
      if (mn > -INFINITY) {
        l[t] = l[t] * (double)__builtin_amdgcn_exp2f((float)(m[t] - mn)) +
               lo * (double)__builtin_amdgcn_exp2f((float)(mo - mn));
        m[t] = mn;
      }
    }
    const int64_t i = c0 + t * 16 + (lane & 15);
    if (lane < 16 && i < M) part[(int64_t)blockIdx.y * M + i] = make_double2(m[t], l[t]);
  }
}

// sum of the weights (np.average's denominator) in a fixed order
__global__ __launch_bounds__(1024) void local_wsum_kernel(
    const double* __restrict__ w, int64_t N, double* __restrict__ out) {
  __shared__ double sh[16];
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < N; j += 1024) s += w[j];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += sh[k];
    out[0] = t;
  }
}

__global__ __launch_bounds__(256) void local_combine_kernel(
    const double2* __restrict__ part, int64_t M, int nchunks,
    const double* __restrict__ wsum, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= M) return;
  double m = -INFINITY;
  for (int c = 0; c < nchunks; ++c) m = fmax(m, part[(int64_t)c * M + i].x);
  double l = 0.0;
  if (m > -INFINITY)
    for (int c = 0; c < nchunks; ++c) {
      const double2 p = part[(int64_t)c * M + i];
      if (p.x > -INFINITY) l += p.y * exp2(p.x - m);
    }
  out[i] = (l > 0.0) ? LN2_L * (m + log2(l)) - log(wsum[0]) : -INFINITY;
}

template <int D>
size_t pdf_workspace(int64_t M, int64_t N, int* nchunks_out) {
  const int64_t ntiles = ceil_div(N, 16);
  const int64_t cblocks = ceil_div(M > 0 ? M : 1, 4 * LocalFeat<D>::NT * 16);
  // enough workgroups for 256 CUs x several waves, chunks of >= 64 tiles
  int64_t nch = ceil_div(4096, cblocks);   // ~4096 blocks (A/B at c5: 2048 -> 4096 10.0 -> 9.2 ms; 1024, 8192, 16384 slower)
  nch = nch < 1 ? 1 : nch;
  const int64_t maxch = ceil_div(ntiles, 64);
  nch = nch > maxch ? maxch : nch;
  nch = nch > 64 ? 64 : nch;
  if (nchunks_out) *nchunks_out = (int)nch;
  size_t off = 0;
  size_only<double>(off, (size_t)ntiles * LocalFeat<D>::KB * 64);
  size_only<double2>(off, (size_t)nch * (M > 0 ? M : 1));
  size_only<double>(off, 1);
  return off + 256;
}

template <int D>
int launch_pdf(const double* x, int64_t M, const double* X, const double* w,
               int64_t N, const double* inv, const double* lnorm, double* out,
               void* ws, size_t ws_bytes, hipStream_t s) {
  int nch = 1;
  if (ws_bytes < pdf_workspace<D>(M, N, &nch))
    return set_error(ABC_ERR_WORKSPACE, "local_logpdf: workspace too small");
  const int64_t ntiles = ceil_div(N, 16);
  constexpr int KB = LocalFeat<D>::KB, NT = LocalFeat<D>::NT;
  Carver c(ws, ws_bytes);
  double* psi = c.take<double>((size_t)ntiles * KB * 64);
  double2* part = c.take<double2>((size_t)nch * M);
  double* wsum = c.take<double>(1);
  const int64_t npack = ntiles * KB * 64;
  hipLaunchKernelGGL(local_pack_kernel<D>, dim3((unsigned)ceil_div(npack, 256)), dim3(256), 0,
                     s, X, w, inv, lnorm, N, ntiles, psi);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(local_wsum_kernel, dim3(1), dim3(1024), 0, s, w, N, wsum);
  ABC_LAUNCHED();
  const int64_t tpc = ceil_div(ntiles, nch);
  const int64_t cblocks = ceil_div(M, 4 * NT * 16);
  hipLaunchKernelGGL(local_mfma_kernel<D>, dim3((unsigned)cblocks, (unsigned)nch), dim3(256),
                     0, s, x, M, X, psi, ntiles, tpc, part);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(local_combine_kernel, dim3((unsigned)ceil_div(M, 256)), dim3(256), 0, s,
                     part, M, nch, wsum, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

}  // namespace

// d > 16: runtime-d kernels (abc_local_wide.hip)
size_t local_wide_fit_workspace(int64_t N, int d);
int local_wide_fit(const double* X, const double* w, int64_t N, int d, int64_t nq,
                   double scaling, double eps, double* covs, double* invs, double* dets,
                   double* chol, double* lnorm, void* ws, size_t ws_bytes, hipStream_t s);
int local_wide_logpdf(const double* x, int64_t M, const double* X, const double* w,
                      int64_t N, int d, const double* inv, const double* lnorm,
                      double* out, hipStream_t s);
}  // namespace abc

using namespace abc;

extern "C" size_t abc_local_fit_workspace(int64_t N, int d) {
  if (d > 16) return local_wide_fit_workspace(N, d);
  size_t off = 0;
  for (int i = 0; i < 3; ++i) size_only<int64_t>(off, (size_t)(N > 0 ? N : 1));
  size_only<float>(off, (size_t)(N > 0 ? N : 1) * (size_t)d);   // X32
  size_only<double>(off, 1);                                     // max |X|
  // partial moments of the row chunks (local_moments_kernel)
  const size_t nm = 2 + (size_t)d + (size_t)d * (d + 1) / 2;
  {
    const int rs = moments_chunks(N > 1 ? N : 1);
    size_only<double>(off, (size_t)(rs < 2 ? 2 : rs) * nm * (size_t)(N > 0 ? N : 1));
  }
  {  // fp32-MFMA k-NN select (abc_local_knn.h)
    const int64_t n1 = N > 0 ? N : 1;
    const int64_t nt = (n1 + 15) / 16;
    size_only<double>(off, (size_t)d);
    size_only<float>(off, (size_t)(nt + KN_PAD) * ((d + 5) / 4) * 64);   // + prefetch padding
    size_only<unsigned long long>(off, 1);
    size_only<int>(off, (size_t)n1);
    size_only<int>(off, (size_t)n1);
    size_only<int>(off, 2);
    size_only<double>(off, nm * (size_t)n1);
  }
  if (d <= 5) {   // dense-neighbourhood MFMA path (mm_*_kernel)
    const int64_t n1 = N > 0 ? N : 1;
    const int64_t nsteps = (n1 + 31) / 32;
    const int64_t nt = ((int64_t)nm * ML_NL + 15) / 16;
    size_only<unsigned long long>(off, 1 + (size_t)d);
    size_only<int>(off, 2);
    size_only<int>(off, (size_t)n1);                 // deferred collect: queue lengths
    size_only<int>(off, (size_t)n1);                 //   certain-below counts
    size_only<int>(off, (size_t)n1 * KN_QCAP);       //   queued rows
    size_only<half8>(off, (size_t)((nsteps + DM_SB) * nt * 64));
    size_only<double>(off, (size_t)mm_chunks(n1, nsteps) * 16 * nt * (size_t)n1);
    size_only<double>(off, nm * (size_t)n1);
    size_only<float>(off, (size_t)(nsteps + DM_SB) * dm_rstep<5>());
  }
  return off + 256;
}

extern "C" int abc_local_fit(const double* X, const double* w, int64_t N,
                             int d, int64_t k, double scaling, double eps,
                             double* covs, double* inv_covs, double* dets,
                             double* chol, double* log_norm, void* ws,
                             size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(N >= 1 && d >= 1 && d <= ABC_MAX_D && k >= 1, "local_fit: bad N/d/k");
  ABC_CHECK_ARG(N < (1ll << 31), "local_fit: N >= 2^31");
  ABC_CHECK_ARG(ws && ws_bytes >= abc_local_fit_workspace(N, d), "local_fit: workspace");
  ABC_CHECK_ARG(X && w && covs && inv_covs && dets && chol && log_norm, "local_fit: null pointer");
  const int64_t nq = (k + 1) < N ? (k + 1) : N;
  hipStream_t s = as_stream(stream);
  if (d > 16)
    return local_wide_fit(X, w, N, d, nq, scaling, eps, covs, inv_covs, dets, chol, log_norm,
                          ws, ws_bytes, s);
  switch (d) {
#define ABC_D(n) case n: return launch_fit<n>(X, w, N, nq, scaling, eps, covs, inv_covs, dets, chol, log_norm, ws, ws_bytes, s);
    ABC_D(1) ABC_D(2) ABC_D(3) ABC_D(4) ABC_D(5) ABC_D(6) ABC_D(7) ABC_D(8)
    ABC_D(9) ABC_D(10) ABC_D(11) ABC_D(12) ABC_D(13) ABC_D(14) ABC_D(15) ABC_D(16)
#undef ABC_D
  }
  return set_error(ABC_ERR_UNSUPPORTED, "local_fit: d=%d", d);
}

extern "C" size_t abc_local_logpdf_workspace(int64_t M, int64_t N, int d) {
  switch (d) {
#define ABC_D(n) case n: return pdf_workspace<n>(M, N, nullptr);
    ABC_D(1) ABC_D(2) ABC_D(3) ABC_D(4) ABC_D(5) ABC_D(6) ABC_D(7) ABC_D(8)
    ABC_D(9) ABC_D(10) ABC_D(11) ABC_D(12) ABC_D(13) ABC_D(14) ABC_D(15) ABC_D(16)
#undef ABC_D
  }
  return 256;
}

extern "C" int abc_local_logpdf(const double* x, int64_t M, const double* X,
                                const double* w, int64_t N, int d,
                                const double* inv_covs,
                                const double* log_norm, double* out,
                                void* ws, size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(M >= 0 && N >= 1 && d >= 1 && d <= ABC_MAX_D, "local_logpdf: bad M/N/d");
  if (M == 0) return ABC_OK;
  hipStream_t s = as_stream(stream);
  if (d > 16) {
    ABC_CHECK_ARG(x && X && w && inv_covs && log_norm && out, "local_logpdf: null pointer");
    return local_wide_logpdf(x, M, X, w, N, d, inv_covs, log_norm, out, s);
  }
  ABC_CHECK_ARG(x && X && w && inv_covs && log_norm && out && ws, "local_logpdf: null pointer");
  switch (d) {
#define ABC_D(n) case n: return launch_pdf<n>(x, M, X, w, N, inv_covs, log_norm, out, ws, ws_bytes, s);
    ABC_D(1) ABC_D(2) ABC_D(3) ABC_D(4) ABC_D(5) ABC_D(6) ABC_D(7) ABC_D(8)
    ABC_D(9) ABC_D(10) ABC_D(11) ABC_D(12) ABC_D(13) ABC_D(14) ABC_D(15) ABC_D(16)
#undef ABC_D
  }
  return set_error(ABC_ERR_UNSUPPORTED, "local_logpdf: d=%d", d);
}
