// LocalTransition for d > 16: runtime-d fp64 kernels (the templated d <= 16
// kernels of abc_local.hip keep their per-particle state in registers, which
// does not scale to d(d+1)/2 moments).  Up to d = 64 the per-particle matrices
// live in LDS; above (BIG) in a per-workgroup slice of the workspace, with
// the same operations in the same order (the reference has no cap on d).
//
// Reference: pyabc/transition/local_transition.py
//   fit :77-96   cKDTree.query(X, k+1), indices[n, 1:] -> local weighted
//                covariance of the neighbour offsets (:125-139), then
//                "while det <= 0: cov += EPS I" and inv / det (:112-123)
//   pdf :98-110  np.average(exp(-d^T inv_j d / 2) / norm_j, weights=w)
//
// fit: one 256-thread workgroup per particle (grid-stride over particles):
//   1. keys of the squared distances to every row (fp64 bits, the same fma
//      chain as abc_local.hip's dist2v) into a per-workgroup slice of the
//      workspace;
//   2. the key of rank nq - 1 by an MSD radix select (8 passes of 8 bits,
//      LDS histogram), the number of equal keys inside the nq nearest taken
//      by index (one ordered scan), the rank-0 index (smallest index at the
//      smallest key, dropped like indices[n, 1:]);
//   3. the members (key < v*, or key == v* and index < j*, minus rank 0)
//      compacted in index order;
//   4. the moments sum lw, lw^2, lw delta, then (a second sweep) lw (delta -
//      m)(delta - m)^T with the weighted mean m, over the members in that
//      order, chunks of rows staged in LDS, each thread owning a few of the
//      2 + d + d(d+1)/2 sums (deterministic);
//   5. thread 0: np.cov of the offsets, the fix-ups, LU (partial pivoting;
//      det and inverse from the same factors, as abc_local.hip), Cholesky.
// pdf: one thread per candidate, population rows (inverse, row, log w -
// log norm) staged in LDS and shared by the block, online log-sum-exp.
#include "abc_common.h"

namespace abc {
namespace {

constexpr double LOG_2PI_W = 1.8378770664093454836;
constexpr int WT = 256;        // threads per workgroup
constexpr int WD_MAX = 64;
constexpr int WCH = 32;        // member rows per LDS chunk (moments)

__device__ __forceinline__ unsigned long long dist_key(const double* __restrict__ xj,
                                                       const double* xn, int d) {
  double s = 0.0;
  for (int q = 0; q < d; ++q) { const double t = xj[q] - xn[q]; s = __builtin_fma(t, t, s); }
  return (unsigned long long)__double_as_longlong(s);
}

// exclusive scan of one int per thread over the 256-thread block
__device__ __forceinline__ int block_exscan(int v, int* sh, int& total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < WT; o <<= 1) {
    const int a = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += a;
    __syncthreads();
  }
  total = sh[WT - 1];
  const int incl = sh[t];
  __syncthreads();
  return incl - v;
}

struct WideFitArgs {
  const double* X;
  const double* w;
  int64_t N;
  int d;
  int64_t nq;
  double scaling, eps;
  unsigned long long* keys;  // [gridDim.x][N]
  int32_t* members;          // [gridDim.x][N]
  double* covs;
  double* invs;
  double* dets;
  double* chol;
  double* lnorm;
  double* big;               // BIG: [gridDim.x][wide_big_doubles(d)] per-block matrices
};

// per-workgroup doubles of the BIG path: xn, mom, a_lu, cov, x, perm (as doubles)
__host__ __device__ inline int64_t wide_big_doubles(int d) {
  const int64_t ld = d + 1;
  return (int64_t)d + (2 + d + (int64_t)d * (d + 1) / 2) + 2 * d * ld + d + d;
}

constexpr int WCH_FLAT = WCH * (WD_MAX + 1);   // LDS doubles of the member-row chunk
static_assert(ABC_MAX_D + 1 <= WCH_FLAT, "a member row (d + 1 doubles) must fit the LDS chunk");

template <bool BIG>
__global__ __launch_bounds__(WT) void local_wide_fit_kernel(WideFitArgs A) {
  const int t = threadIdx.x;
  const int d = A.d;
  const int64_t N = A.N;
  const int nm = 2 + d + d * (d + 1) / 2;
  const int ld = BIG ? d + 1 : WD_MAX + 1;     // row stride of cov / a_lu
  __shared__ unsigned int hist[256];
  __shared__ int scan_sh[WT];
  __shared__ unsigned long long red_k[WT];
  __shared__ long long red_j[WT];
  __shared__ unsigned long long s_prefix;
  __shared__ long long s_rank, s_jcut, s_r0, s_nmem;
  __shared__ double chunk_l[WCH_FLAT];          // member rows (+ lw in column d)
  __shared__ double xn_l[BIG ? 1 : WD_MAX];
  __shared__ double mom_l[BIG ? 1 : 2 + WD_MAX + WD_MAX * (WD_MAX + 1) / 2];
  __shared__ double a_lu_l[BIG ? 1 : WD_MAX * (WD_MAX + 1)];
  __shared__ double cov_l[BIG ? 1 : WD_MAX * (WD_MAX + 1)];
  __shared__ int perm_l[BIG ? 1 : WD_MAX];
  __shared__ double mean_l[BIG ? 1 : WD_MAX];
  double* bg = BIG ? A.big + (int64_t)blockIdx.x * wide_big_doubles(d) : nullptr;
  double* xn = BIG ? bg : xn_l;
  double* mom = BIG ? bg + d : mom_l;
  double* a_lu = BIG ? mom + nm : a_lu_l;
  double* cov = BIG ? a_lu + (int64_t)d * ld : cov_l;
  double* xsol = BIG ? cov + (int64_t)d * ld : nullptr;   // the inverse's column
  int* perm = BIG ? reinterpret_cast<int*>(xsol + d) : perm_l;
  const int rows_per_chunk = WCH_FLAT / (d + 1) < WCH ? WCH_FLAT / (d + 1) : WCH;
  unsigned long long* keys = A.keys + (int64_t)blockIdx.x * N;
  int32_t* mem = A.members + (int64_t)blockIdx.x * N;
  for (int64_t n = blockIdx.x; n < N; n += gridDim.x) {
    for (int q = t; q < d; q += WT) xn[q] = A.X[n * d + q];
    __syncthreads();
    // 1. keys; the running minimum (key, index) gives the rank-0 index
    unsigned long long kmin = ~0ull;
    long long jmin = N;
    for (int64_t j = t; j < N; j += WT) {
      const unsigned long long k = dist_key(A.X + j * d, xn, d);
      keys[j] = k;
      if (k < kmin) { kmin = k; jmin = j; }   // j ascending per thread
    }
    red_k[t] = kmin;
    red_j[t] = jmin;
    __syncthreads();
    for (int o = WT / 2; o > 0; o >>= 1) {
      if (t < o) {
        const unsigned long long ko = red_k[t + o];
        const long long jo = red_j[t + o];
        if (ko < red_k[t] || (ko == red_k[t] && jo < red_j[t])) { red_k[t] = ko; red_j[t] = jo; }
      }
      __syncthreads();
    }
    if (t == 0) { s_r0 = red_j[0]; s_prefix = 0ull; s_rank = A.nq - 1; }
    __syncthreads();
    // 2. MSD radix select of rank nq - 1 (keys sharing the prefix so far)
    for (int pass = 0; pass < 8; ++pass) {
      const int sh = 56 - 8 * pass;
      hist[t] = 0u;
      __syncthreads();
      const unsigned long long pre = s_prefix;
      for (int64_t j = t; j < N; j += WT) {
        const unsigned long long k = keys[j];
        const bool in = pass == 0 ? true : ((k >> (sh + 8)) == (pre >> (sh + 8)));
        if (in) atomicAdd(&hist[(k >> sh) & 255ull], 1u);
      }
      __syncthreads();
      if (t == 0) {
        long long r = s_rank;
        int b = 0;
        for (; b < 255 && r >= (long long)hist[b]; ++b) r -= hist[b];
        s_rank = r;
        s_prefix = pre | ((unsigned long long)b << sh);
      }
      __syncthreads();
    }
    const unsigned long long vs = s_prefix;
    const long long tie_rank = s_rank;   // 0-based rank among keys == v*, by index
    // the index of that equal key: ordered sweep over index chunks of WT
    if (t == 0) s_jcut = N;
    __syncthreads();
    int seen = 0;
    for (int64_t j0 = 0; j0 < N; j0 += WT) {
      const int64_t j = j0 + t;
      const int eq = (j < N && keys[j] == vs) ? 1 : 0;
      int tot;
      const int before = block_exscan(eq, scan_sh, tot);
      if (eq && seen + before == tie_rank) s_jcut = j + 1;   // (key, j) <= (v*, j*)
      seen += tot;
      if (seen > tie_rank) break;   // uniform: every thread holds the same seen
    }
    __syncthreads();
    const long long jcut = s_jcut, r0 = s_r0;
    // 3. members in index order
    int cnt = 0;
    for (int64_t j0 = 0; j0 < N; j0 += WT) {
      const int64_t j = j0 + t;
      int m = 0;
      if (j < N) {
        const unsigned long long k = keys[j];
        m = ((k < vs) || (k == vs && j < jcut)) && j != r0;
      }
      int tot;
      const int pos = block_exscan(m, scan_sh, tot);
      if (m) mem[cnt + pos] = (int32_t)j;
      cnt += tot;
    }
    if (t == 0) s_nmem = cnt;
    __syncthreads();
    const int64_t nmem = s_nmem;
    // 4. moments over the members, one chunk of rows at a time; each thread
    // owns the sums f = t + e WT (16 per pass; more passes above d = 89, each
    // streaming the members again).  Two sweeps, as np.cov's own two passes
    // (average, then the products of the centred offsets): first lw, lw^2
    // and lw delta, then lw (delta - m)(delta - m)^T with the weighted mean m
    // -- the one-sweep form E[dd^T] - m m^T cancelled when the neighbourhood
    // sits off its particle (4e-11 relative at d = 80,
    // profiles/r06_d80_weight_bound_probe.log).
    const int cs = d + 1;                  // chunk row stride
    double* chunk = chunk_l;
    double* mean = BIG ? xsol : mean_l;    // (xsol is free until step 5)
    for (int sweep = 0; sweep < 2; ++sweep) {
    const int fa = sweep == 0 ? 0 : 2 + d, fb = sweep == 0 ? 2 + d : nm;
    for (int f0 = fa; f0 < fb; f0 += 16 * WT) {
      double acc[16];
      int ea[16], eb[16];
      const int rem = fb - f0;
      const int per = (rem + WT - 1) / WT < 16 ? (rem + WT - 1) / WT : 16;
      for (int e = 0; e < per; ++e) {
        acc[e] = 0.0;
        // sum f: 0 -> lw, 1 -> lw^2, 2 + a -> lw delta_a, then the upper
        // triangle (a <= b) row by row -> lw delta_a delta_b
        const int f = f0 + t + e * WT;
        int a = -1, b = -1;
        if (f >= 2 && f < 2 + d) a = f - 2;
        if (f >= 2 + d && f < nm) {
          int g = f - 2 - d;
          a = 0;
          while (g >= d - a) { g -= d - a; ++a; }
          b = a + g;
        }
        ea[e] = a;
        eb[e] = b;
      }
      for (int64_t c0 = 0; c0 < nmem; c0 += rows_per_chunk) {
        const int rows = (int)((nmem - c0) < rows_per_chunk ? (nmem - c0) : rows_per_chunk);
        for (int e = t; e < rows * cs; e += WT) {
          const int r = e / cs, q = e - r * cs;
          const int64_t j = mem[c0 + r];
          chunk[r * cs + q] = q < d ? (sweep == 0 ? A.X[j * d + q] - xn[q]
                                                  : (A.X[j * d + q] - xn[q]) - mean[q])
                                    : A.w[j];
        }
        __syncthreads();
        for (int e = 0; e < per; ++e) {
          const int f = f0 + t + e * WT;
          if (f >= fb) break;
          double sm = acc[e];
          if (f == 0) {
            for (int r = 0; r < rows; ++r) sm += chunk[r * cs + d];
          } else if (f == 1) {
            for (int r = 0; r < rows; ++r) sm += chunk[r * cs + d] * chunk[r * cs + d];
          } else if (eb[e] < 0) {
            const int a = ea[e];
            for (int r = 0; r < rows; ++r) sm += chunk[r * cs + d] * chunk[r * cs + a];
          } else {
            const int a = ea[e], b = eb[e];
            for (int r = 0; r < rows; ++r)
              sm += chunk[r * cs + d] * chunk[r * cs + a] * chunk[r * cs + b];
          }
          acc[e] = sm;
        }
        __syncthreads();
      }
      for (int e = 0; e < per; ++e) {
        const int f = f0 + t + e * WT;
        if (f < fb) mom[f] = acc[e];
      }
    }
    __syncthreads();
    if (sweep == 0) {
      for (int q = t; q < d; q += WT) mean[q] = mom[2 + q] / mom[0];
      __syncthreads();
    }
    }
    // 5. covariance, fix-ups, factorisations (thread 0)
    if (t == 0) {
      if (N == 1) {
        // indices is 1-D -> deltas = |X|, one sample -> diag(|X[0]|)
        for (int a = 0; a < d; ++a)
          for (int b = 0; b < d; ++b) cov[(a) * ld + (b)] = (a == b) ? fabs(A.X[a]) : 0.0;
      } else if (A.nq - 1 == 1) {
        // one neighbour: smart_cov -> diag(|delta|), delta = sum lw d / sum lw
        for (int a = 0; a < d; ++a)
          for (int b = 0; b < d; ++b) cov[(a) * ld + (b)] = (a == b) ? fabs(mom[2 + a] / mom[0]) : 0.0;
      } else {
        const double sw = mom[0];
        const double sa2 = mom[1] / (sw * sw);
        int f = 2 + d;
        for (int a = 0; a < d; ++a)
          for (int b = a; b < d; ++b, ++f) {
            // (mom[f]: the centred products of the second sweep)
            const double v = (mom[f] / sw) / (1.0 - sa2);
            cov[(a) * ld + (b)] = v;
            cov[(b) * ld + (a)] = v;
          }
      }
      double csum = 0.0;
      for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b) csum += cov[(a) * ld + (b)];
      if (fabs(csum) == 0.0)
        for (int a = 0; a < d; ++a) cov[(a) * ld + (a)] = fabs(A.X[a]);  // X[0, a]
      for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b) cov[(a) * ld + (b)] *= A.scaling;
      double det = 0.0;
      for (int it = 0;; ++it) {
        for (int a = 0; a < d; ++a)
          for (int b = 0; b < d; ++b) a_lu[(a) * ld + (b)] = cov[(a) * ld + (b)];
        // LU, getrf order: pivot = first max |a[r][c]|
        det = 1.0;
        for (int i = 0; i < d; ++i) perm[i] = i;
        for (int c = 0; c < d; ++c) {
          int p = c;
          double best = fabs(a_lu[(c) * ld + (c)]);
          for (int r = c + 1; r < d; ++r)
            if (fabs(a_lu[(r) * ld + (c)]) > best) { best = fabs(a_lu[(r) * ld + (c)]); p = r; }
          if (a_lu[(p) * ld + (c)] == 0.0) { det = 0.0; break; }
          if (p != c) {
            for (int j = 0; j < d; ++j) { const double x = a_lu[(c) * ld + (j)]; a_lu[(c) * ld + (j)] = a_lu[(p) * ld + (j)]; a_lu[(p) * ld + (j)] = x; }
            const int x = perm[c]; perm[c] = perm[p]; perm[p] = x;
            det = -det;
          }
          det *= a_lu[(c) * ld + (c)];
          const double rp = 1.0 / a_lu[(c) * ld + (c)];
          for (int r = c + 1; r < d; ++r) {
            const double fct = a_lu[(r) * ld + (c)] * rp;
            a_lu[(r) * ld + (c)] = fct;
            for (int j = c + 1; j < d; ++j) a_lu[(r) * ld + (j)] -= fct * a_lu[(c) * ld + (j)];
          }
        }
        if (!(det <= 0.0) || it >= 1000000) break;  // NaN exits, as "while det <= 0" does
        for (int a = 0; a < d; ++a) cov[(a) * ld + (a)] += A.eps;
      }
      double* inv = A.invs + n * d * d;
      double* L = A.chol + n * d * d;
      double* cv = A.covs + n * d * d;
      // inverse: column j solves L U x = P e_j (x staged in the output row)
      for (int j = 0; j < d; ++j) {
        double x_l[BIG ? 1 : WD_MAX];
        double* x = BIG ? xsol : x_l;
        for (int i = 0; i < d; ++i) {
          double v = perm[i] == j ? 1.0 : 0.0;
          for (int k = 0; k < i; ++k) v -= a_lu[(i) * ld + (k)] * x[k];
          x[i] = v;
        }
        for (int i = d - 1; i >= 0; --i) {
          double v = x[i];
          for (int k = i + 1; k < d; ++k) v -= a_lu[(i) * ld + (k)] * x[k];
          x[i] = v / a_lu[(i) * ld + (i)];
        }
        for (int i = 0; i < d; ++i) inv[i * d + j] = x[i];
      }
      // Cholesky (a_lu reused); sqrt|diag| if a pivot is not positive
      bool ok = true;
      for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b) a_lu[(a) * ld + (b)] = 0.0;
      for (int j = 0; j < d && ok; ++j) {
        double s = cov[(j) * ld + (j)];
        for (int k = 0; k < j; ++k) s -= a_lu[(j) * ld + (k)] * a_lu[(j) * ld + (k)];
        if (!(s > 0.0)) { ok = false; break; }
        a_lu[(j) * ld + (j)] = sqrt(s);
        for (int i = j + 1; i < d; ++i) {
          double x = cov[(i) * ld + (j)];
          for (int k = 0; k < j; ++k) x -= a_lu[(i) * ld + (k)] * a_lu[(j) * ld + (k)];
          a_lu[(i) * ld + (j)] = x / a_lu[(j) * ld + (j)];
        }
      }
      for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b) {
          cv[a * d + b] = cov[(a) * ld + (b)];
          L[a * d + b] = ok ? a_lu[(a) * ld + (b)] : ((a == b) ? sqrt(fabs(cov[(a) * ld + (a)])) : 0.0);
        }
      A.dets[n] = det;
      A.lnorm[n] = 0.5 * (d * LOG_2PI_W + log(det));
    }
    __syncthreads();
  }
}

// d > 64: the same sum with the inverse and the rows read from global
// memory (no LDS staging, no register rows): q_ij = sum_a dl_a sum_b inv_ab dl_b
// in local_wide_pdf_kernel's order
__global__ __launch_bounds__(WT) void local_wide_pdf_big_kernel(
    const double* __restrict__ x, int64_t M, const double* __restrict__ X,
    const double* __restrict__ w, int64_t N, int d, const double* __restrict__ inv,
    const double* __restrict__ lnorm, double* __restrict__ out) {
  __shared__ double wsum_sh[WT];
  const int t = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * WT + t;
  const int64_t ie = i < M ? i : M - 1;
  const double* xi = x + ie * d;
  double m = -INFINITY, l = 0.0;
  for (int64_t j = 0; j < N; ++j) {
    const double wj = w[j];
    const double* Xj = X + j * d;
    const double* ij = inv + j * d * d;
    double qf = 0.0;
    for (int a = 0; a < d; ++a) {
      double y = 0.0;
      for (int b = 0; b < d; ++b) y = __builtin_fma(ij[a * d + b], Xj[b] - xi[b], y);
      qf = __builtin_fma(Xj[a] - xi[a], y, qf);
    }
    const double s = (wj > 0.0 ? log(wj) : -INFINITY) - lnorm[j] - 0.5 * qf;
    if (s > m) { l = l * exp(m - s) + 1.0; m = s; }
    else if (s > -INFINITY) l += exp(s - m);
  }
  double sw = 0.0;
  for (int64_t j = t; j < N; j += WT) sw += w[j];
  wsum_sh[t] = sw;
  __syncthreads();
  for (int o = WT / 2; o > 0; o >>= 1) {
    if (t < o) wsum_sh[t] += wsum_sh[t + o];
    __syncthreads();
  }
  if (i < M) out[i] = (l > 0.0) ? m + log(l) - log(wsum_sh[0]) : -INFINITY;
}

// log density of candidate i: log sum_j w_j exp(-q_ij / 2) / norm_j - log sum w
constexpr int WP_ROWS = 4;   // population rows staged per LDS round
__global__ __launch_bounds__(WT) void local_wide_pdf_kernel(
    const double* __restrict__ x, int64_t M, const double* __restrict__ X,
    const double* __restrict__ w, int64_t N, int d, const double* __restrict__ inv,
    const double* __restrict__ lnorm, double* __restrict__ out) {
  __shared__ double sinv[WP_ROWS][WD_MAX * WD_MAX];
  __shared__ double sx[WP_ROWS][WD_MAX];
  __shared__ double sc[WP_ROWS];
  __shared__ double wsum_sh[WT];
  const int t = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * WT + t;
  double xi[WD_MAX];
  for (int q = 0; q < d; ++q) xi[q] = i < M ? x[i * d + q] : 0.0;
  double m = -INFINITY, l = 0.0;
  for (int64_t j0 = 0; j0 < N; j0 += WP_ROWS) {
    const int rows = (int)((N - j0) < WP_ROWS ? (N - j0) : WP_ROWS);
    for (int e = t; e < rows * d * d; e += WT) {
      const int r = e / (d * d), q = e - r * d * d;
      sinv[r][q] = inv[(j0 + r) * d * d + q];
    }
    for (int e = t; e < rows * d; e += WT) {
      const int r = e / d, q = e - r * d;
      sx[r][q] = X[(j0 + r) * d + q];
    }
    if (t < rows) {
      const double wj = w[j0 + t];
      sc[t] = (wj > 0.0 ? log(wj) : -INFINITY) - lnorm[j0 + t];
    }
    __syncthreads();
    for (int r = 0; r < rows; ++r) {
      double dl[WD_MAX];
      for (int q = 0; q < d; ++q) dl[q] = sx[r][q] - xi[q];
      double qf = 0.0;
      for (int a = 0; a < d; ++a) {
        double y = 0.0;
        for (int b = 0; b < d; ++b) y = __builtin_fma(sinv[r][a * d + b], dl[b], y);
        qf = __builtin_fma(dl[a], y, qf);
      }
      const double s = sc[r] - 0.5 * qf;
      if (s > m) { l = l * exp(m - s) + 1.0; m = s; }
      else if (s > -INFINITY) l += exp(s - m);
    }
    __syncthreads();
  }
  // np.average's denominator, fixed order per thread then a tree
  double sw = 0.0;
  for (int64_t j = t; j < N; j += WT) sw += w[j];
  wsum_sh[t] = sw;
  __syncthreads();
  for (int o = WT / 2; o > 0; o >>= 1) {
    if (t < o) wsum_sh[t] += wsum_sh[t + o];
    __syncthreads();
  }
  if (i < M) out[i] = (l > 0.0) ? m + log(l) - log(wsum_sh[0]) : -INFINITY;
}

int wide_fit_blocks(int64_t N, int d) {
  // keys + member list (12 B per row) + the BIG matrices per workgroup,
  // capped at ~1 GiB
  const int64_t per = 12 * (N > 0 ? N : 1) + (d > WD_MAX ? 8 * wide_big_doubles(d) : 0);
  int64_t g = (int64_t)(1ll << 30) / per;
  g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
  return (int)(g < N ? g : N);
}

}  // namespace

size_t local_wide_fit_workspace(int64_t N, int d) {
  const int64_t n1 = N > 0 ? N : 1;
  const int g = wide_fit_blocks(n1, d);
  size_t off = 0;
  size_only<unsigned long long>(off, (size_t)g * n1);
  size_only<int32_t>(off, (size_t)g * n1);
  if (d > WD_MAX) size_only<double>(off, (size_t)g * wide_big_doubles(d));
  return off + 256;
}

int local_wide_fit(const double* X, const double* w, int64_t N, int d, int64_t nq,
                   double scaling, double eps, double* covs, double* invs, double* dets,
                   double* chol, double* lnorm, void* ws, size_t ws_bytes, hipStream_t s) {
  if (ws_bytes < local_wide_fit_workspace(N, d))
    return set_error(ABC_ERR_WORKSPACE, "local_fit (d > 16): workspace too small");
  const int g = wide_fit_blocks(N, d);
  Carver c(ws, ws_bytes);
  WideFitArgs A{X, w, N, d, nq, scaling, eps, nullptr, nullptr,
                covs, invs, dets, chol, lnorm, nullptr};
  A.keys = c.take<unsigned long long>((size_t)g * N);
  A.members = c.take<int32_t>((size_t)g * N);
  if (d > WD_MAX) {
    A.big = c.take<double>((size_t)g * wide_big_doubles(d));
    if (!c.ok) return set_error(ABC_ERR_WORKSPACE, "local_fit (d > 64): workspace carve");
    hipLaunchKernelGGL(local_wide_fit_kernel<true>, dim3((unsigned)g), dim3(WT), 0, s, A);
  } else {
    hipLaunchKernelGGL(local_wide_fit_kernel<false>, dim3((unsigned)g), dim3(WT), 0, s, A);
  }
  ABC_LAUNCHED();
  return ABC_OK;
}

int local_wide_logpdf(const double* x, int64_t M, const double* X, const double* w,
                      int64_t N, int d, const double* inv, const double* lnorm,
                      double* out, hipStream_t s) {
  if (M == 0) return ABC_OK;
  if (d > WD_MAX)
    hipLaunchKernelGGL(local_wide_pdf_big_kernel, dim3((unsigned)ceil_div(M, WT)), dim3(WT), 0,
                       s, x, M, X, w, N, d, inv, lnorm, out);
  else
    hipLaunchKernelGGL(local_wide_pdf_kernel, dim3((unsigned)ceil_div(M, WT)), dim3(WT), 0, s,
                       x, M, X, w, N, d, inv, lnorm, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

}  // namespace abc
