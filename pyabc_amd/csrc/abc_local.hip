// LocalTransition on CDNA4: per-particle k-NN covariance fit, density, rvs.
//
// Reference: pyabc/transition/local_transition.py
//   fit   :77-96   cKDTree.query(X, k+1) per particle, then a Python loop of
//                  _cov_and_inv (:112-123) / _cov (:125-139) per particle
//   pdf   :98-110  np.average(exp(-d^T inv_j d / 2) / norm_j, weights=w)
//   rvs   :141-145 j ~ Cat(w); theta ~ N(X_j, cov_j)  (abc_local_propose in
//                  abc_sampler.hip uses the Cholesky factors written here)
//
// fit: one 256-thread workgroup per particle n.  The k+1 nearest particles in
// (squared distance, index) order are found by an exact MSD radix select on
// the fp64 bits of the squared distances (8 passes of 8 bits, LDS
// histograms); a final ordered pass accumulates the weighted moments of the
// neighbour offsets (ties at the k-th distance taken by index, rank 0
// dropped like the reference's indices[n, 1:]).  Thread 0 then applies the
// reference's fix-ups (diag(|X[0]|) for an all-zero covariance, scaling,
// "while det <= 0: cov += EPS I") and writes cov, inverse (Gauss-Jordan with
// partial pivoting), det (LU), Cholesky and log normalisation.
#include "abc_common.h"

namespace abc {
namespace {

constexpr double LOG_2PI = 1.8378770664093454836;

template <int D>
__device__ __forceinline__ double dist2(const double* __restrict__ X, int64_t j,
                                        const double (&xn)[D]) {
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < D; ++q) { double t = X[j * D + q] - xn[q]; s += t * t; }
  return s;
}

template <int D>
__device__ double det_lu(const double (&a_in)[D][D]) {
  double a[D][D];
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) a[i][j] = a_in[i][j];
  double det = 1.0;
  for (int c = 0; c < D; ++c) {
    int p = c;
    double best = fabs(a[c][c]);
    for (int r = c + 1; r < D; ++r)
      if (fabs(a[r][c]) > best) { best = fabs(a[r][c]); p = r; }
    if (a[p][c] == 0.0) return 0.0;
    if (p != c) {
      for (int j = 0; j < D; ++j) { double t = a[c][j]; a[c][j] = a[p][j]; a[p][j] = t; }
      det = -det;
    }
    det *= a[c][c];
    for (int r = c + 1; r < D; ++r) {
      double f = a[r][c] / a[c][c];
      for (int j = c + 1; j < D; ++j) a[r][j] -= f * a[c][j];
    }
  }
  return det;
}

template <int D>
__device__ void inverse_gj(const double (&a_in)[D][D], double (&inv)[D][D]) {
  double a[D][2 * D];
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) { a[i][j] = a_in[i][j]; a[i][D + j] = (i == j) ? 1.0 : 0.0; }
  for (int c = 0; c < D; ++c) {
    int p = c;
    double best = fabs(a[c][c]);
    for (int r = c + 1; r < D; ++r)
      if (fabs(a[r][c]) > best) { best = fabs(a[r][c]); p = r; }
    if (p != c)
      for (int j = 0; j < 2 * D; ++j) { double t = a[c][j]; a[c][j] = a[p][j]; a[p][j] = t; }
    const double piv = a[c][c];
    for (int j = 0; j < 2 * D; ++j) a[c][j] /= piv;
    for (int r = 0; r < D; ++r) {
      if (r == c) continue;
      const double f = a[r][c];
      if (f != 0.0)
        for (int j = 0; j < 2 * D; ++j) a[r][j] -= f * a[c][j];
    }
  }
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) inv[i][j] = a[i][D + j];
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

template <int D>
__global__ __launch_bounds__(256) void local_fit_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t N,
    int64_t nq, double scaling, double eps, double* __restrict__ covs,
    double* __restrict__ invs, double* __restrict__ dets,
    double* __restrict__ chol, double* __restrict__ lnorm) {
  constexpr int NM = 2 + D + D * D;  // sum lw, sum lw^2, sum lw d, sum lw dd^T
  __shared__ unsigned hist[256];
  __shared__ unsigned long long sh_prefix;
  __shared__ long long sh_rank;
  __shared__ unsigned long long sh_rank0;
  __shared__ double red[NM][4];
  __shared__ int sh_ties[4];
  const int64_t n = blockIdx.x;
  const int tid = threadIdx.x;
  double xn[D];
#pragma unroll
  for (int q = 0; q < D; ++q) xn[q] = X[n * D + q];

  double cov[D][D];
  if (N == 1) {
    // indices is 1-D -> deltas = |X|, one sample -> diag(|X[0]|)
    for (int a = 0; a < D; ++a)
      for (int b = 0; b < D; ++b) cov[a][b] = (a == b) ? fabs(X[a]) : 0.0;
  } else {
    if (tid == 0) { sh_prefix = 0ull; sh_rank = nq - 1; sh_rank0 = (unsigned long long)N; }
    __syncthreads();
    // MSD radix select of the element at rank nq-1
    for (int pass = 0; pass < 8; ++pass) {
      const int shift = 56 - 8 * pass;
      hist[tid] = 0u;
      __syncthreads();
      const unsigned long long pre = sh_prefix;
      for (int64_t j = tid; j < N; j += 256) {
        const unsigned long long key = (unsigned long long)__double_as_longlong(dist2<D>(X, j, xn));
        const bool match = (pass == 0) || ((key >> (shift + 8)) == pre);
        if (match) atomicAdd(&hist[(key >> shift) & 255ull], 1u);
        // rank-0 element: smallest index at squared distance 0
        if (pass == 0 && key == 0ull) atomicMin(&sh_rank0, (unsigned long long)j);
      }
      __syncthreads();
      if (tid == 0) {
        long long r = sh_rank;
        int b = 0;
        for (; b < 256; ++b) {
          if (r < (long long)hist[b]) break;
          r -= hist[b];
        }
        sh_rank = r;
        sh_prefix = (pre << 8) | (unsigned long long)b;
      }
      __syncthreads();
    }
    const unsigned long long vstar = sh_prefix;
    const long long ties_in = sh_rank + 1;  // ties at vstar included (by index)
    const long long rank0 = (long long)sh_rank0;
    // ordered accumulation pass
    double m[NM];
#pragma unroll
    for (int t = 0; t < NM; ++t) m[t] = 0.0;
    long long ties_before = 0;
    for (int64_t c0 = 0; c0 < N; c0 += 256) {
      const int64_t j = c0 + tid;
      unsigned long long key = ~0ull;
      double dj[D];
      if (j < N) {
#pragma unroll
        for (int q = 0; q < D; ++q) dj[q] = X[j * D + q] - xn[q];
        key = (unsigned long long)__double_as_longlong(dist2<D>(X, j, xn));
      }
      const int tie = (j < N && key == vstar) ? 1 : 0;
      // exclusive prefix of ties in index order within the chunk (ballots)
      const unsigned long long bal = __ballot(tie);
      const int lane = tid & 63, wv = tid >> 6;
      if (lane == 0) sh_ties[wv] = __popcll(bal);
      __syncthreads();
      int before = __popcll(bal & ((1ull << lane) - 1ull)), total = 0;
      for (int t = 0; t < 4; ++t) { const int v = sh_ties[t]; if (t < wv) before += v; total += v; }
      __syncthreads();
      bool inc = (j < N) && (key < vstar || (tie && ties_before + before < ties_in));
      if (j == rank0) inc = false;
      if (inc) {
        const double lw = w[j];
        m[0] += lw; m[1] += lw * lw;
#pragma unroll
        for (int a = 0; a < D; ++a) {
          m[2 + a] += lw * dj[a];
#pragma unroll
          for (int b = 0; b < D; ++b) m[2 + D + a * D + b] += lw * dj[a] * dj[b];
        }
      }
      ties_before += total;
    }
    // deterministic block reduction: wave shuffle, then 4 waves in order
#pragma unroll
    for (int t = 0; t < NM; ++t) {
      double v = wave_sum(m[t]);
      if ((tid & 63) == 0) red[t][tid >> 6] = v;
    }
    __syncthreads();
    if (tid != 0) return;
    double M[NM];
    for (int t = 0; t < NM; ++t) M[t] = ((red[t][0] + red[t][1]) + red[t][2]) + red[t][3];
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
          cov[a][b] = (M[2 + D + a * D + b] / sw - mean[a] * mean[b]) / (1.0 - sa2);
    }
  }
  if (tid != 0) return;
  double csum = 0.0;
  for (int a = 0; a < D; ++a)
    for (int b = 0; b < D; ++b) csum += cov[a][b];
  if (fabs(csum) == 0.0)
    for (int a = 0; a < D; ++a) cov[a][a] = fabs(X[a]);  // X[0, a]
  for (int a = 0; a < D; ++a)
    for (int b = 0; b < D; ++b) cov[a][b] *= scaling;
  double det = det_lu<D>(cov);
  for (int it = 0; det <= 0.0 && it < 1000000; ++it) {
    for (int a = 0; a < D; ++a) cov[a][a] += eps;
    det = det_lu<D>(cov);
  }
  double inv[D][D], L[D][D];
  inverse_gj<D>(cov, inv);
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

// density: block of 256 candidates, population staged through LDS in tiles
template <int D>
__global__ __launch_bounds__(256) void local_pdf_kernel(
    const double* __restrict__ x, int64_t M, const double* __restrict__ X,
    const double* __restrict__ w, int64_t N, const double* __restrict__ invs,
    const double* __restrict__ lnorm, double* __restrict__ out) {
  constexpr int TJ = 32;
  constexpr int REC = D + D * D + 1;  // X_j, inv_j, log w_j - lnorm_j
  __shared__ double tile[TJ * REC];
  __shared__ double wsum_sh[4];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double xi[D];
#pragma unroll
  for (int q = 0; q < D; ++q) xi[q] = (i < M) ? x[i * D + q] : 0.0;
  double m = -INFINITY, l = 0.0, wsum = 0.0;
  for (int64_t j0 = 0; j0 < N; j0 += TJ) {
    const int nj = (int)((N - j0) < TJ ? (N - j0) : TJ);
    __syncthreads();
    for (int e = threadIdx.x; e < nj * REC; e += 256) {
      const int jj = e / REC, f = e % REC;
      const int64_t j = j0 + jj;
      double v;
      if (f < D) v = X[j * D + f];
      else if (f < D + D * D) v = invs[j * D * D + (f - D)];
      else { const double wj = w[j]; v = (wj > 0.0) ? log(wj) - lnorm[j] : -INFINITY; }
      tile[jj * REC + f] = v;
    }
    __syncthreads();
    for (int jj = 0; jj < nj; ++jj) {
      const double* r = tile + jj * REC;
      double dv[D];
#pragma unroll
      for (int q = 0; q < D; ++q) dv[q] = r[q] - xi[q];
      double md = 0.0;
#pragma unroll
      for (int a = 0; a < D; ++a) {
        double t = 0.0;
#pragma unroll
        for (int b = 0; b < D; ++b) t += r[D + a * D + b] * dv[b];
        md += dv[a] * t;
      }
      const double s = r[D + D * D] - 0.5 * md;
      if (s > m) { l = l * exp(m - s) + 1.0; m = s; }
      else if (s > -INFINITY) l += exp(s - m);
    }
  }
  // sum of weights (np.average denominator), same for every candidate
  double ws = 0.0;
  for (int64_t j = threadIdx.x; j < N; j += 256) ws += w[j];
  ws = wave_sum(ws);
  if ((threadIdx.x & 63) == 0) wsum_sh[threadIdx.x >> 6] = ws;
  __syncthreads();
  wsum = ((wsum_sh[0] + wsum_sh[1]) + wsum_sh[2]) + wsum_sh[3];
  if (i < M) out[i] = (l > 0.0) ? m + log(l) - log(wsum) : -INFINITY;
}

template <int D>
int launch_fit(const double* X, const double* w, int64_t N, int64_t nq,
               double scaling, double eps, double* covs, double* inv,
               double* dets, double* chol, double* lnorm, hipStream_t s) {
  hipLaunchKernelGGL(local_fit_kernel<D>, dim3((unsigned)N), dim3(256), 0, s, X, w, N, nq,
                     scaling, eps, covs, inv, dets, chol, lnorm);
  ABC_LAUNCHED();
  return ABC_OK;
}

template <int D>
int launch_pdf(const double* x, int64_t M, const double* X, const double* w,
               int64_t N, const double* inv, const double* lnorm, double* out,
               hipStream_t s) {
  hipLaunchKernelGGL(local_pdf_kernel<D>, dim3((unsigned)ceil_div(M, 256)), dim3(256), 0, s,
                     x, M, X, w, N, inv, lnorm, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" size_t abc_local_fit_workspace(int64_t N, int d) {
  (void)N; (void)d;
  return 0;
}

extern "C" int abc_local_fit(const double* X, const double* w, int64_t N,
                             int d, int64_t k, double scaling, double eps,
                             double* covs, double* inv_covs, double* dets,
                             double* chol, double* log_norm, void* ws,
                             size_t ws_bytes, void* stream) {
  (void)ws; (void)ws_bytes;
  ABC_CHECK_ARG(N >= 1 && d >= 1 && d <= 8 && k >= 1, "local_fit: bad N/d/k (d <= 8)");
  ABC_CHECK_ARG(X && w && covs && inv_covs && dets && chol && log_norm, "local_fit: null pointer");
  const int64_t nq = (k + 1) < N ? (k + 1) : N;
  hipStream_t s = as_stream(stream);
  switch (d) {
#define ABC_D(n) case n: return launch_fit<n>(X, w, N, nq, scaling, eps, covs, inv_covs, dets, chol, log_norm, s);
    ABC_D(1) ABC_D(2) ABC_D(3) ABC_D(4) ABC_D(5) ABC_D(6) ABC_D(7) ABC_D(8)
#undef ABC_D
  }
  return set_error(ABC_ERR_UNSUPPORTED, "local_fit: d=%d", d);
}

extern "C" int abc_local_logpdf(const double* x, int64_t M, const double* X,
                                const double* w, int64_t N, int d,
                                const double* inv_covs,
                                const double* log_norm, double* out,
                                void* stream) {
  ABC_CHECK_ARG(M >= 0 && N >= 1 && d >= 1 && d <= 8, "local_logpdf: bad M/N/d");
  if (M == 0) return ABC_OK;
  ABC_CHECK_ARG(x && X && w && inv_covs && log_norm && out, "local_logpdf: null pointer");
  hipStream_t s = as_stream(stream);
  switch (d) {
#define ABC_D(n) case n: return launch_pdf<n>(x, M, X, w, N, inv_covs, log_norm, out, s);
    ABC_D(1) ABC_D(2) ABC_D(3) ABC_D(4) ABC_D(5) ABC_D(6) ABC_D(7) ABC_D(8)
#undef ABC_D
  }
  return set_error(ABC_ERR_UNSUPPORTED, "local_logpdf: d=%d", d);
}
