// MultivariateNormalTransition.fit's host half on the device: from the
// weighted moments (abc_weighted_moments), the KDE covariance, its PSD
// eigen-whitening and the sampling factor, with no host read in the fit.
//
// Reference: pyabc/transition/multivariatenormal.py:72-83
//   cov = smart_cov(X, w) * bandwidth_selector(ess, d)^2 * scaling
//     (np.cov(X, aweights=w, rowvar=False); ess = 1 / sum w^2,
//      silverman :27-37 or scott :14-24)
//   normal = st.multivariate_normal(cov=cov, allow_singular=True)
//     -> scipy.stats._multivariate._PSD: s, u = eigh(cov); cut-off
//        1e6 eps max|s| ("not positive semidefinite" below -cut-off);
//        U = u[:, s > cut] / sqrt(s); log pdet = sum log s[kept]
//
// One workgroup: the d x d matrix (d <= 64) in LDS.  A full-rank covariance
// (certified by a lower bound on its smallest eigenvalue, see the fast path)
// is whitened by its Cholesky factor (U = L^-T).  Otherwise a parallel cyclic
// Jacobi eigen-decomposition in fp64 (round-robin pair ordering: each step
// rotates d/2 disjoint (p, q) pairs, rows then columns; sweeps until every
// off-diagonal is below 2^-53 sqrt(|a_pp a_qq|)), eigenpairs sorted by
// decreasing eigenvalue, the whitening U (kept columns scaled by 1/sqrt(s),
// cut ones zero -- so the MFMA image can be packed at rank d before the
// host knows the rank), and L L^T = cov from the eigen factor (QR of
// (V diag(sqrt s))^T, as the host's psd_whitening).  stats = [rank, log pdet,
// support tol, -log max w, bandwidth, min s, max s, ok].
#include "abc_common.h"

namespace abc {
namespace {

constexpr int FD = 64;

// FT threads: one wave for d <= 16 (its barriers are nearly free), four above
template <int FT>
__global__ __launch_bounds__(FT) void mvn_fit_kernel(const double* __restrict__ mom, int d,
                                                     double scaling, int rule,
                                                     double* __restrict__ cov_out,
                                                     double* __restrict__ evec,
                                                     double* __restrict__ evals,
                                                     double* __restrict__ U,
                                                     double* __restrict__ L,
                                                     double* __restrict__ stats) {
  __shared__ double A[FD][FD + 1];
  __shared__ double V[FD][FD + 1];
  __shared__ double C[FD][FD + 1];   // the covariance, then its Cholesky work
  __shared__ double rc[FD / 2], rs[FD / 2];
  __shared__ int rp[FD / 2], rq[FD / 2];
  __shared__ double lam[FD], srt[FD];
  __shared__ double s_piv;
  __shared__ int s_done;
  const int t = threadIdx.x;
  const double sw = mom[0], sw2 = mom[1];
  const double wmax = mom[2 + d + d * d];
  // bandwidth of the effective sample size 1 / sum w^2 (weights normalised)
  const double ess = 1.0 / sw2;
  const double bw = rule == 1 ? pow(ess, -1.0 / (d + 4))
                              : pow(4.0 / ess / (d + 2), 1.0 / (d + 4));
  const double bw2 = bw * bw;
  const double den = sw - sw2 / sw;
  for (int e = t; e < d * d; e += FT) {
    const int i = e / d, j = e % d;
    // the host's operation order: ((cov_b * sw) / (sw - sw2 / sw)) * bw^2 * scaling
    double c = mom[2 + d + e] * sw;
    c = c / den;
    c = c * bw2;
    c = c * scaling;
    A[i][j] = c;
    C[i][j] = c;
    V[i][j] = i == j ? 1.0 : 0.0;
    cov_out[e] = c;
  }
  __syncthreads();
  // ---- fast path (full rank, certified): Cholesky C = L L^T, W = L^-1 and
  // U = W^T (U U^T = C^-1: any such factor whitens the same quadratic
  // form).  Full rank is certified when lambda_min >= 1 / |W|_F^2 exceeds
  // 4 x scipy's cut-off bound 1e6 eps trace(C) >= 1e6 eps lambda_max: then
  // _PSD would keep every eigenvalue, log pdet = 2 sum log L_jj.  Otherwise
  // (singular or nearly so) the Jacobi path below decides the rank.
  {
    double tr = 0.0;
    for (int i = 0; i < d; ++i) tr += A[i][i];
    const double cutf = 1e6 * 0x1p-52 * tr;
    bool pos = true;
    for (int j = 0; j < d; ++j) {
      if (t == 0) {
        const double sj = C[j][j];
        s_piv = sj > cutf ? sqrt(sj) : 0.0;
        C[j][j] = s_piv;
      }
      __syncthreads();
      const double ljj = s_piv;
      pos = pos && ljj > 0.0;
      for (int i = j + 1 + t; i < d; i += FT) C[i][j] = ljj > 0.0 ? C[i][j] / ljj : 0.0;
      __syncthreads();
      for (int e = t; e < (d - j - 1) * (d - j - 1); e += FT) {
        const int i = j + 1 + e / (d - j - 1), k = j + 1 + e % (d - j - 1);
        if (k <= i) C[i][k] -= C[i][j] * C[k][j];
      }
      __syncthreads();
    }
    double fro = 0.0;
    if (pos) {
      // W = L^-1 (lower), one column per thread, into V
      for (int j = t; j < d; j += FT)
        for (int i = 0; i < d; ++i) {
          double v = i == j ? 1.0 : 0.0;
          if (i < j) { V[i][j] = 0.0; continue; }
          for (int k = j; k < i; ++k) v -= C[i][k] * V[k][j];
          V[i][j] = v / C[i][i];
        }
      __syncthreads();
      for (int i = 0; i < d; ++i)
        for (int j = 0; j <= i; ++j) fro += V[i][j] * V[i][j];
    }
    const bool certified = pos && 1.0 / fro > 4.0 * cutf;
    if (certified) {
      for (int e = t; e < d * d; e += FT) {
        const int i = e / d, j = e % d;
        U[e] = V[j][i];                       // U = W^T = L^-T
        L[e] = j <= i ? C[i][j] : 0.0;
        evec[e] = NAN;                        // not computed on this path
      }
      if (t < d) evals[t] = NAN;
      if (t == 0) {
        double lp = 0.0;
        for (int j = 0; j < d; ++j) lp += log(C[j][j]);
        stats[0] = (double)d;
        stats[1] = 2.0 * lp;
        stats[2] = 1e3 * cutf;
        stats[3] = -log(wmax);
        stats[4] = bw;
        stats[5] = 1.0 / fro;                 // lambda_min lower bound
        stats[6] = tr;                        // lambda_max upper bound
        stats[7] = 1.0;
      }
      return;
    }
    // not certified: the covariance back into C for the semidefinite
    // Cholesky after the eigen-decomposition, V back to the identity
    for (int e = t; e < d * d; e += FT) {
      const int i = e / d, j = e % d;
      C[i][j] = A[i][j];
      V[i][j] = i == j ? 1.0 : 0.0;
    }
    __syncthreads();
  }
  // ---- parallel cyclic Jacobi
  const int n2 = d + (d & 1);           // even number of players (d itself = a dummy)
  const int np = n2 / 2;
  for (int sweep = 0; sweep < 60; ++sweep) {
    // convergence: every off-diagonal below 2^-53 sqrt(|a_pp a_qq|) (or 0)
    int big = 0;
    for (int e = t; e < d * d; e += FT) {
      const int i = e / d, j = e % d;
      if (i < j) {
        const double a = fabs(A[i][j]);
        if (a > 0.0 && a > 0x1p-53 * sqrt(fabs(A[i][i] * A[j][j])) && a > 1e-300) big = 1;
      }
    }
    if (t == 0) s_done = 1;
    __syncthreads();
    if (big) s_done = 0;
    __syncthreads();
    if (s_done) break;
    for (int step = 0; step < n2 - 1; ++step) {
      if (t < np) {
        int p, q;
        if (t == 0) { p = 0; q = 1 + step % (n2 - 1); }
        else {
          p = 1 + (step + t) % (n2 - 1);
          q = 1 + (step - t + n2 - 1) % (n2 - 1);
        }
        if (p > q) { const int x = p; p = q; q = x; }
        double c = 1.0, s = 0.0;
        if (q < d) {
          const double apq = A[p][q];
          if (apq != 0.0) {
            const double tau = (A[q][q] - A[p][p]) / (2.0 * apq);
            const double tt = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
            c = 1.0 / sqrt(1.0 + tt * tt);
            s = tt * c;
          }
        }
        rp[t] = p; rq[t] = q < d ? q : p; rc[t] = c; rs[t] = s;
      }
      __syncthreads();
      // rows: A <- J^T A
      for (int e = t; e < np * d; e += FT) {
        const int k = e / d, j = e % d;
        const int p = rp[k], q = rq[k];
        if (p == q) continue;
        const double c = rc[k], s = rs[k];
        const double a = A[p][j], b = A[q][j];
        A[p][j] = c * a - s * b;
        A[q][j] = s * a + c * b;
      }
      __syncthreads();
      // columns: A <- A J, V <- V J
      for (int e = t; e < np * d; e += FT) {
        const int k = e / d, i = e % d;
        const int p = rp[k], q = rq[k];
        if (p == q) continue;
        const double c = rc[k], s = rs[k];
        const double a = A[i][p], b = A[i][q];
        A[i][p] = c * a - s * b;
        A[i][q] = s * a + c * b;
        const double va = V[i][p], vb = V[i][q];
        V[i][p] = c * va - s * vb;
        V[i][q] = s * va + c * vb;
      }
      __syncthreads();
      if (t < np && rp[t] != rq[t]) { A[rp[t]][rq[t]] = 0.0; A[rq[t]][rp[t]] = 0.0; }
      __syncthreads();
    }
  }
  // ---- eigenpairs by decreasing eigenvalue (ties by index), PSD cut-off
  if (t < d) lam[t] = A[t][t];
  __syncthreads();
  double mx = 0.0, mn = INFINITY;
  bool nan = false;
  for (int i = 0; i < d; ++i) {
    mx = fmax(mx, fabs(lam[i]));
    mn = fmin(mn, lam[i]);
    nan = nan || !(lam[i] == lam[i]);
  }
  const double cut = 1e6 * 0x1p-52 * mx;
  if (t < d) {
    int r = 0;
    for (int j = 0; j < d; ++j) r += (lam[j] > lam[t] || (lam[j] == lam[t] && j < t)) ? 1 : 0;
    srt[r] = lam[t];
    evals[r] = lam[t];
    const bool keep = lam[t] > cut;
    const double f = keep ? 1.0 / sqrt(lam[t]) : 0.0;
    for (int i = 0; i < d; ++i) {
      evec[i * d + r] = V[i][t];
      U[i * d + r] = V[i][t] * f;
    }
  }
  __syncthreads();
  if (t == 0) {
    // log pdet over the kept eigenvalues, in decreasing order
    int rank = 0;
    double lp = 0.0;
    for (int r = 0; r < d; ++r)
      if (srt[r] > cut) { ++rank; lp += log(srt[r]); }
    stats[0] = (double)rank;
    stats[1] = lp;
    stats[2] = 1e3 * cut;
    stats[3] = -log(wmax);
    stats[4] = bw;
    stats[5] = mn;
    stats[6] = mx;
    stats[7] = (nan || mn < -cut) ? 0.0 : 1.0;
  }
  // ---- L L^T = cov, lower: from the eigen factor B = V diag(sqrt(max(s, 0)))
  // (B B^T = cov for any PSD cov, the host's psd_whitening): Householder QR
  // of B^T = Q R, L = R^T with the rows of R signed so diag(L) >= 0.  An
  // unpivoted semidefinite Cholesky zeroing pivots at or below the cut-off
  // left off-diagonal terms up to sqrt(cut c_ii) out of L L^T for a direction
  // whose variance sits near the cut.
  for (int e = t; e < d * d; e += FT) {
    const int k = e / d, i = e % d;
    C[k][i] = V[i][k] * sqrt(fmax(lam[k], 0.0));   // C = B^T
  }
  __syncthreads();
  for (int j = 0; j < d; ++j) {
    if (t == 0) {
      double nrm = 0.0;
      for (int i = j; i < d; ++i) nrm += C[i][j] * C[i][j];
      nrm = sqrt(nrm);
      const double x0 = C[j][j];
      const double alpha = x0 >= 0.0 ? -nrm : nrm;
      // the reflector v = x - alpha e_1 into lam (the eigenvalues are in C)
      double vn = 0.0;
      for (int i = j; i < d; ++i) {
        const double v = (i == j) ? x0 - alpha : C[i][j];
        lam[i] = v;                                   // lam: the reflector
        vn += v * v;
      }
      s_piv = vn;                                     // |v|^2 (0: nothing to do)
    }
    __syncthreads();
    const double vn = s_piv;
    if (vn > 0.0) {
      for (int k = j + t; k < d; k += FT) {
        double dot = 0.0;
        for (int i = j; i < d; ++i) dot += lam[i] * C[i][k];
        const double f = 2.0 * dot / vn;
        for (int i = j; i < d; ++i) C[i][k] -= f * lam[i];
      }
    }
    __syncthreads();
  }
  for (int e = t; e < d * d; e += FT) {
    const int i = e / d, j = e % d;
    L[e] = j <= i ? (C[j][j] < 0.0 ? -C[j][i] : C[j][i]) : 0.0;
  }
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" int abc_mvn_fit(const double* moments, int d, double scaling, int bw_rule,
                           double* cov, double* evec, double* evals, double* U, double* L,
                           double* stats, void* stream) {
  ABC_CHECK_ARG(d >= 1 && d <= FD, "mvn_fit: d=%d outside [1, %d]", d, FD);
  ABC_CHECK_ARG(bw_rule == 0 || bw_rule == 1, "mvn_fit: bw_rule %d", bw_rule);
  ABC_CHECK_ARG(moments && cov && evec && evals && U && L && stats, "mvn_fit: null pointer");
  if (d <= 16)
    hipLaunchKernelGGL(mvn_fit_kernel<64>, dim3(1), dim3(64), 0, as_stream(stream), moments,
                       d, scaling, bw_rule, cov, evec, evals, U, L, stats);
  else
    hipLaunchKernelGGL(mvn_fit_kernel<256>, dim3(1), dim3(256), 0, as_stream(stream), moments,
                       d, scaling, bw_rule, cov, evec, evals, U, L, stats);
  ABC_LAUNCHED();
  return ABC_OK;
}
