// Stochastic acceptance: noise-model kernels, the tempered accept step and the
// temperature-scheme reductions.
//
// Reference:
//   StochasticKernel family   pyabc/distance/kernel.py:18-592
//     NormalKernel :153-226, IndependentNormalKernel :229-303,
//     IndependentLaplaceKernel :306-378, BinomialKernel :381-445,
//     PoissonKernel :448-495, NegativeBinomialKernel :498-552
//   StochasticAcceptor.__call__ acceptor/acceptor.py:434-476
//   AcceptanceRateScheme / match_acceptance_rate epsilon/temperature.py:276-378
//   EssScheme / _ess                            epsilon/temperature.py:660-742
//
// All three are row-parallel and HBM-bound: one pass over [B x S] sum stats
// (kernel), one over [B] densities (accept), one over [R] records per
// objective evaluation (temperature).  Reductions use a fixed grid and a fixed
// combine order, so results are deterministic for a given input.
#include <algorithm>

#include "abc_common.h"

namespace abc {
namespace {

// Philox slot of the acceptance uniform (np.random.uniform in the reference,
// acceptor.py:466); disjoint from the proposal (attempt * 65536 + ...) and the
// simulator (0x40000000 + k/4) slots of abc_sampler.hip.
constexpr uint32_t SLOT_ACCEPT = 0xFFFFFFF0u;

__device__ __forceinline__ double xlogy(double a, double b) {
  return a == 0.0 ? 0.0 : a * log(b);
}
__device__ __forceinline__ double xlog1py(double a, double b) {
  return a == 0.0 ? 0.0 : a * log1p(b);
}

// One noise-model log density per row: log pdf(x_0 | x).
//   kind 0 IndependentNormal  -0.5 * (c + sum diff^2 / par)     (kernel.py:285-303)
//   kind 1 IndependentLaplace -(c + sum |diff| / par)           (kernel.py:361-378)
//   kind 2 Normal             -0.5 * (c + ||diff U||^2)         (scipy logpdf, U [K x r])
//   kind 3 Poisson            sum xlogy(k, mu) - lgamma(k+1) - mu, mu = int(x)
//   kind 4 Binomial(p)        sum log C(n, k) + xlogy(k, p) + xlog1py(n-k, -p), n = int(x)
//   kind 5 NegBinomial(p)     sum lgamma(n+k) - lgamma(k+1) - lgamma(n) + n log p + xlog1py(k, -p)
// c = the host-side constant (log normalisation); x0k[j] observed value of
// kernel element j (kernel key order), cols[j] its column in x.
__global__ __launch_bounds__(256) void kernel_logpdf_kernel(
    const double* __restrict__ x, int64_t B, int S,
    const int32_t* __restrict__ cols, int K, const double* __restrict__ x0k,
    int kind, const double* __restrict__ par, const double* __restrict__ U,
    int r, double c, int ret_lin, double* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* xr = x + b * S;
  double v;
  if (kind == 0 || kind == 1) {
    double s = 0.0;
    for (int j = 0; j < K; ++j) {
      const double df = xr[cols[j]] - x0k[j];
      s += (kind == 0) ? (df * df) / par[j] : fabs(df) / par[j];
    }
    v = (kind == 0) ? -0.5 * (c + s) : -(c + s);
  } else if (kind == 2) {
    double maha = 0.0;
    for (int q = 0; q < r; ++q) {
      double z = 0.0;
      for (int j = 0; j < K; ++j) z += (xr[cols[j]] - x0k[j]) * U[j * r + q];
      maha += z * z;
    }
    v = -0.5 * (c + maha);
  } else {
    const double p = par[0];
    double s = 0.0;
    bool bad = false, zero = false;
    for (int j = 0; j < K; ++j) {
      const double k = x0k[j];                       // integral (host cast)
      const double m = trunc(xr[cols[j]]);           // np.asarray(.., dtype=int)
      if (kind == 3) {                               // Poisson(k; mu = m)
        if (!(m >= 0.0)) { bad = true; continue; }
        if (k < 0.0) { zero = true; continue; }
        s += xlogy(k, m) - lgamma(k + 1.0) - m;
      } else if (kind == 4) {                        // Binomial(k; n = m, p)
        if (!(m >= 0.0)) { bad = true; continue; }
        if (k < 0.0 || k > m) { zero = true; continue; }
        s += lgamma(m + 1.0) - (lgamma(k + 1.0) + lgamma(m - k + 1.0)) +
             xlogy(k, p) + xlog1py(m - k, -p);
      } else {                                       // NegBinomial(k; n = m, p)
        if (!(m > 0.0)) { bad = true; continue; }
        if (k < 0.0) { zero = true; continue; }
        s += lgamma(m + k) - lgamma(k + 1.0) - lgamma(m) + m * log(p) +
             xlog1py(k, -p);
      }
    }
    v = bad ? NAN : (zero ? -INFINITY : s);
  }
  out[b] = ret_lin ? exp(v) : v;
}

// acceptor.py:453-474: acc = (dens / c)^(1/T) (lin) or exp((dens - c) / T)
// (log); accept iff acc >= u, u ~ U[0,1) from the candidate's own stream.
// key = u - acc (<= 0 iff accepted; NaN rejects, as in the reference) feeds
// the order-preserving compaction; accw = acc / min(1, acc) (0 if acc == 0).
__global__ __launch_bounds__(256) void stochastic_accept_kernel(
    const double* __restrict__ dens, int64_t B, double pdf_norm,
    double inv_temp, int scale_log, int apply_iw, uint64_t seed, uint32_t gen,
    int64_t idx0, double* __restrict__ key, double* __restrict__ accw) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double dv = dens[b];
  const double acc = scale_log ? exp((dv - pdf_norm) * inv_temp)
                               : pow(dv / pdf_norm, inv_temp);
  const u32x4 rr = philox((uint64_t)(idx0 + b), SLOT_ACCEPT, gen, seed);
  const double u = uniform53(rr.x, rr.y);
  key[b] = u - acc;
  double w;
  if (acc == 0.0) w = 0.0;
  else if (apply_iw) w = acc / fmin(1.0, acc);
  else w = 1.0;
  accw[b] = w;
}

// ---- temperature-scheme reductions ----------------------------------------
constexpr int TS_T = 256, TS_BLOCKS = 1024;

// l_i = log of the acceptance base: dens - c (log scale) or log(dens / c)
__device__ __forceinline__ double accept_base(double dv, double pdf_norm,
                                              int scale_log) {
  return scale_log ? dv - pdf_norm : log(dv / pdf_norm);
}

// mode 0 (AcceptanceRateScheme): a = sum e^{z_i} min(e^{beta l_i}, 1),
//                                 b = sum e^{z_i}
// mode 1 (EssScheme):            a = sum w_i e^{beta l_i}, b = sum (w_i e^{beta l_i})^2
//                                 with linear weights w = lr
// mode 2:                        a = max (lr_i - lr_sub_i)
// mode 3 (AcceptanceRateScheme, linear weights w = lr):
//                                 a = sum w_i min(e^{beta l_i}, 1), b = sum w_i
// with z_i = lr_i - lr_sub_i - shift (log importance weight t_pd / t_pd_prev
// of record i; lr_sub may be null).
__global__ __launch_bounds__(TS_T) void temper_partial_kernel(
    const double* __restrict__ dens, const double* __restrict__ lr,
    const double* __restrict__ lr_sub, int64_t R, double pdf_norm,
    int scale_log, int mode, double beta, double shift,
    double* __restrict__ part) {
  __shared__ double sa[TS_T / 64], sb[TS_T / 64];
  double a = (mode == 2) ? -INFINITY : 0.0, bsum = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * TS_T + threadIdx.x; i < R;
       i += (int64_t)gridDim.x * TS_T) {
    const double li = lr_sub ? lr[i] - lr_sub[i] : lr[i];
    if (mode == 2) { a = fmax(a, li); continue; }
    const double z = li - shift;
    const double l = accept_base(dens[i], pdf_norm, scale_log);
    // beta == 0: values**0 == 1 even where the base is 0 (temperature.py:741)
    const double bl = (beta == 0.0) ? 0.0 : beta * l;
    if (mode == 3) {
      a += lr[i] * exp(fmin(bl, 0.0));
      bsum += lr[i];
    } else if (mode == 0) {
      const double ez = exp(z);
      a += ez * exp(fmin(bl, 0.0));
      bsum += ez;
    } else {
      const double t = lr[i] * exp(bl);
      a += t;
      bsum += t * t;
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (mode == 2) a = wave_max(a);
  else { a = wave_sum(a); bsum = wave_sum(bsum); }
  if (lane == 0) { sa[wv] = a; sb[wv] = bsum; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double A = sa[0], Bv = sb[0];
    for (int k = 1; k < TS_T / 64; ++k) {
      A = (mode == 2) ? fmax(A, sa[k]) : A + sa[k];
      Bv += sb[k];
    }
    part[2 * blockIdx.x] = A;
    part[2 * blockIdx.x + 1] = Bv;
  }
}

__global__ __launch_bounds__(TS_T) void temper_final_kernel(
    const double* __restrict__ part, int nb, int mode, double* __restrict__ out) {
  __shared__ double sa[TS_T / 64], sb[TS_T / 64];
  double a = (mode == 2) ? -INFINITY : 0.0, bsum = 0.0;
  for (int i = threadIdx.x; i < nb; i += TS_T) {
    a = (mode == 2) ? fmax(a, part[2 * i]) : a + part[2 * i];
    bsum += part[2 * i + 1];
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (mode == 2) a = wave_max(a);
  else { a = wave_sum(a); bsum = wave_sum(bsum); }
  if (lane == 0) { sa[wv] = a; sb[wv] = bsum; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double A = sa[0], Bv = sb[0];
    for (int k = 1; k < TS_T / 64; ++k) {
      A = (mode == 2) ? fmax(A, sa[k]) : A + sa[k];
      Bv += sb[k];
    }
    out[0] = A;
    out[1] = Bv;
  }
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" int abc_kernel_logpdf(const double* x, int64_t B, int S,
                                 const int32_t* cols, int K, const double* x0k,
                                 int kind, const double* par, const double* U,
                                 int r, double c, int ret_lin, double* out,
                                 void* stream) {
  ABC_CHECK_ARG(B >= 0 && S >= 1 && K >= 1, "kernel_logpdf: bad B/S/K");
  ABC_CHECK_ARG(kind >= 0 && kind <= 5, "kernel_logpdf: unknown kind %d", kind);
  ABC_CHECK_ARG(kind != 2 || (U && r >= 1 && r <= K), "kernel_logpdf: bad U/r");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(x && cols && x0k && par && out, "kernel_logpdf: null pointer");
  hipLaunchKernelGGL(kernel_logpdf_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256), 0,
                     as_stream(stream), x, B, S, cols, K, x0k, kind, par, U, r, c,
                     ret_lin, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_stochastic_accept(const double* dens, int64_t B,
                                     double pdf_norm, double temperature,
                                     int scale_log, int apply_iw,
                                     uint64_t seed, uint32_t generation,
                                     int64_t idx0, double* key, double* accw,
                                     void* stream) {
  ABC_CHECK_ARG(B >= 0, "stochastic_accept: B < 0");
  ABC_CHECK_ARG(temperature > 0.0, "stochastic_accept: temperature must be > 0");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(dens && key && accw, "stochastic_accept: null pointer");
  hipLaunchKernelGGL(stochastic_accept_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256),
                     0, as_stream(stream), dens, B, pdf_norm, 1.0 / temperature,
                     scale_log, apply_iw, seed, generation, idx0, key, accw);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" size_t abc_temper_workspace(void) {
  return sizeof(double) * 2 * TS_BLOCKS + 256;
}

extern "C" int abc_temper_sums(const double* dens, const double* lr,
                               const double* lr_sub, int64_t R, double pdf_norm, int scale_log, int mode,
                               double beta, double shift, double* out,
                               void* ws, size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(R >= 0 && mode >= 0 && mode <= 3, "temper_sums: bad R/mode");
  ABC_CHECK_ARG(out && ws && lr && (mode == 2 || dens), "temper_sums: null pointer");
  if (ws_bytes < abc_temper_workspace())
    return set_error(ABC_ERR_WORKSPACE, "temper_sums: workspace too small");
  const int nb = (int)std::min<int64_t>(TS_BLOCKS, std::max<int64_t>(1, ceil_div(R, TS_T)));
  double* part = static_cast<double*>(ws);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(temper_partial_kernel, dim3(nb), dim3(TS_T), 0, s, dens, lr, lr_sub,
                     R, pdf_norm, scale_log, mode, beta, shift, part);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(temper_final_kernel, dim3(1), dim3(TS_T), 0, s, part, nb, mode, out);
  ABC_LAUNCHED();
  return ABC_OK;
}
