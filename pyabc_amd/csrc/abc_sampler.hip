// Batched candidate generation for one ABC-SMC generation.
//
// Reference per-candidate closure (pyabc/smc.py:588-724):
//   _generate_valid_proposal (smc.py:610-662): theta = Transition.rvs(),
//     re-draw while prior pdf == 0; t == 0: theta = prior.rvs()
//   Model.accept (model.py:163-218) -> summary stats -> PNormDistance
//     (distance/distance.py:79-105) -> UniformAcceptor d <= eps
//     (acceptor/acceptor.py:235-244)
// Here each stage is a coalesced kernel over a batch of B candidates whose
// randomness is a pure function of (seed, generation, global index, slot):
// results do not depend on batch size, rank count or scheduling.
#include "abc_common.h"

namespace abc {
namespace {

constexpr double LOG_SQRT_2PI = 0.91893853320467274178;
constexpr uint32_t SLOTS_PER_ATTEMPT = 65536;
constexpr uint32_t SLOT_ANCESTOR = 0;
constexpr uint32_t SLOT_PERTURB = 1;     // 4 normals per slot
constexpr uint32_t SLOT_PRIOR = 32;      // + 512 k + iteration
constexpr uint32_t SLOT_SIM = 0x40000000u;

// normals q .. q+3 of one slot
__device__ __forceinline__ void normals4(uint64_t g, uint32_t slot, uint32_t gen,
                                         uint64_t seed, double n[4]) {
  u32x4 r = philox(g, slot, gen, seed);
  box_muller(r.x, r.y, n[0], n[1]);
  box_muller(r.z, r.w, n[2], n[3]);
}

// ---- priors (scipy.stats pdf conventions, closed support [a, b]) ----------
__device__ double prior_logpdf1(int kind, const double* p, double x) {
  switch (kind) {
    case ABC_PRIOR_FLAT:
      return 0.0;
    case ABC_PRIOR_NORM: {
      double y = (x - p[0]) / p[1];
      return -0.5 * y * y - LOG_SQRT_2PI - log(p[1]);
    }
    case ABC_PRIOR_UNIFORM: {
      double y = (x - p[0]) / p[1];
      return (y >= 0.0 && y <= 1.0) ? -log(p[1]) : -INFINITY;
    }
    case ABC_PRIOR_EXPON: {
      double y = (x - p[0]) / p[1];
      return (y >= 0.0) ? -y - log(p[1]) : -INFINITY;
    }
    case ABC_PRIOR_LAPLACE: {
      double y = (x - p[0]) / p[1];
      return -fabs(y) - log(2.0 * p[1]);
    }
    case ABC_PRIOR_LOGNORM: {  // s, loc, scale
      double y = (x - p[1]) / p[2];
      if (!(y > 0.0)) return -INFINITY;
      double ly = log(y) / p[0];
      return -0.5 * ly * ly - log(p[0] * y) - LOG_SQRT_2PI - log(p[2]);
    }
    case ABC_PRIOR_GAMMA: {  // a, loc, scale
      double a = p[0], y = (x - p[1]) / p[2];
      if (y < 0.0) return -INFINITY;
      if (y == 0.0) return a < 1.0 ? INFINITY : (a == 1.0 ? -log(p[2]) : -INFINITY);
      return (a - 1.0) * log(y) - y - lgamma(a) - log(p[2]);
    }
    case ABC_PRIOR_BETA: {  // a, b, loc, scale
      double a = p[0], b = p[1], y = (x - p[2]) / p[3];
      if (y < 0.0 || y > 1.0) return -INFINITY;
      double lb = lgamma(a) + lgamma(b) - lgamma(a + b);
      double t1 = (a == 1.0) ? 0.0 : (a - 1.0) * log(y);
      double t2 = (b == 1.0) ? 0.0 : (b - 1.0) * log1p(-y);
      return t1 + t2 - lb - log(p[3]);
    }
  }
  return NAN;
}

// Marsaglia-Tsang gamma(a, 1) draw; stream = (g, base + iteration)
__device__ double gamma_draw(double a, uint64_t g, uint32_t base, uint32_t gen,
                             uint64_t seed) {
  double boost = 1.0;
  uint32_t it = 0;
  if (a < 1.0) {
    u32x4 r = philox(g, base + 500, gen, seed);
    boost = pow(uniform01(r.x), 1.0 / a);
    a += 1.0;
  }
  const double dd = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * dd);
  for (; it < 480; ++it) {
    u32x4 r = philox(g, base + it, gen, seed);
    double n0, n1;
    box_muller(r.x, r.y, n0, n1);
    double v = 1.0 + c * n0;
    if (v <= 0.0) continue;
    v = v * v * v;
    double u = uniform01(r.z);
    if (log(u) < 0.5 * n0 * n0 + dd - dd * v + dd * log(v)) return dd * v * boost;
  }
  return dd * boost;  // practically unreachable
}

__device__ double prior_draw1(int kind, const double* p, uint64_t g,
                              uint32_t base, uint32_t gen, uint64_t seed) {
  u32x4 r = philox(g, base, gen, seed);
  double n0, n1;
  switch (kind) {
    case ABC_PRIOR_NORM:
      box_muller(r.x, r.y, n0, n1);
      return p[0] + p[1] * n0;
    case ABC_PRIOR_UNIFORM:
      return p[0] + p[1] * uniform53(r.x, r.y);
    case ABC_PRIOR_EXPON:
      return p[0] - p[1] * log(uniform01(r.x));
    case ABC_PRIOR_LAPLACE: {
      double u = uniform01(r.x) - 0.5;
      return p[0] - p[1] * copysign(1.0, u) * log1p(-2.0 * fabs(u));
    }
    case ABC_PRIOR_LOGNORM:
      box_muller(r.x, r.y, n0, n1);
      return p[1] + p[2] * exp(p[0] * n0);
    case ABC_PRIOR_GAMMA:
      return p[1] + p[2] * gamma_draw(p[0], g, base + 1, gen, seed);
    case ABC_PRIOR_BETA: {
      double x = gamma_draw(p[0], g, base + 1, gen, seed);
      double y = gamma_draw(p[1], g, base + 1 + 256, gen, seed);
      return p[2] + p[3] * x / (x + y);
    }
  }
  return NAN;
}

__device__ __forceinline__ double prior_logpdf(const int32_t* kind,
                                               const double* params, int d,
                                               const double* th) {
  double s = 0.0;
  for (int k = 0; k < d; ++k) s += prior_logpdf1(kind[k], params + 4 * k, th[k]);
  return s;
}

__device__ __forceinline__ int64_t upper_bound(const double* cdf, int64_t N,
                                               double target) {
  int64_t lo = 0, hi = N;  // first index with cdf[idx] > target
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (cdf[mid] > target) hi = mid; else lo = mid + 1;
  }
  return lo < N ? lo : N - 1;
}

// One thread per candidate.  L: [d x d] row-major (per-particle when
// per_particle_L, the LocalTransition Cholesky factors).  D > 0 fixes d at
// compile time so the per-candidate vectors live in registers (D = 0: any
// d <= 64, arrays in scratch).
// Ancestor = first index with cdf > target (np.searchsorted side="right",
// clamped to N - 1).  With a guide table (guide[k] = that index for the
// target k * total / N, abc_cdf_guide) the search starts in a bracket of
// ~3 table bins: O(1) expected instead of log2 N dependent loads.
__device__ __forceinline__ int64_t ancestor_search(const double* __restrict__ cdf,
                                                   const int32_t* __restrict__ guide,
                                                   int64_t N, double total,
                                                   double target) {
  if (guide == nullptr) return upper_bound(cdf, N, target);
  const double step = total / (double)N;
  int64_t k = (int64_t)floor(target / step) - 1;  // t_k < target (one-bin margin)
  k = k < 0 ? 0 : (k > N - 1 ? N - 1 : k);
  int64_t lo = guide[k];
  int64_t hi = k + 3 < N ? (int64_t)guide[k + 3] + 1 : N;  // t_{k+3} > target
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cdf[mid] > target) hi = mid; else lo = mid + 1;
  }
  return lo < N ? lo : N - 1;
}

__global__ void cdf_guide_kernel(const double* __restrict__ cdf, int64_t N,
                                 int32_t* __restrict__ guide) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N) return;
  const double total = cdf[N - 1];
  const double t = (double)k * (total / (double)N);
  guide[k] = (int32_t)upper_bound(cdf, N, t);
}

template <int D, bool PER_PARTICLE_L>
__global__ __launch_bounds__(256) void propose_kernel(
    const double* __restrict__ X, const double* __restrict__ cdf,
    const int32_t* __restrict__ guide, int64_t N,
    int d_rt, const double* __restrict__ L, const int32_t* __restrict__ kind,
    const double* __restrict__ params, uint64_t seed, uint32_t gen,
    int64_t idx0, int64_t B, int max_attempts, double* __restrict__ theta,
    double* __restrict__ lp_out, int64_t* __restrict__ anc_out,
    int32_t* __restrict__ att_out) {
  constexpr int DM = D > 0 ? D : 64;
  const int d = D > 0 ? D : d_rt;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t g = (uint64_t)(idx0 + b);
  double th[DM];
  double lp = -INFINITY;
  int64_t j = -1;
  int att = 0;
  const double total = (X != nullptr) ? cdf[N - 1] : 0.0;
  for (; att < max_attempts; ++att) {
    const uint32_t s0 = (uint32_t)att * SLOTS_PER_ATTEMPT;
    if (X == nullptr) {
#pragma unroll
      for (int k = 0; k < DM; ++k)
        if (k < d)
          th[k] = prior_draw1(kind[k], params + 4 * k, g, s0 + SLOT_PRIOR + 512u * k, gen, seed);
    } else {
      u32x4 r = philox(g, s0 + SLOT_ANCESTOR, gen, seed);
      j = ancestor_search(cdf, guide, N, total, uniform53(r.x, r.y) * total);
      double n[(DM + 3) / 4 * 4];
#pragma unroll
      for (int q = 0; q < DM; q += 4) {
        if (q < d) {
          double n4[4];
          normals4(g, s0 + SLOT_PERTURB + (uint32_t)(q >> 2), gen, seed, n4);
#pragma unroll
          for (int e = 0; e < 4; ++e) n[q + e] = n4[e];
        }
      }
      const double* Lj = PER_PARTICLE_L ? L + j * d * d : L;
#pragma unroll
      for (int k = 0; k < DM; ++k) {
        if (k < d) {
          double acc = X[j * d + k];
#pragma unroll
          for (int q = 0; q < DM; ++q)
            if (q < d) acc += Lj[k * d + q] * n[q];
          th[k] = acc;
        }
      }
    }
    lp = 0.0;
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) lp += prior_logpdf1(kind[k], params + 4 * k, th[k]);
    if (lp > -INFINITY) break;  // prior density > 0 (smc.py:654-656)
  }
#pragma unroll
  for (int k = 0; k < DM; ++k)
    if (k < d) theta[b * d + k] = th[k];
  lp_out[b] = lp;
  if (anc_out) anc_out[b] = j;
  if (att_out) att_out[b] = (lp > -INFINITY) ? att + 1 : max_attempts + 1;
}

template <bool PPL>
void launch_propose(int d, dim3 grid, hipStream_t s, const double* X,
                    const double* cdf, const int32_t* guide, int64_t N, const double* L,
                    const int32_t* kind, const double* params, uint64_t seed,
                    uint32_t gen, int64_t idx0, int64_t B, int max_attempts,
                    double* theta, double* lp, int64_t* anc, int32_t* att) {
#define ABC_PROPOSE_CASE(DD)                                                     \
  case DD:                                                                       \
    hipLaunchKernelGGL((propose_kernel<DD, PPL>), grid, dim3(256), 0, s, X, cdf, \
                       guide, N, d, L, kind, params, seed, gen, idx0, B,         \
                       max_attempts, theta, lp, anc, att);                       \
    break;
  switch (d) {
    ABC_PROPOSE_CASE(1) ABC_PROPOSE_CASE(2) ABC_PROPOSE_CASE(3)
    ABC_PROPOSE_CASE(4) ABC_PROPOSE_CASE(5) ABC_PROPOSE_CASE(6)
    ABC_PROPOSE_CASE(8) ABC_PROPOSE_CASE(10) ABC_PROPOSE_CASE(12)
    ABC_PROPOSE_CASE(16)
    default: ABC_PROPOSE_CASE(0)
  }
#undef ABC_PROPOSE_CASE
}

__global__ void prior_logpdf_kernel(const double* __restrict__ th, int64_t B,
                                    int d, const int32_t* __restrict__ kind,
                                    const double* __restrict__ params,
                                    double* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) out[b] = prior_logpdf(kind, params, d, th + b * d);
}

// x[b,k] = a[k] theta[b, src[k]] + sigma[k] n_k; stat k uses normal k of the
// candidate's simulation stream (slot SLOT_SIM + k/4).
__global__ __launch_bounds__(256) void simulate_lg_kernel(
    const double* __restrict__ theta, int64_t B, int d, int S,
    const int32_t* __restrict__ src, const double* __restrict__ a,
    const double* __restrict__ sigma, uint64_t seed, uint32_t gen,
    int64_t idx0, double* __restrict__ x) {
  // one thread per (candidate, group of 4 stats): coalesced over k
  const int G = (S + 3) >> 2;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * G) return;
  const int64_t b = e / G;
  const int q = (int)(e % G) * 4;
  double n4[4];
  normals4((uint64_t)(idx0 + b), SLOT_SIM + (uint32_t)(q >> 2), gen, seed, n4);
  for (int t = 0; t < 4 && q + t < S; ++t) {
    const int k = q + t;
    x[b * S + k] = a[k] * theta[b * d + src[k]] + sigma[k] * n4[t];
  }
}

// ---- PNormDistance ---------------------------------------------------------
__device__ __forceinline__ double pterm(double v, double p) {
  return (p == 1.0) ? v : (p == 2.0 ? v * v : pow(v, p));
}

__global__ __launch_bounds__(256) void pnorm_row_kernel(
    const double* __restrict__ x, int64_t B, int S,
    const double* __restrict__ x0, const double* __restrict__ wf, double p,
    double* __restrict__ d) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* xr = x + b * S;
  double s = 0.0;
  if (isinf(p)) {
    for (int k = 0; k < S; ++k) s = fmax(s, fabs(wf[k] * (xr[k] - x0[k])));
    d[b] = s;
  } else {
    for (int k = 0; k < S; ++k) s += pterm(fabs(wf[k] * (xr[k] - x0[k])), p);
    d[b] = (p == 1.0) ? s : (p == 2.0 ? sqrt(s) : pow(s, 1.0 / p));
  }
}

// wide rows: lanes stride over k (coalesced), each wave takes PW_ROWS rows at
// once so that many row loads are in flight per lane (one row per wave left
// the HBM stream latency-bound at ~40% of peak).  Per row the order of the
// sum is unchanged: lane-strided partials, then the wave tree.
constexpr int PW_ROWS = 8;
__global__ __launch_bounds__(256) void pnorm_wave_kernel(
    const double* __restrict__ x, int64_t B, int S,
    const double* __restrict__ x0, const double* __restrict__ wf, double p,
    double* __restrict__ d) {
  const int lane = threadIdx.x & 63;
  const int64_t b0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * PW_ROWS;
  if (b0 >= B) return;  // whole wave
  const bool inf = isinf(p);
  double s[PW_ROWS];
#pragma unroll
  for (int r = 0; r < PW_ROWS; ++r) s[r] = 0.0;
  for (int k = lane; k < S; k += 64) {
    const double wk = wf[k], ck = x0[k];
    double v[PW_ROWS];
#pragma unroll
    for (int r = 0; r < PW_ROWS; ++r) v[r] = b0 + r < B ? x[(b0 + r) * S + k] : ck;
#pragma unroll
    for (int r = 0; r < PW_ROWS; ++r) {
      const double a = fabs(wk * (v[r] - ck));
      s[r] = inf ? fmax(s[r], a) : s[r] + pterm(a, p);
    }
  }
#pragma unroll
  for (int r = 0; r < PW_ROWS; ++r) {
    const double t = inf ? wave_max(s[r]) : wave_sum(s[r]);
    if (lane == 0 && b0 + r < B)
      d[b0 + r] = inf ? t : ((p == 1.0) ? t : (p == 2.0 ? sqrt(t) : pow(t, 1.0 / p)));
  }
}

// ---- order-preserving accept compaction ------------------------------------
constexpr int CT_T = 256, CT_I = 8, CT_TILE = CT_T * CT_I;

__device__ int64_t block_exscan_i64(int64_t v, int64_t* sh, int64_t& total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < CT_T; o <<= 1) {
    int64_t add = (t >= o) ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  total = sh[CT_T - 1];
  int64_t incl = sh[t];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(CT_T) void accept_count_kernel(
    const double* __restrict__ d, int64_t B, double eps,
    int64_t* __restrict__ tile_cnt) {
  __shared__ int64_t sh[CT_T];
  const int64_t base = (int64_t)blockIdx.x * CT_TILE + threadIdx.x * CT_I;
  int64_t c = 0;
  for (int k = 0; k < CT_I; ++k)
    if (base + k < B && d[base + k] <= eps) ++c;
  int64_t tot;
  block_exscan_i64(c, sh, tot);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(CT_T) void accept_scan_kernel(
    int64_t* __restrict__ tile_cnt, int64_t n, int64_t* __restrict__ count) {
  __shared__ int64_t sh[CT_T];
  const int64_t per = (n + CT_T - 1) / CT_T;
  const int64_t b0 = threadIdx.x * per;
  int64_t s = 0;
  for (int64_t k = 0; k < per; ++k)
    if (b0 + k < n) s += tile_cnt[b0 + k];
  int64_t tot;
  int64_t off = block_exscan_i64(s, sh, tot);
  for (int64_t k = 0; k < per; ++k)
    if (b0 + k < n) { int64_t v = tile_cnt[b0 + k]; tile_cnt[b0 + k] = off; off += v; }
  if (threadIdx.x == 0) *count = tot;
}

__global__ __launch_bounds__(CT_T) void accept_write_kernel(
    const double* __restrict__ d, int64_t B, double eps,
    const int64_t* __restrict__ tile_off, int64_t* __restrict__ idx) {
  __shared__ int64_t sh[CT_T];
  const int64_t base = (int64_t)blockIdx.x * CT_TILE + threadIdx.x * CT_I;
  int64_t c = 0;
  for (int k = 0; k < CT_I; ++k)
    if (base + k < B && d[base + k] <= eps) ++c;
  int64_t tot;
  int64_t pos = block_exscan_i64(c, sh, tot) + tile_off[blockIdx.x];
  for (int k = 0; k < CT_I; ++k)
    if (base + k < B && d[base + k] <= eps) idx[pos++] = base + k;
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" int abc_cdf_guide(const double* cdf, int64_t N, int32_t* guide,
                             void* stream) {
  ABC_CHECK_ARG(N >= 1 && N < (1ll << 31), "cdf_guide: bad N");
  ABC_CHECK_ARG(cdf && guide, "cdf_guide: null pointer");
  hipLaunchKernelGGL(cdf_guide_kernel, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0,
                     as_stream(stream), cdf, N, guide);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_propose(const double* X, const double* cdf,
                           const int32_t* guide, int64_t N,
                           int d, const double* L, const int32_t* prior_kind,
                           const double* prior_params, uint64_t seed,
                           uint32_t generation, int64_t idx0, int64_t B,
                           int max_attempts, double* theta,
                           double* prior_logpdf, int64_t* ancestor,
                           int32_t* attempts, void* stream) {
  ABC_CHECK_ARG(d >= 1 && d <= 64 && B >= 0 && max_attempts >= 1, "propose: bad d/B");
  ABC_CHECK_ARG(max_attempts < (1 << 15), "propose: max_attempts too large");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(theta && prior_logpdf && prior_kind && prior_params, "propose: null pointer");
  ABC_CHECK_ARG(X == nullptr || (cdf && L && N >= 1), "propose: population needs cdf, L, N");
  launch_propose<false>(d, dim3((unsigned)ceil_div(B, 256)), as_stream(stream), X, cdf,
                        guide, N, L, prior_kind, prior_params, seed, generation, idx0, B,
                        max_attempts, theta, prior_logpdf, ancestor, attempts);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_local_propose(const double* X, const double* cdf,
                                 const int32_t* guide, int64_t N,
                                 int d, const double* chol,
                                 const int32_t* prior_kind,
                                 const double* prior_params, uint64_t seed,
                                 uint32_t generation, int64_t idx0, int64_t B,
                                 int max_attempts, double* theta,
                                 double* prior_logpdf, int64_t* ancestor,
                                 int32_t* attempts, void* stream) {
  ABC_CHECK_ARG(d >= 1 && d <= 64 && B >= 0 && max_attempts >= 1, "local_propose: bad d/B");
  ABC_CHECK_ARG(max_attempts < (1 << 15), "local_propose: max_attempts too large");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(X && cdf && chol && N >= 1 && theta && prior_logpdf && prior_kind &&
                prior_params, "local_propose: null pointer");
  launch_propose<true>(d, dim3((unsigned)ceil_div(B, 256)), as_stream(stream), X, cdf,
                       guide, N, chol, prior_kind, prior_params, seed, generation, idx0, B,
                       max_attempts, theta, prior_logpdf, ancestor, attempts);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_prior_logpdf(const double* theta, int64_t B, int d,
                                const int32_t* prior_kind,
                                const double* prior_params, double* out,
                                void* stream) {
  ABC_CHECK_ARG(d >= 1 && d <= 64 && B >= 0, "prior_logpdf: bad d/B");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(theta && prior_kind && prior_params && out, "prior_logpdf: null pointer");
  hipLaunchKernelGGL(prior_logpdf_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256), 0,
                     as_stream(stream), theta, B, d, prior_kind, prior_params, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_simulate_linear_gaussian(const double* theta, int64_t B,
                                            int d, int S, const int32_t* src,
                                            const double* a,
                                            const double* sigma, uint64_t seed,
                                            uint32_t generation, int64_t idx0,
                                            double* x, void* stream) {
  ABC_CHECK_ARG(d >= 1 && S >= 1 && B >= 0, "simulate: bad d/S/B");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(theta && src && a && sigma && x, "simulate: null pointer");
  const int64_t n = B * ((S + 3) / 4);
  hipLaunchKernelGGL(simulate_lg_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                     as_stream(stream), theta, B, d, S, src, a, sigma, seed, generation,
                     idx0, x);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_pnorm(const double* x, int64_t B, int S, const double* x0,
                         const double* wf, double p, double* d, void* stream) {
  ABC_CHECK_ARG(S >= 1 && B >= 0 && p >= 1.0, "pnorm: bad S/B/p");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(x && x0 && wf && d, "pnorm: null pointer");
  if (S <= 32)
    hipLaunchKernelGGL(pnorm_row_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256), 0,
                       as_stream(stream), x, B, S, x0, wf, p, d);
  else
    hipLaunchKernelGGL(pnorm_wave_kernel, dim3((unsigned)ceil_div(B, 4 * PW_ROWS)), dim3(256), 0,
                       as_stream(stream), x, B, S, x0, wf, p, d);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" size_t abc_compact_workspace(int64_t B) {
  return align_up(sizeof(int64_t) * (size_t)ceil_div(B > 0 ? B : 1, CT_TILE), 256) + 256;
}

extern "C" int abc_accept_compact(const double* d, int64_t B, double eps,
                                  int64_t* idx, int64_t* count, void* ws,
                                  size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(B >= 0, "compact: B < 0");
  ABC_CHECK_ARG(count && ws, "compact: null pointer");
  if (ws_bytes < abc_compact_workspace(B))
    return set_error(ABC_ERR_WORKSPACE, "compact: workspace too small");
  hipStream_t s = as_stream(stream);
  if (B == 0) {
    ABC_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), s));
    return ABC_OK;
  }
  ABC_CHECK_ARG(d && idx, "compact: null pointer");
  const int64_t nt = ceil_div(B, CT_TILE);
  int64_t* tiles = static_cast<int64_t*>(ws);
  hipLaunchKernelGGL(accept_count_kernel, dim3((unsigned)nt), dim3(CT_T), 0, s, d, B, eps, tiles);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(accept_scan_kernel, dim3(1), dim3(CT_T), 0, s, tiles, nt, count);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(accept_write_kernel, dim3((unsigned)nt), dim3(CT_T), 0, s, d, B, eps,
                     tiles, idx);
  ABC_LAUNCHED();
  return ABC_OK;
}
