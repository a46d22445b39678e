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
#include "abc_candidate.h"

namespace abc {
namespace {

__global__ void cdf_guide_kernel(const double* __restrict__ cdf, int64_t N,
                                 int32_t* __restrict__ guide) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N) return;
  const double total = cdf[N - 1];
  const double t = (double)k * (total / (double)N);
  guide[k] = (int32_t)upper_bound(cdf, N, t);
}

template <int D, int MODE>
__global__ __launch_bounds__(256) void propose_kernel(
    ProposalArgs A, int64_t idx0, int64_t B, double* __restrict__ theta,
    double* __restrict__ lp_out, int64_t* __restrict__ anc_out,
    int32_t* __restrict__ att_out) {
  constexpr int DM = D > 0 ? D : 64;
  __shared__ BlockConsts C;
  stage_block_consts<D, MODE>(C, A, nullptr, nullptr);
  const int d = D > 0 ? D : A.d;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double th[DM];
  int64_t j;
  const int att = propose_one<D, MODE>(A, C, (uint64_t)(idx0 + b), th, j);
#pragma unroll
  for (int k = 0; k < (D > 0 ? D : d); ++k) theta[b * d + k] = th[k];
  lp_out[b] = att <= A.max_attempts ? prior_logpdf(A.kind, A.params, d, th) : -INFINITY;
  if (anc_out) anc_out[b] = j;
  if (att_out) att_out[b] = att;
}

// d > 64 (the register kernels hold theta in d registers): theta is
// accumulated in its output row, the support box of the d coordinates sits in
// dynamic LDS; the streams, the per-coordinate fma order and the re-draw loop
// are propose_one's (abc_candidate.h), the ancestor the cdf search's.
template <int MODE>
__global__ __launch_bounds__(256) void propose_wide_kernel(
    ProposalArgs A, int64_t idx0, int64_t B, double* __restrict__ theta,
    double* __restrict__ lp_out, int64_t* __restrict__ anc_out,
    int32_t* __restrict__ att_out) {
  extern __shared__ double box[];   // [d][lo, hi]
  const int d = A.d;
  for (int k = threadIdx.x >> 6; k < d; k += blockDim.x >> 6)
    support_bounds_wave(A.kind[k], A.params + 4 * k, box + 2 * k);
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t g = (uint64_t)(idx0 + b);
  double* th = theta + b * d;
  int64_t j = -1;
  int used = A.max_attempts + 1;
  const double total = MODE != PROP_PRIOR ? A.cdf[A.N - 1] : 0.0;
  for (int att = 0; att < A.max_attempts; ++att) {
    const uint32_t s0 = (uint32_t)att * SLOTS_PER_ATTEMPT;
    if (MODE == PROP_PRIOR) {
      for (int k = 0; k < d; ++k)
        th[k] = prior_draw1(A.kind[k], A.params + 4 * k, g, s0 + SLOT_PRIOR + 512u * k, A.gen,
                            A.seed);
    } else {
      const u32x4 ra = philox(g, s0 + SLOT_ANCESTOR, A.gen, A.seed);
      u32x4 r = ra;
      const double target = uniform53(ra.x, ra.y) * total;
      j = ancestor_search(A.cdf, A.guide, A.N, total, target);
      const double* Lj = MODE == PROP_LOCAL ? A.L + j * d * d : A.L;
      for (int k = 0; k < d; ++k) th[k] = 0.0;
      for (int q = 0; q < d; q += 2) {
        uint32_t wa, wb;
        perturb_words(q >> 1, ra, r, g, s0, A.gen, A.seed, wa, wb);
        double n0, n1;
        box_muller(wa, wb, n0, n1);
        const bool two = q + 1 < d;
        for (int k = q; k < d; ++k) {
          th[k] = fma(Lj[k * d + q], n0, th[k]);
          if (two && k >= q + 1) th[k] = fma(Lj[k * d + q + 1], n1, th[k]);
        }
      }
      for (int k = 0; k < d; ++k) th[k] = A.X[j * d + k] + th[k];
    }
    bool ok = true;
    for (int k = 0; k < d; ++k) ok = ok & (box[2 * k] <= th[k]) & (th[k] <= box[2 * k + 1]);
    if (ok) { used = att + 1; break; }
  }
  lp_out[b] = used <= A.max_attempts ? prior_logpdf(A.kind, A.params, d, th) : -INFINITY;
  if (anc_out) anc_out[b] = j;
  if (att_out) att_out[b] = used;
}

template <bool PPL>
void launch_propose(int d, dim3 grid, hipStream_t s, const double* X,
                    const double* cdf, const int32_t* guide, int64_t N, const double* L,
                    const int32_t* kind, const double* params, uint64_t seed,
                    uint32_t gen, int64_t idx0, int64_t B, int max_attempts,
                    double* theta, double* lp, int64_t* anc, int32_t* att) {
  const ProposalArgs A{X, cdf, guide, N, L, kind, params, d, max_attempts, seed, gen};
  if (d > 64) {
    const size_t lds = sizeof(double) * 2 * (size_t)d;
    if (X == nullptr)
      hipLaunchKernelGGL((propose_wide_kernel<PROP_PRIOR>), grid, dim3(256), lds, s, A, idx0, B,
                         theta, lp, anc, att);
    else
      hipLaunchKernelGGL((propose_wide_kernel<PPL ? PROP_LOCAL : PROP_MVN>), grid, dim3(256),
                         lds, s, A, idx0, B, theta, lp, anc, att);
    return;
  }
#define ABC_PROPOSE_CASE(DD)                                                        \
  case DD:                                                                          \
    if (X == nullptr)                                                               \
      hipLaunchKernelGGL((propose_kernel<DD, PROP_PRIOR>), grid, dim3(256), 0, s, A, \
                         idx0, B, theta, lp, anc, att);                             \
    else                                                                            \
      hipLaunchKernelGGL((propose_kernel<DD, PPL ? PROP_LOCAL : PROP_MVN>), grid,    \
                         dim3(256), 0, s, A, idx0, B, theta, lp, anc, att);         \
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

// u[b] in (0, 1) from word 0..1 of candidate b's prior stream for dimension
// k in the attempt it accepted (slot (att - 1) 65536 + SLOT_PRIOR + 512 k):
// the uniform an ABC_PRIOR_HOST coordinate's t = 0 draw ppf(u) is made from
__global__ void prior_uniforms_kernel(const int32_t* __restrict__ att, int64_t B, int k,
                                      uint64_t seed, uint32_t gen, int64_t idx0,
                                      double* __restrict__ u) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int a = att ? (att[b] > 0 ? att[b] - 1 : 0) : 0;
  const u32x4 r = philox((uint64_t)(idx0 + b),
                         (uint32_t)a * SLOTS_PER_ATTEMPT + SLOT_PRIOR + 512u * (uint32_t)k,
                         gen, seed);
  u[b] = ((double)(r.x >> 5) * 67108864.0 + (double)(r.y >> 6) + 0.5) *
         (1.0 / 9007199254740992.0);
}

// x[b,k] = a[k] theta[b, src[k]] + sigma[k] n_k; stat k uses normal k of the
// candidate's simulation stream (slot SLOT_SIM + k/4).
__global__ __launch_bounds__(256) void simulate_lg_kernel(
    const double* __restrict__ theta, int64_t B, int d, int S,
    const int32_t* __restrict__ src, const double* __restrict__ a,
    const double* __restrict__ sigma, uint64_t seed, uint32_t gen,
    int64_t idx0, double* __restrict__ x) {
  // one thread per (candidate, group of 4 stats): coalesced over k
  __shared__ float sbmt[BM_TAB_SIZE];
  stage_bm_tab(sbmt);
  const int G = (S + 3) >> 2;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * G) return;
  const int64_t b = e / G;
  const int q = (int)(e % G) * 4;
  double n4[4];
  normals4((uint64_t)(idx0 + b), SLOT_SIM + (uint32_t)(q >> 2), gen, seed, n4, 4, sbmt);
  for (int t = 0; t < 4 && q + t < S; ++t) {
    const int k = q + t;
    x[b * S + k] = a[k] * theta[b * d + src[k]] + sigma[k] * n4[t];
  }
}

// ---- PNormDistance (pterm / pnorm_acc: abc_candidate.h) -------------------

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

__global__ void mask_gave_up_kernel(double* __restrict__ d, const int32_t* __restrict__ att,
                                    int64_t B, int max_attempts, double value) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B && att[b] > max_attempts) d[b] = value;
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" int abc_mask_gave_up(double* dist, const int32_t* attempts, int64_t B,
                                int max_attempts, double value, void* stream) {
  ABC_CHECK_ARG(B >= 0, "mask_gave_up: B < 0");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(dist && attempts, "mask_gave_up: null pointer");
  hipLaunchKernelGGL(mask_gave_up_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256), 0,
                     as_stream(stream), dist, attempts, B, max_attempts, value);
  ABC_LAUNCHED();
  return ABC_OK;
}

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
  ABC_CHECK_ARG(d >= 1 && d <= ABC_MAX_D && B >= 0 && max_attempts >= 1, "propose: bad d/B");
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
  ABC_CHECK_ARG(d >= 1 && d <= ABC_MAX_D && B >= 0 && max_attempts >= 1, "local_propose: bad d/B");
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
  ABC_CHECK_ARG(d >= 1 && d <= ABC_MAX_D && B >= 0, "prior_logpdf: bad d/B");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(theta && prior_kind && prior_params && out, "prior_logpdf: null pointer");
  hipLaunchKernelGGL(prior_logpdf_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256), 0,
                     as_stream(stream), theta, B, d, prior_kind, prior_params, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_prior_uniforms(const int32_t* attempts, double* u, int64_t B, int k,
                                  uint64_t seed, uint32_t generation, int64_t idx0,
                                  void* stream) {
  ABC_CHECK_ARG(B >= 0 && k >= 0 && k < 64, "prior_uniforms: bad B/k");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(u, "prior_uniforms: null pointer");
  hipLaunchKernelGGL(prior_uniforms_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256), 0,
                     as_stream(stream), attempts, B, k, seed, generation, idx0, u);
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
