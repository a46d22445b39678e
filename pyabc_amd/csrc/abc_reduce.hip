// Deterministic fp64 reductions and scans for the fits and the sampler.
//
// abc_weighted_moments: the numpy work inside
//   MultivariateNormalTransition.fit (pyabc/transition/multivariatenormal.py:72-83)
//   -> smart_cov (pyabc/transition/util.py:4-16) = np.cov(X, aweights=w).
// abc_inclusive_scan_f64: cumulative weights for the ancestor draw of
//   MultivariateNormalTransition.rvs (multivariatenormal.py:85-91).
// All reductions use a fixed block count and a fixed combine order, so the
// results are bitwise reproducible run to run (no float atomics).
#include "abc_common.h"

namespace abc {
namespace {

constexpr int MOM_BLOCKS = 256;
constexpr int MOM_ROWS = 64;  // rows staged in LDS per step

// pass 1: columns (w, w^2, w x_0 .. w x_{d-1})
__global__ __launch_bounds__(256) void moments1_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t N,
    int d, double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* xs = lds;                    // [MOM_ROWS][d]
  double* ws = lds + MOM_ROWS * d;     // [MOM_ROWS]
  const int ncol = 2 + d;
  double acc[2] = {0.0, 0.0};          // this thread's columns c0, c0+256
  for (int64_t r0 = (int64_t)blockIdx.x * MOM_ROWS; r0 < N;
       r0 += (int64_t)gridDim.x * MOM_ROWS) {
    const int nr = (int)((N - r0) < MOM_ROWS ? (N - r0) : MOM_ROWS);
    __syncthreads();
    for (int e = threadIdx.x; e < nr * d; e += blockDim.x) xs[e] = X[r0 * d + e];
    for (int e = threadIdx.x; e < nr; e += blockDim.x) ws[e] = w[r0 + e];
    __syncthreads();
    for (int h = 0; h < 2; ++h) {
      const int c = threadIdx.x + 256 * h;
      if (c >= ncol) continue;
      double s = 0.0;
      for (int r = 0; r < nr; ++r) {
        const double wr = ws[r];
        s += (c == 0) ? wr : (c == 1 ? wr * wr : wr * xs[r * d + (c - 2)]);
      }
      acc[h] += s;
    }
  }
  for (int h = 0; h < 2; ++h) {
    const int c = threadIdx.x + 256 * h;
    if (c < ncol) part[(int64_t)blockIdx.x * ncol + c] = acc[h];
  }
}

__global__ void moments1_final(const double* __restrict__ part, int nblk,
                               int d, double* __restrict__ out) {
  const int ncol = 2 + d;
  for (int c = threadIdx.x; c < ncol; c += blockDim.x) {
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * ncol + c];
    out[c] = s;  // 0: sum w, 1: sum w^2, 2+q: sum w x_q (mean fixed below)
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double sw = out[0];
    for (int q = 0; q < d; ++q) out[2 + q] = out[2 + q] / sw;
  }
}

// max w for the generic path (single block; fixed order)
__global__ void mom1_max_generic(const double* __restrict__ w, int64_t N,
                                 double* __restrict__ out) {
  __shared__ double sh[256];
  double m = 0.0;
  for (int64_t r = threadIdx.x; r < N; r += blockDim.x) m = fmax(m, w[r]);
  sh[threadIdx.x] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int t = 1; t < 256; ++t) m = fmax(m, sh[t]);
    *out = m;
  }
}

// pass 2: sum w (x - mean)(x - mean)^T, one (a, b) entry per thread slot
__global__ __launch_bounds__(256) void moments2_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t N,
    int d, const double* __restrict__ mom, double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* xs = lds;                    // centred rows
  double* ws = lds + MOM_ROWS * d;
  const double* mean = mom + 2;
  const int npair = d * d;
  double acc[16];
  for (int h = 0; h < 16; ++h) acc[h] = 0.0;
  for (int64_t r0 = (int64_t)blockIdx.x * MOM_ROWS; r0 < N;
       r0 += (int64_t)gridDim.x * MOM_ROWS) {
    const int nr = (int)((N - r0) < MOM_ROWS ? (N - r0) : MOM_ROWS);
    __syncthreads();
    for (int e = threadIdx.x; e < nr * d; e += blockDim.x)
      xs[e] = X[r0 * d + e] - mean[e % d];
    for (int e = threadIdx.x; e < nr; e += blockDim.x) ws[e] = w[r0 + e];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      const int pidx = threadIdx.x + 256 * h;
      if (pidx >= npair) break;
      const int a = pidx / d, b = pidx % d;
      double s = 0.0;
      for (int r = 0; r < nr; ++r) s += ws[r] * xs[r * d + a] * xs[r * d + b];
      acc[h] += s;
    }
  }
#pragma unroll
  for (int h = 0; h < 16; ++h) {
    const int pidx = threadIdx.x + 256 * h;
    if (pidx < npair) part[(int64_t)blockIdx.x * npair + pidx] = acc[h];
  }
}

__global__ void moments2_final(const double* __restrict__ part, int nblk,
                               int d, double* __restrict__ out) {
  const int npair = d * d;
  const double sw = out[0];
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < npair; c += gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * npair + c];
    out[2 + d + c] = s / sw;
  }
}

// ---- wide path (d > 64): one column / one (a, b) entry per thread ---------
// Rows are read straight from X (a block's threads read consecutive columns
// of the same row: coalesced; the pair pass re-reads a row from cache).
// Fixed block counts and combine order, as above.
__global__ __launch_bounds__(256) void moments1_wide(const double* __restrict__ X,
                                                     const double* __restrict__ w,
                                                     int64_t N, int d,
                                                     double* __restrict__ part) {
  const int ncol = 2 + d;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= ncol) return;
  double acc = 0.0;
  for (int64_t r = blockIdx.x; r < N; r += gridDim.x) {
    const double wr = w[r];
    acc += (c == 0) ? wr : (c == 1 ? wr * wr : wr * X[r * d + (c - 2)]);
  }
  part[(int64_t)blockIdx.x * ncol + c] = acc;
}

__global__ __launch_bounds__(256) void moments2_wide(const double* __restrict__ X,
                                                     const double* __restrict__ w,
                                                     int64_t N, int d,
                                                     const double* __restrict__ mom,
                                                     double* __restrict__ part) {
  const int64_t npair = (int64_t)d * d;
  const int64_t pidx = (int64_t)blockIdx.y * 256 + threadIdx.x;
  if (pidx >= npair) return;
  const int a = (int)(pidx / d), b = (int)(pidx % d);
  const double ma = mom[2 + a], mb = mom[2 + b];
  double acc = 0.0;
  for (int64_t r = blockIdx.x; r < N; r += gridDim.x)
    acc += w[r] * (X[r * d + a] - ma) * (X[r * d + b] - mb);
  part[(int64_t)blockIdx.x * npair + pidx] = acc;
}

// row blocks of the wide path: the pair partials stay <= 2^24 doubles
int wide_blocks(int64_t N, int d) {
  const int64_t cap = ((int64_t)1 << 24) / ((int64_t)d * d);
  int64_t nb = cap < MOM_BLOCKS ? cap : MOM_BLOCKS;
  if (nb < 1) nb = 1;
  return (int)(N < nb ? N : nb);
}

// ---- fast path: d fixed at compile time, one row per thread ----------------
// Rows are strided over the grid; each thread keeps its row sums in
// registers; blocks reduce by wave butterflies + LDS in fixed order (bitwise
// reproducible); the final kernels reduce the block partials by a fixed tree.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// sum over the block of NV per-thread values -> out[0..NV) (thread 0 writes)
template <int NV>
__device__ __forceinline__ void block_sums(const double (&v)[NV], double* sh,
                                           double* __restrict__ out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const double t = wave_sum(v[c]);
    if (lane == 0) sh[wv * NV + c] = t;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < NV; c += blockDim.x)
    out[c] = (sh[c] + sh[NV + c]) + (sh[2 * NV + c] + sh[3 * NV + c]);
}

template <int D>
__global__ __launch_bounds__(256) void mom1_fast(const double* __restrict__ X,
                                                 const double* __restrict__ w,
                                                 int64_t N, double* __restrict__ part,
                                                 double* __restrict__ pmax) {
  constexpr int NV = D + 2;
  __shared__ double sh[4 * NV];
  __shared__ double shm[4];
  double v[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) v[c] = 0.0;
  double mx = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N;
       r += (int64_t)gridDim.x * blockDim.x) {
    const double wr = w[r];
    v[0] += wr;
    v[1] += wr * wr;
    mx = fmax(mx, wr);
#pragma unroll
    for (int q = 0; q < D; ++q) v[2 + q] += wr * X[r * D + q];
  }
  block_sums<NV>(v, sh, part + (int64_t)blockIdx.x * NV);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) shm[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) pmax[blockIdx.x] = fmax(fmax(shm[0], shm[1]), fmax(shm[2], shm[3]));
}

// out[c] = sum over nblk partials of column c (ncol columns), one wave per
// column, fixed order; `scale_from` >= 0 divides columns >= scale_from by
// out[0] (already final) -- used for the mean / covariance normalisation
__global__ __launch_bounds__(256) void mom_final(const double* __restrict__ part,
                                                 int nblk, int ncol, int col0,
                                                 double* __restrict__ out,
                                                 bool divide) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= ncol) return;
  double s = 0.0;
  for (int b = lane; b < nblk; b += 64) s += part[(int64_t)b * ncol + c];
  s = wave_sum(s);
  if (lane == 0) out[col0 + c] = divide ? s / out[0] : s;
}

__global__ void mom_max_final(const double* __restrict__ pmax, int nblk,
                              double* __restrict__ out) {
  double m = 0.0;
  for (int b = threadIdx.x; b < nblk; b += 64) m = fmax(m, pmax[b]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  if (threadIdx.x == 0) *out = m;
}

template <int D>
__global__ __launch_bounds__(256) void mom2_fast(const double* __restrict__ X,
                                                 const double* __restrict__ w,
                                                 int64_t N,
                                                 const double* __restrict__ mom,
                                                 double* __restrict__ part) {
  constexpr int NV = D * (D + 1) / 2;  // upper triangle, row-major
  __shared__ double sh[4 * NV];
  double mean[D];
#pragma unroll
  for (int q = 0; q < D; ++q) mean[q] = mom[2 + q] / mom[0];  // raw sums here
  double v[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) v[c] = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N;
       r += (int64_t)gridDim.x * blockDim.x) {
    const double wr = w[r];
    double xc[D];
#pragma unroll
    for (int q = 0; q < D; ++q) xc[q] = X[r * D + q] - mean[q];
    int c = 0;
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
      for (int b = a; b < D; ++b) v[c++] += wr * xc[a] * xc[b];
  }
  block_sums<NV>(v, sh, part + (int64_t)blockIdx.x * NV);
}

// upper-triangle sums -> full symmetric d x d, divided by sum w; means
// divided by sum w (same fp64 division as the generic path)
template <int D>
__global__ void mom2_expand(const double* __restrict__ tri, double* __restrict__ out) {
  const int t = threadIdx.x;
  if (t < D) out[2 + t] = out[2 + t] / out[0];
  if (t >= D * D) return;
  int a = t / D, b = t % D;
  if (a > b) { const int x = a; a = b; b = x; }
  const int c = a * D - a * (a - 1) / 2 + (b - a);
  out[2 + D + t] = tri[c] / out[0];
}

template <int D>
void moments_fast(const double* X, const double* w, int64_t N, double* out,
                  double* p1, double* p2, double* pmax, double* tri, hipStream_t s) {
  constexpr int NV1 = D + 2, NV2 = D * (D + 1) / 2;
  const int nblk = (int)(ceil_div(N, 256) < MOM_BLOCKS ? ceil_div(N, 256) : MOM_BLOCKS);
  hipLaunchKernelGGL(mom1_fast<D>, dim3(nblk), dim3(256), 0, s, X, w, N, p1, pmax);
  // raw column sums (sum w, sum w^2, sum w x); means are divided in mom2
  hipLaunchKernelGGL(mom_final, dim3((unsigned)ceil_div(NV1, 4)), dim3(256), 0, s, p1, nblk,
                     NV1, 0, out, false);
  hipLaunchKernelGGL(mom_max_final, dim3(1), dim3(64), 0, s, pmax, nblk,
                     out + 2 + D + D * D);
  hipLaunchKernelGGL(mom2_fast<D>, dim3(nblk), dim3(256), 0, s, X, w, N, out, p2);
  hipLaunchKernelGGL(mom_final, dim3((unsigned)ceil_div(NV2, 4)), dim3(256), 0, s, p2, nblk,
                     NV2, 0, tri, false);
  hipLaunchKernelGGL(mom2_expand<D>, dim3(1), dim3(256), 0, s, tri, out);
}

// ---- scan -------------------------------------------------------------------
constexpr int SCAN_T = 256, SCAN_I = 8, SCAN_TILE = SCAN_T * SCAN_I;

__device__ double block_exclusive_scan(double v, double* sh, double& total) {
  // Hillis-Steele over 256 threads in LDS (fixed order -> deterministic).
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < SCAN_T; o <<= 1) {
    double add = (t >= o) ? sh[t - o] : 0.0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  total = sh[SCAN_T - 1];
  double incl = sh[t];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(SCAN_T) void scan_tile_sums(
    const double* __restrict__ in, int64_t N, double* __restrict__ sums) {
  __shared__ double sh[SCAN_T];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_I;
  double s = 0.0;
  for (int k = 0; k < SCAN_I; ++k)
    if (base + k < N) s += in[base + k];
  double tot;
  block_exclusive_scan(s, sh, tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_T) void scan_sums(double* __restrict__ sums,
                                                    int64_t n) {
  // exclusive scan of n tile sums, sequential chunks per thread
  __shared__ double sh[SCAN_T];
  const int64_t per = (n + SCAN_T - 1) / SCAN_T;
  const int64_t b0 = threadIdx.x * per;
  double s = 0.0;
  for (int64_t k = 0; k < per; ++k)
    if (b0 + k < n) s += sums[b0 + k];
  double tot;
  double off = block_exclusive_scan(s, sh, tot);
  for (int64_t k = 0; k < per; ++k) {
    if (b0 + k < n) {
      double v = sums[b0 + k];
      sums[b0 + k] = off;
      off += v;
    }
  }
}

__global__ __launch_bounds__(SCAN_T) void scan_apply(
    const double* __restrict__ in, int64_t N, const double* __restrict__ sums,
    double* __restrict__ out) {
  __shared__ double sh[SCAN_T];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_I;
  double v[SCAN_I];
  double s = 0.0;
  for (int k = 0; k < SCAN_I; ++k) {
    v[k] = (base + k < N) ? in[base + k] : 0.0;
    s += v[k];
  }
  double tot;
  double run = block_exclusive_scan(s, sh, tot) + sums[blockIdx.x];
  for (int k = 0; k < SCAN_I; ++k) {
    run += v[k];
    if (base + k < N) out[base + k] = run;
  }
}

__global__ void gather_rows_kernel(const double* __restrict__ in,
                                   const int64_t* __restrict__ idx, int64_t n,
                                   int cols, double* __restrict__ out) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * cols) return;
  int64_t i = e / cols;
  int c = (int)(e % cols);
  out[e] = in[idx[i] * cols + c];
}

constexpr int GB_MAX = 8;
struct GatherBatch {
  const double* in[GB_MAX];
  double* out[GB_MAX];
  int cols[GB_MAX];
  int64_t row0[GB_MAX];  // first output row
  int n_arrays, total_cols;
};

// several row gathers with the same index list in one launch: thread ->
// (row i, column c over the concatenated columns of all arrays)
__global__ void gather_batch_kernel(GatherBatch g, const int64_t* __restrict__ idx,
                                    int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * g.total_cols) return;
  const int64_t i = e / g.total_cols;
  int c = (int)(e % g.total_cols);
  int a = 0;
  while (a < g.n_arrays - 1 && c >= g.cols[a]) { c -= g.cols[a]; ++a; }
  const int64_t src = idx[i];
  g.out[a][(g.row0[a] + i) * g.cols[a] + c] = g.in[a][src * g.cols[a] + c];
}

__global__ void importance_weights_kernel(const double* __restrict__ lp,
                                          const double* __restrict__ lt,
                                          const double* __restrict__ accw,
                                          int64_t A, double scale,
                                          double* __restrict__ w) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < A) {
    // prior_pd * acceptance_weight * fraction / transition_pd (smc.py:803-809)
    double v = exp(lp[i] - lt[i]) * scale;
    w[i] = accw ? v * accw[i] : v;
  }
}


// ---- Population._normalize_weights + effective_sample_size ---------------
constexpr int NW_BLOCKS = 256;
__global__ __launch_bounds__(256) void wsum_kernel(const double* __restrict__ w,
                                                   int64_t N,
                                                   double* __restrict__ part) {
  double s = 0.0, s2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N;
       i += (int64_t)gridDim.x * 256) {
    const double v = w[i];
    s += v; s2 += v * v;
  }
  __shared__ double sh[2][4];
  s = wave_sum(s); s2 = wave_sum(s2);
  if ((threadIdx.x & 63) == 0) { sh[0][threadIdx.x >> 6] = s; sh[1][threadIdx.x >> 6] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ((sh[0][0] + sh[0][1]) + sh[0][2]) + sh[0][3];
    part[2 * blockIdx.x + 1] = ((sh[1][0] + sh[1][1]) + sh[1][2]) + sh[1][3];
  }
}
__global__ void wsum_final(const double* __restrict__ part, int nblk,
                           double* __restrict__ stats) {
  if (threadIdx.x != 0) return;
  double s = 0.0, s2 = 0.0;
  for (int b = 0; b < nblk; ++b) { s += part[2 * b]; s2 += part[2 * b + 1]; }
  stats[0] = s;             // sum w
  stats[1] = s * s / s2;    // ESS (weighted_statistics.py:73-83)
  stats[2] = s2;
}
__global__ void wscale_kernel(double* __restrict__ w, int64_t N,
                              const double* __restrict__ stats) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N) w[i] = w[i] / stats[0];
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" size_t abc_weighted_moments_workspace(int64_t N, int d) {
  const int64_t nb2 = d > 64 ? wide_blocks(N > 0 ? N : 1, d) : MOM_BLOCKS;
  size_t off = 0;
  size_only<double>(off, (size_t)MOM_BLOCKS * (2 + d));
  size_only<double>(off, (size_t)nb2 * d * d);
  size_only<double>(off, (size_t)MOM_BLOCKS);
  size_only<double>(off, (size_t)d * d);
  return off + 256;
}

extern "C" int abc_weighted_moments(const double* X, const double* w,
                                    int64_t N, int d, double* out, void* ws,
                                    size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(N >= 1 && d >= 1 && d <= ABC_MAX_D, "moments: bad N=%lld d=%d", (long long)N, d);
  ABC_CHECK_ARG(X && w && out && ws, "moments: null pointer");
  if (ws_bytes < abc_weighted_moments_workspace(N, d))
    return set_error(ABC_ERR_WORKSPACE, "moments: workspace too small");
  Carver cv(ws, ws_bytes);
  double* p1 = cv.take<double>((size_t)MOM_BLOCKS * (2 + d));
  double* p2 = cv.take<double>((size_t)(d > 64 ? wide_blocks(N, d) : MOM_BLOCKS) * d * d);
  double* pmax = cv.take<double>((size_t)MOM_BLOCKS);
  double* tri = cv.take<double>((size_t)d * d);
  hipStream_t s = as_stream(stream);
  switch (d) {
#define ABC_MOM_CASE(D) \
    case D: moments_fast<D>(X, w, N, out, p1, p2, pmax, tri, s); ABC_LAUNCHED(); return ABC_OK;
    ABC_MOM_CASE(1) ABC_MOM_CASE(2) ABC_MOM_CASE(3) ABC_MOM_CASE(4)
    ABC_MOM_CASE(5) ABC_MOM_CASE(6) ABC_MOM_CASE(8) ABC_MOM_CASE(10)
    ABC_MOM_CASE(12) ABC_MOM_CASE(16)
#undef ABC_MOM_CASE
    default: break;
  }
  if (d > 64) {
    const int nb = wide_blocks(N, d);
    hipLaunchKernelGGL(moments1_wide, dim3(nb, (unsigned)ceil_div(2 + d, 256)), dim3(256), 0, s,
                       X, w, N, d, p1);
    ABC_LAUNCHED();
    hipLaunchKernelGGL(moments1_final, dim3(1), dim3(256), 0, s, p1, nb, d, out);
    ABC_LAUNCHED();
    hipLaunchKernelGGL(moments2_wide, dim3(nb, (unsigned)ceil_div((int64_t)d * d, 256)), dim3(256),
                       0, s, X, w, N, d, out, p2);
    ABC_LAUNCHED();
    hipLaunchKernelGGL(moments2_final, dim3((unsigned)ceil_div((int64_t)d * d, 256)), dim3(256), 0,
                       s, p2, nb, d, out);
    ABC_LAUNCHED();
    hipLaunchKernelGGL(mom1_max_generic, dim3(1), dim3(256), 0, s, w, N, out + 2 + d + d * d);
    ABC_LAUNCHED();
    return ABC_OK;
  }
  const int nblk = (int)(ceil_div(N, MOM_ROWS) < MOM_BLOCKS ? ceil_div(N, MOM_ROWS) : MOM_BLOCKS);
  const size_t lds = sizeof(double) * (MOM_ROWS * d + MOM_ROWS);
  hipLaunchKernelGGL(moments1_kernel, dim3(nblk), dim3(256), lds, s, X, w, N, d, p1);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(moments1_final, dim3(1), dim3(256), 0, s, p1, nblk, d, out);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(moments2_kernel, dim3(nblk), dim3(256), lds, s, X, w, N, d, out, p2);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(moments2_final, dim3(1), dim3(256), 0, s, p2, nblk, d, out);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(mom1_max_generic, dim3(1), dim3(256), 0, s, w, N, out + 2 + d + d * d);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" size_t abc_scan_workspace(int64_t N) {
  return align_up(sizeof(double) * (size_t)(ceil_div(N > 0 ? N : 1, SCAN_TILE)), 256) + 256;
}

extern "C" int abc_inclusive_scan_f64(const double* in, double* out, int64_t N,
                                      void* ws, size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(N >= 0, "scan: N < 0");
  if (N == 0) return ABC_OK;
  ABC_CHECK_ARG(in && out && ws, "scan: null pointer");
  if (ws_bytes < abc_scan_workspace(N))
    return set_error(ABC_ERR_WORKSPACE, "scan: workspace too small");
  const int64_t ntile = ceil_div(N, SCAN_TILE);
  double* sums = static_cast<double*>(ws);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(scan_tile_sums, dim3((unsigned)ntile), dim3(SCAN_T), 0, s, in, N, sums);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(scan_sums, dim3(1), dim3(SCAN_T), 0, s, sums, ntile);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(scan_apply, dim3((unsigned)ntile), dim3(SCAN_T), 0, s, in, N, sums, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_gather_rows(const double* in, const int64_t* idx, int64_t n,
                               int cols, double* out, void* stream) {
  ABC_CHECK_ARG(n >= 0 && cols >= 1, "gather: bad n/cols");
  if (n == 0) return ABC_OK;
  ABC_CHECK_ARG(in && idx && out, "gather: null pointer");
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)ceil_div(n * cols, 256)), dim3(256),
                     0, as_stream(stream), in, idx, n, cols, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_gather_rows_batch(int n_arrays, const double* const* ins,
                                     const int* cols, double* const* outs,
                                     const int64_t* out_row0, const int64_t* idx,
                                     int64_t n, void* stream) {
  ABC_CHECK_ARG(n_arrays >= 1 && n_arrays <= GB_MAX && n >= 0, "gather_batch: bad sizes");
  if (n == 0) return ABC_OK;
  ABC_CHECK_ARG(ins && cols && outs && out_row0 && idx, "gather_batch: null pointer");
  GatherBatch g{};
  g.n_arrays = n_arrays;
  g.total_cols = 0;
  for (int a = 0; a < n_arrays; ++a) {
    ABC_CHECK_ARG(ins[a] && outs[a] && cols[a] >= 1 && out_row0[a] >= 0,
                  "gather_batch: array %d", a);
    g.in[a] = ins[a];
    g.out[a] = outs[a];
    g.cols[a] = cols[a];
    g.row0[a] = out_row0[a];
    g.total_cols += cols[a];
  }
  hipLaunchKernelGGL(gather_batch_kernel,
                     dim3((unsigned)ceil_div(n * g.total_cols, 256)), dim3(256), 0,
                     as_stream(stream), g, idx, n);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_importance_weights(const double* prior_logpdf,
                                      const double* trans_logpdf,
                                      const double* acc_weights, int64_t A,
                                      double scale, double* w, void* stream) {
  ABC_CHECK_ARG(A >= 0, "weights: A < 0");
  if (A == 0) return ABC_OK;
  ABC_CHECK_ARG(prior_logpdf && trans_logpdf && w, "weights: null pointer");
  hipLaunchKernelGGL(importance_weights_kernel, dim3((unsigned)ceil_div(A, 256)), dim3(256),
                     0, as_stream(stream), prior_logpdf, trans_logpdf, acc_weights, A,
                     scale, w);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" size_t abc_normalize_weights_workspace(int64_t N) {
  (void)N;
  return sizeof(double) * 2 * NW_BLOCKS + 256;
}

extern "C" int abc_normalize_weights(double* w, int64_t N, double* stats,
                                     void* ws, size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(N >= 1, "normalize: N < 1");
  ABC_CHECK_ARG(w && stats && ws, "normalize: null pointer");
  if (ws_bytes < abc_normalize_weights_workspace(N))
    return set_error(ABC_ERR_WORKSPACE, "normalize: workspace too small");
  hipStream_t s = as_stream(stream);
  const int nblk = (int)(ceil_div(N, 256) < NW_BLOCKS ? ceil_div(N, 256) : NW_BLOCKS);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(wsum_kernel, dim3(nblk), dim3(256), 0, s, w, N, part);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wsum_final, dim3(1), dim3(64), 0, s, part, nblk, stats);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(wscale_kernel, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, s, w, N, stats);
  ABC_LAUNCHED();
  return ABC_OK;
}
