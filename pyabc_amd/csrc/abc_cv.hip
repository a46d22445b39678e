// Bootstrapped coefficient of variation of the KDE at the test points.
//
// pyabc/cv/bootstrap.py:86-108 (calc_cv): the B bootstrapped transitions'
// densities at the N test points form an array [B, N]; per test point
//   variation_i = std_i / mean_i            (scipy.stats.variation, axis 0,
//                                            ddof 0, two-pass)
// and the model's contribution to the mean CV is
//   cv = sum_i (variation_i * scale) * w_i  (scale = n_m / sum n).
// The density kernels hand over log densities, so the exp is fused here.
// One HBM pass over B*N doubles (L2 serves the second pass of each column);
// the reduction uses a fixed block count and order, so cv is bitwise
// reproducible.
#include "abc_common.h"

namespace abc {
namespace {

constexpr int CV_BLOCKS = 256;

__global__ __launch_bounds__(256) void cv_column_kernel(
    const double* __restrict__ logdens, int64_t B, int64_t N,
    const double* __restrict__ w, double scale,
    double* __restrict__ variation, double* __restrict__ part) {
  double acc = 0.0;
  const double inv_b = 1.0 / (double)B;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N;
       i += (int64_t)gridDim.x * 256) {
    // numpy reduces axis 0 of a C-contiguous array row by row: the same
    // sequential order here
    double s = 0.0;
    for (int64_t b = 0; b < B; ++b) s += exp(logdens[b * N + i]);
    const double mean = s * inv_b;
    double s2 = 0.0;
    for (int64_t b = 0; b < B; ++b) {
      const double dv = exp(logdens[b * N + i]) - mean;
      s2 += dv * dv;
    }
    const double v = sqrt(s2 * inv_b) / mean;
    variation[i] = v;
    acc += (v * scale) * w[i];
  }
  __shared__ double sh[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

__global__ void cv_final_kernel(const double* __restrict__ part, int nblk,
                                double* __restrict__ cv) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += part[b];
  cv[0] = s;
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" size_t abc_bootstrap_cv_workspace(int64_t N) {
  (void)N;
  return sizeof(double) * CV_BLOCKS + 256;
}

extern "C" int abc_bootstrap_cv(const double* logdens, int64_t B, int64_t N,
                                const double* w, double scale,
                                double* variation, double* cv, void* ws,
                                size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(B >= 1 && N >= 1, "bootstrap_cv: B < 1 or N < 1");
  ABC_CHECK_ARG(logdens && w && variation && cv && ws,
                "bootstrap_cv: null pointer");
  if (ws_bytes < abc_bootstrap_cv_workspace(N))
    return set_error(ABC_ERR_WORKSPACE, "bootstrap_cv: workspace too small");
  hipStream_t s = as_stream(stream);
  const int nblk = (int)(ceil_div(N, 256) < CV_BLOCKS ? ceil_div(N, 256) : CV_BLOCKS);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(cv_column_kernel, dim3(nblk), dim3(256), 0, s, logdens, B,
                     N, w, scale, variation, part);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(cv_final_kernel, dim3(1), dim3(64), 0, s, part, nblk, cv);
  ABC_LAUNCHED();
  return ABC_OK;
}
