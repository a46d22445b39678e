// MultivariateNormalTransition.pdf on CDNA4 MFMA.
//
// Reference: pyabc/transition/multivariatenormal.py:99-113 evaluates, per
// candidate, sum_j w_j * scipy.mvn(0, Sigma).pdf(x - X_j): O(N d) per call,
// O(A N d) per generation.  Here the whole candidate batch is one
// "whitened cross-term GEMM" fused with exp2 and a weighted log-sum-exp:
//
//   y_j = (X_j - mu) U,  z_i = (x_i - mu) U          (U U^T = Sigma^+)
//   log2e * (c_j + z_i . y_j),  c_j = log w_j + shift - |y_j|^2 / 2
//   sum_j w_j exp(-|z_i - y_j|^2 / 2) = exp(-|z_i|^2 / 2 - shift)
//                                       * sum_j 2^(log2e (c_j + z_i . y_j))
//
// The cross term runs on v_mfma_f64_16x16x4_f64 (parity mode) or
// v_mfma_f32_16x16x4_f32 (fast mode), K = r + 1 padded to a multiple of 4:
// the c_j column rides in the GEMM (A = [y_j, log2e c_j], B = [log2e z_i, 1]).
// Layout is "swapped": population rows are the MFMA M dimension (A operand)
// and candidates the N dimension (B operand), so each lane owns ONE candidate
// and four population rows of every 16x16 tile: the log-sum-exp is reduced in
// registers with no cross-lane traffic until the end.  The accumulator input
// C = -m (the candidate's running reference) so the MFMA emits s - m
// directly; m starts at |z|^2 log2e / 2, which bounds s - m above by
// log2(max w e^shift), and a rare wave-uniform branch re-centres m when a
// value would overflow (> 2^64) or every value so far underflowed.
#include "abc_common.h"

namespace abc {
namespace {

constexpr double LOG2E = 1.4426950408889634074;
constexpr double LN2 = 0.69314718055994530942;
constexpr float THR_HI = 64.f;   // re-centre if s - m exceeds this (log2)
constexpr float THR_LO = -64.f;  // ... or if nothing accumulated and below

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <class T> struct Acc;
template <> struct Acc<float> {
  typedef f32x4 V;
  static __device__ __forceinline__ V mfma(float a, float b, V c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};
template <> struct Acc<double> {
  typedef f64x4 V;
  static __device__ __forceinline__ V mfma(double a, double b, V c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
};

// ---- packing ---------------------------------------------------------------
// A image: packed[t][lane][kb], t = 16-row population tile, lane 0..63,
// kb = 0..KB-1; element (row 16t + (lane & 15), k = 4 kb + (lane >> 4)).
template <class T>
__global__ void pack_population_kernel(const double* __restrict__ X,
                                       const double* __restrict__ w, int64_t N,
                                       int d, const double* __restrict__ mu,
                                       const double* __restrict__ U, int r,
                                       int KB, double shift,
                                       T* __restrict__ packed, int64_t NT) {
  int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= NT * 16) return;
  const int K = 4 * KB;
  T yv[64];
  double c;
  if (row < N) {
    double y2 = 0.0;
    for (int k = 0; k < r; ++k) {
      double acc = 0.0;
      for (int q = 0; q < d; ++q) acc += (X[row * d + q] - mu[q]) * U[q * r + k];
      T yt = (T)acc;          // the operand the MFMA will see
      yv[k] = yt;
      y2 += (double)yt * (double)yt;
    }
    double wj = w[row];
    c = (wj > 0.0) ? (log(wj) + shift - 0.5 * y2) * LOG2E : -INFINITY;
  } else {
    for (int k = 0; k < r; ++k) yv[k] = (T)0;
    c = -INFINITY;
  }
  int64_t t = row >> 4;
  int rl = (int)(row & 15);
  for (int k = 0; k < K; ++k) {
    T v = (k < r) ? yv[k] : (k == r ? (T)c : (T)0);
    int kb = k >> 2, lane = rl + 16 * (k & 3);
    packed[(t * 64 + lane) * KB + kb] = v;
  }
}

// B image for candidates + per-candidate m0 = |u|^2 log2e / 2 (fp64), where
// u = b / log2e is the whitened point the T-precision operand represents.
template <class T>
__global__ void pack_candidates_kernel(const double* __restrict__ x, int64_t M,
                                       int d, const double* __restrict__ mu,
                                       const double* __restrict__ U, int r,
                                       int KB, T* __restrict__ packed,
                                       double* __restrict__ m0, int64_t MT) {
  int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= MT * 16) return;
  const int K = 4 * KB;
  T bv[64];
  double b2 = 0.0;
  if (col < M) {
    for (int k = 0; k < r; ++k) {
      double acc = 0.0;
      for (int q = 0; q < d; ++q) acc += (x[col * d + q] - mu[q]) * U[q * r + k];
      T bt = (T)(acc * LOG2E);
      bv[k] = bt;
      b2 += (double)bt * (double)bt;
    }
    m0[col] = 0.5 * b2 / LOG2E;
  } else {
    for (int k = 0; k < r; ++k) bv[k] = (T)0;
  }
  int64_t t = col >> 4;
  int cl = (int)(col & 15);
  for (int k = 0; k < K; ++k) {
    T v = (k < r) ? bv[k] : (k == r ? (T)1 : (T)0);
    int kb = k >> 2, lane = cl + 16 * (k & 3);
    packed[(t * 64 + lane) * KB + kb] = v;
  }
}

// ---- the fused cross-term GEMM + exp2 + log-sum-exp -----------------------
// One wave = CT candidate tiles (16 CT candidates) x one population chunk.
// Block = 4 waves.  Grid is 1-D: block b -> (xcd = b % 8) so that all blocks
// of one population chunk share an XCD's L2 (speed only, never correctness).
template <class T, int KB, int CT>
__global__ __launch_bounds__(256) void mvn_lse_kernel(
    const T* __restrict__ A, const T* __restrict__ Bp,
    const double* __restrict__ m0, int64_t MT, int64_t NT, int nchunk,
    int64_t tiles_per_chunk, int64_t ngroups, double* __restrict__ part_m,
    double* __restrict__ part_l, int64_t Mpad) {
  typedef typename Acc<T>::V V;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // XCD-aware decomposition of the 1-D grid.
  const int64_t bid = blockIdx.x;
  const int cpx = nchunk >> 3;  // chunks per XCD (nchunk % 8 == 0)
  const int64_t xcd = bid & 7, j = bid >> 3;
  const int chunk = (int)(xcd + 8 * (j % cpx));
  const int64_t group = j / cpx;
  if (group >= ngroups) return;
  const int64_t ct0 = (group * 4 + wave) * CT;

  T b[CT][KB];
  T m[CT];
  double l[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int64_t ct = ct0 + c;
    const bool live = ct < MT;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
      b[c][kb] = live ? Bp[(ct * 64 + lane) * KB + kb] : (T)0;
    const int64_t cand = ct * 16 + (lane & 15);
    m[c] = live ? (T)m0[cand] : (T)0;
    l[c] = 0.0;
  }

  const int64_t t_begin = (int64_t)chunk * tiles_per_chunk;
  const int64_t t_end = t_begin + tiles_per_chunk < NT ? t_begin + tiles_per_chunk : NT;

  T a[KB], an[KB];
  if (t_begin < t_end) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) a[kb] = A[(t_begin * 64 + lane) * KB + kb];
  }
  for (int64_t t = t_begin; t < t_end; ++t) {
    const int64_t tn = (t + 1 < t_end) ? t + 1 : t;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) an[kb] = A[(tn * 64 + lane) * KB + kb];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      V acc = {-m[c], -m[c], -m[c], -m[c]};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) acc = Acc<T>::mfma(a[kb], b[c][kb], acc);
      float d0 = (float)acc[0], d1 = (float)acc[1], d2 = (float)acc[2],
            d3 = (float)acc[3];
      float tmax = fmaxf(fmaxf(d0, d1), fmaxf(d2, d3));
      bool need = (tmax > THR_HI) ||
                  (l[c] == 0.0 && tmax < THR_LO && tmax > -INFINITY);
      if (__builtin_expect(__any(need), 0)) {
        for (int it = 0; it < 8; ++it) {
          if (need) {
            T mn = m[c] + (T)tmax;
            l[c] *= exp2((double)m[c] - (double)mn);
            m[c] = mn;
          }
          V acc2 = {-m[c], -m[c], -m[c], -m[c]};
#pragma unroll
          for (int kb = 0; kb < KB; ++kb)
            acc2 = Acc<T>::mfma(a[kb], b[c][kb], acc2);
          d0 = (float)acc2[0]; d1 = (float)acc2[1];
          d2 = (float)acc2[2]; d3 = (float)acc2[3];
          tmax = fmaxf(fmaxf(d0, d1), fmaxf(d2, d3));
          need = (tmax > THR_HI) ||
                 (l[c] == 0.0 && tmax < THR_LO && tmax > -INFINITY);
          if (!__any(need)) break;
        }
      }
      float e = (__builtin_amdgcn_exp2f(d0) + __builtin_amdgcn_exp2f(d1)) +
                (__builtin_amdgcn_exp2f(d2) + __builtin_amdgcn_exp2f(d3));
      l[c] += (double)e;
    }
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) a[kb] = an[kb];
  }

  // Combine the four lane groups (lanes l, l^16, l^32, l^48 hold the same
  // candidate) and store one (m, l) partial per candidate and chunk.
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    double mm = (double)m[c], ll = l[c];
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      double mo = __shfl_xor(mm, o, 64), lo = __shfl_xor(ll, o, 64);
      double mx = fmax(mm, mo);
      double s = 0.0;
      if (ll > 0.0) s += ll * exp2(mm - mx);
      if (lo > 0.0) s += lo * exp2(mo - mx);
      mm = (ll > 0.0 || lo > 0.0) ? mx : mm;
      ll = s;
    }
    const int64_t ct = ct0 + c;
    if (lane < 16 && ct < MT) {
      const int64_t cand = ct * 16 + lane;
      part_m[(int64_t)chunk * Mpad + cand] = mm;
      part_l[(int64_t)chunk * Mpad + cand] = ll;
    }
  }
}

__global__ void mvn_combine_kernel(const double* __restrict__ part_m,
                                   const double* __restrict__ part_l,
                                   const double* __restrict__ m0, int nchunk,
                                   int64_t M, int64_t Mpad, double log_const,
                                   double* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  double mx = -INFINITY;
  for (int c = 0; c < nchunk; ++c) {
    double lv = part_l[(int64_t)c * Mpad + i];
    if (lv > 0.0) mx = fmax(mx, part_m[(int64_t)c * Mpad + i]);
  }
  if (mx == -INFINITY) { out[i] = -INFINITY; return; }
  double s = 0.0;
  for (int c = 0; c < nchunk; ++c) {
    double lv = part_l[(int64_t)c * Mpad + i];
    if (lv > 0.0) s += lv * exp2(part_m[(int64_t)c * Mpad + i] - mx);
  }
  out[i] = LN2 * (mx + log2(s) - m0[i]) + log_const;
}

// ---- direct-difference fp64 VALU kernel (any rank, singular support) -------
__global__ __launch_bounds__(256) void mvn_direct_kernel(
    const double* __restrict__ x, int64_t M, const double* __restrict__ X,
    const double* __restrict__ w, int64_t N, int d,
    const double* __restrict__ U, int r, const double* __restrict__ V, int nv,
    double tol, double log_const, double* __restrict__ out) {
  __shared__ double sm[4], sl[4];
  const int64_t i = blockIdx.x;
  if (i >= M) return;
  double xi[64];
  for (int q = 0; q < d; ++q) xi[q] = x[i * d + q];
  double m = -INFINITY, l = 0.0;
  for (int64_t j = threadIdx.x; j < N; j += blockDim.x) {
    double wj = w[j];
    if (!(wj > 0.0)) continue;
    double dev[64];
    for (int q = 0; q < d; ++q) dev[q] = xi[q] - X[j * d + q];
    bool ok = true;
    if (nv > 0) {
      double res = 0.0;
      for (int k = 0; k < nv; ++k) {
        double p = 0.0;
        for (int q = 0; q < d; ++q) p += dev[q] * V[q * nv + k];
        res += p * p;
      }
      ok = sqrt(res) < tol;
    }
    if (!ok) continue;
    double maha = 0.0;
    for (int k = 0; k < r; ++k) {
      double p = 0.0;
      for (int q = 0; q < d; ++q) p += dev[q] * U[q * r + k];
      maha += p * p;
    }
    double s = log(wj) - 0.5 * maha;
    if (s > m) { l = l * exp(m - s) + 1.0; m = s; }
    else l += exp(s - m);
  }
  // wave reduce (m, l)
  for (int o = 32; o > 0; o >>= 1) {
    double mo = __shfl_xor(m, o, 64), lo = __shfl_xor(l, o, 64);
    double mx = fmax(m, mo);
    double s = 0.0;
    if (l > 0.0) s += l * exp(m - mx);
    if (lo > 0.0) s += lo * exp(mo - mx);
    m = (l > 0.0 || lo > 0.0) ? mx : m;
    l = s;
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[wv] = m; sl[wv] = l; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double mx = -INFINITY;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k)
      if (sl[k] > 0.0) mx = fmax(mx, sm[k]);
    double s = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k)
      if (sl[k] > 0.0) s += sl[k] * exp(sm[k] - mx);
    out[i] = (s > 0.0) ? mx + log(s) + log_const : -INFINITY;
  }
}

// d > 64: the candidate row in LDS (dynamic, d doubles), the differences
// recomputed per whitening column from the population row (in cache); the
// same per-pair arithmetic and (max, sum) reduction as mvn_direct_kernel
__global__ __launch_bounds__(256) void mvn_direct_wide_kernel(
    const double* __restrict__ x, int64_t M, const double* __restrict__ X,
    const double* __restrict__ w, int64_t N, int d,
    const double* __restrict__ U, int r, const double* __restrict__ V, int nv,
    double tol, double log_const, double* __restrict__ out) {
  extern __shared__ double xs[];
  __shared__ double sm[4], sl[4];
  const int64_t i = blockIdx.x;
  if (i >= M) return;
  for (int q = threadIdx.x; q < d; q += blockDim.x) xs[q] = x[i * d + q];
  __syncthreads();
  double m = -INFINITY, l = 0.0;
  for (int64_t j = threadIdx.x; j < N; j += blockDim.x) {
    const double wj = w[j];
    if (!(wj > 0.0)) continue;
    const double* Xj = X + j * d;
    if (nv > 0) {
      double res = 0.0;
      for (int k = 0; k < nv; ++k) {
        double p = 0.0;
        for (int q = 0; q < d; ++q) p += (xs[q] - Xj[q]) * V[q * nv + k];
        res += p * p;
      }
      if (!(sqrt(res) < tol)) continue;
    }
    double maha = 0.0;
    for (int k = 0; k < r; ++k) {
      double p = 0.0;
      for (int q = 0; q < d; ++q) p += (xs[q] - Xj[q]) * U[q * r + k];
      maha += p * p;
    }
    const double s = log(wj) - 0.5 * maha;
    if (s > m) { l = l * exp(m - s) + 1.0; m = s; }
    else l += exp(s - m);
  }
  for (int o = 32; o > 0; o >>= 1) {
    double mo = __shfl_xor(m, o, 64), lo = __shfl_xor(l, o, 64);
    double mx = fmax(m, mo);
    double s = 0.0;
    if (l > 0.0) s += l * exp(m - mx);
    if (lo > 0.0) s += lo * exp(mo - mx);
    m = (l > 0.0 || lo > 0.0) ? mx : m;
    l = s;
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[wv] = m; sl[wv] = l; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double mx = -INFINITY;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k)
      if (sl[k] > 0.0) mx = fmax(mx, sm[k]);
    double s = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k)
      if (sl[k] > 0.0) s += sl[k] * exp(sm[k] - mx);
    out[i] = (s > 0.0) ? mx + log(s) + log_const : -INFINITY;
  }
}

struct Plan {
  int KB, CT, nchunk;
  int64_t MT, NT, MTpad, groups, tiles_per_chunk, Mpad;
  size_t esize;
};

Plan make_plan(int64_t M, int64_t N, int r, int prec) {
  Plan p;
  p.KB = (int)ceil_div(r + 1, 4);
  p.CT = 4;
  p.esize = prec == ABC_PREC_F32 ? 4 : 8;
  p.MT = ceil_div(M > 0 ? M : 1, 16);
  p.NT = ceil_div(N > 0 ? N : 1, 16);
  const int64_t waves = ceil_div(p.MT, p.CT);
  p.groups = ceil_div(waves, 4);
  p.MTpad = p.groups * 4 * p.CT;
  p.Mpad = p.MTpad * 16;
  // enough waves to fill 256 CUs several times over, chunks >= 32 tiles
  int64_t want = ceil_div(16384, p.groups * 4);
  int64_t maxc = ceil_div(p.NT, 32);
  int64_t nc = want < maxc ? want : maxc;
  nc = ceil_div(nc < 1 ? 1 : nc, 8) * 8;  // multiple of 8 for the XCD map
  if (nc > 1024) nc = 1024;
  p.nchunk = (int)nc;
  p.tiles_per_chunk = ceil_div(p.NT, p.nchunk);
  return p;
}

size_t plan_ws(const Plan& p) {
  size_t off = 0;
  if (p.esize == 4) size_only<float>(off, (size_t)p.MTpad * 64 * p.KB);
  else size_only<double>(off, (size_t)p.MTpad * 64 * p.KB);
  size_only<double>(off, (size_t)p.Mpad);                      // m0
  size_only<double>(off, (size_t)p.nchunk * p.Mpad);           // part m
  size_only<double>(off, (size_t)p.nchunk * p.Mpad);           // part l
  return off + 256;
}

template <class T, int KB>
void launch_lse(const Plan& p, const T* A, const T* B, const double* m0,
                double* pm, double* pl, hipStream_t s) {
  const int64_t blocks = p.groups * p.nchunk;
  hipLaunchKernelGGL((mvn_lse_kernel<T, KB, 4>), dim3((unsigned)blocks),
                     dim3(256), 0, s, A, B, m0, p.MT, p.NT, p.nchunk,
                     p.tiles_per_chunk, p.groups, pm, pl, p.Mpad);
}

template <class T>
int dispatch_lse(const Plan& p, const T* A, const T* B, const double* m0,
                 double* pm, double* pl, hipStream_t s) {
  switch (p.KB) {
#define ABC_KB(n) case n: launch_lse<T, n>(p, A, B, m0, pm, pl, s); break;
    ABC_KB(1) ABC_KB(2) ABC_KB(3) ABC_KB(4) ABC_KB(5) ABC_KB(6) ABC_KB(7)
    ABC_KB(8) ABC_KB(9) ABC_KB(10) ABC_KB(11) ABC_KB(12) ABC_KB(13)
    ABC_KB(14) ABC_KB(15)
#undef ABC_KB
    default:
      return set_error(ABC_ERR_UNSUPPORTED, "mvn_logpdf: r=%d too large", 4 * p.KB);
  }
  return ABC_OK;
}

}  // namespace
}  // namespace abc

namespace abc {
size_t x3_packed_bytes(int64_t N, int r);
int x3_max_rank();
int x3_pack_population(const double* X, const double* w, int64_t N, int d,
                       const double* mu, const double* U, int r,
                       double log_w_shift, const double* shift_dev, void* packed,
                       double* range, hipStream_t s);
size_t x3_logpdf_workspace(int64_t M, int64_t N, int r);
int x3_logpdf(const double* x, int64_t M, int d, const void* packed,
              const double* X, const double* w, int64_t N, const double* mu,
              const double* U, int r, double log_const, double log_norm,
              double* out, const int64_t* hint, void* ws, size_t ws_bytes,
              hipStream_t s, int prof_channel = ABC_PROF_DENSITY,
              const unsigned int* count_dev = nullptr);
}  // namespace abc

using namespace abc;

extern "C" size_t abc_mvn_packed_bytes(int64_t N, int r, int prec) {
  if (prec == ABC_PREC_X3) return x3_packed_bytes(N, r);
  const int KB = (int)ceil_div(r + 1, 4);
  const int64_t NT = ceil_div(N > 0 ? N : 1, 16);
  return (size_t)NT * 64 * KB * (prec == ABC_PREC_F32 ? 4 : 8);
}

extern "C" int abc_mvn_pack_population(const double* X, const double* w,
                                       int64_t N, int d, const double* mu,
                                       const double* U, int r,
                                       double log_w_shift,
                                       const double* log_w_shift_dev, int prec,
                                       void* packed, double* range,
                                       void* stream) {
  ABC_CHECK_ARG(N >= 0 && d >= 1 && d <= 64, "pack: bad N=%lld d=%d", (long long)N, d);
  ABC_CHECK_ARG(r >= 1 && r <= 59, "pack: rank r=%d outside [1, 59]", r);
  ABC_CHECK_ARG(prec == ABC_PREC_F32 || prec == ABC_PREC_F64 || prec == ABC_PREC_X3,
                "pack: bad prec");
  ABC_CHECK_ARG(packed && mu && U && (N == 0 || (X && w)), "pack: null pointer");
  ABC_CHECK_ARG(log_w_shift_dev == nullptr || prec == ABC_PREC_X3,
                "pack: a device shift is read by the X3 image only");
  if (prec == ABC_PREC_X3)
    return x3_pack_population(X, w, N, d, mu, U, r, log_w_shift, log_w_shift_dev, packed,
                              range, as_stream(stream));
  if (range) ABC_HIP(hipMemsetAsync(range, 0, 2 * sizeof(double), as_stream(stream)));
  const int KB = (int)ceil_div(r + 1, 4);
  const int64_t NT = ceil_div(N > 0 ? N : 1, 16);
  const int64_t rows = NT * 16;
  dim3 grid((unsigned)ceil_div(rows, 128)), block(128);
  if (prec == ABC_PREC_F32)
    hipLaunchKernelGGL(pack_population_kernel<float>, grid, block, 0, as_stream(stream),
                       X, w, N, d, mu, U, r, KB, log_w_shift, (float*)packed, NT);
  else
    hipLaunchKernelGGL(pack_population_kernel<double>, grid, block, 0, as_stream(stream),
                       X, w, N, d, mu, U, r, KB, log_w_shift, (double*)packed, NT);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" size_t abc_mvn_logpdf_workspace(int64_t M, int64_t N, int r, int prec) {
  if (prec == ABC_PREC_X3) return x3_logpdf_workspace(M, N, r);
  return plan_ws(make_plan(M, N, r, prec));
}

extern "C" int abc_mvn_logpdf(const double* x, int64_t M, int d,
                              const void* packed, const double* X,
                              const double* w, int64_t N, const double* mu,
                              const double* U, int r, int prec,
                              double log_const, double log_w_shift,
                              double* out, const int64_t* hint_rows, void* ws,
                              size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(M >= 0 && N >= 1 && d >= 1 && d <= 64, "logpdf: bad M/N/d");
  ABC_CHECK_ARG(r >= 1 && r <= 59, "logpdf: rank r=%d outside [1, 59]", r);
  ABC_CHECK_ARG(prec == ABC_PREC_F32 || prec == ABC_PREC_F64 || prec == ABC_PREC_X3,
                "logpdf: bad prec");
  if (M == 0) return ABC_OK;
  ABC_CHECK_ARG(x && packed && mu && U && out, "logpdf: null pointer");
  if (prec == ABC_PREC_X3)
    return x3_logpdf(x, M, d, packed, X, w, N, mu, U, r, log_const,
                     log_const + log_w_shift, out, hint_rows, ws, ws_bytes,
                     as_stream(stream));
  Plan p = make_plan(M, N, r, prec);
  if (ws_bytes < plan_ws(p))
    return set_error(ABC_ERR_WORKSPACE, "logpdf: workspace %zu < %zu", ws_bytes, plan_ws(p));
  hipStream_t s = as_stream(stream);
  Carver cv(ws, ws_bytes);
  void* Bp = (p.esize == 4) ? (void*)cv.take<float>((size_t)p.MTpad * 64 * p.KB)
                            : (void*)cv.take<double>((size_t)p.MTpad * 64 * p.KB);
  double* m0 = cv.take<double>((size_t)p.Mpad);
  double* pm = cv.take<double>((size_t)p.nchunk * p.Mpad);
  double* pl = cv.take<double>((size_t)p.nchunk * p.Mpad);
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "logpdf: workspace carve");
  dim3 gB((unsigned)ceil_div(p.MTpad * 16, 128)), bB(128);
  int rc;
  if (p.esize == 4) {
    hipLaunchKernelGGL(pack_candidates_kernel<float>, gB, bB, 0, s, x, M, d, mu, U, r,
                       p.KB, (float*)Bp, m0, p.MTpad);
    ABC_LAUNCHED();
    profile_start(s);
    rc = dispatch_lse<float>(p, (const float*)packed, (const float*)Bp, m0, pm, pl, s);
    profile_stop(s);
  } else {
    hipLaunchKernelGGL(pack_candidates_kernel<double>, gB, bB, 0, s, x, M, d, mu, U, r,
                       p.KB, (double*)Bp, m0, p.MTpad);
    ABC_LAUNCHED();
    profile_start(s);
    rc = dispatch_lse<double>(p, (const double*)packed, (const double*)Bp, m0, pm, pl, s);
    profile_stop(s);
  }
  if (rc) return rc;
  ABC_LAUNCHED();
  hipLaunchKernelGGL(mvn_combine_kernel, dim3((unsigned)ceil_div(M, 256)), dim3(256), 0, s,
                     pm, pl, m0, p.nchunk, M, p.Mpad, log_const, out);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_mvn_logpdf_direct(const double* x, int64_t M,
                                     const double* X, const double* w,
                                     int64_t N, int d, const double* U, int r,
                                     const double* V, int nv,
                                     double support_tol, double log_const,
                                     double* out, void* stream) {
  ABC_CHECK_ARG(M >= 0 && N >= 1 && d >= 1 && d <= ABC_MAX_D, "direct: bad M/N/d");
  ABC_CHECK_ARG(r >= 0 && r <= d && nv >= 0 && nv <= d, "direct: bad r/nv");
  if (M == 0) return ABC_OK;
  ABC_CHECK_ARG(x && X && w && out && (r == 0 || U) && (nv == 0 || V), "direct: null pointer");
  if (d > 64)
    hipLaunchKernelGGL(mvn_direct_wide_kernel, dim3((unsigned)M), dim3(256),
                       sizeof(double) * (size_t)d, as_stream(stream), x, M, X, w, N, d, U, r, V,
                       nv, support_tol, log_const, out);
  else
    hipLaunchKernelGGL(mvn_direct_kernel, dim3((unsigned)M), dim3(256), 0, as_stream(stream),
                       x, M, X, w, N, d, U, r, V, nv, support_tol, log_const, out);
  ABC_LAUNCHED();
  return ABC_OK;
}
