// Stable segmented LSD radix sort of fp64 keys (abc_sort_pairs_f64) and the
// sort-based weighted quantile (abc_weighted_quantile_sorted: the exact
// fallback of the weighted MSD select of abc_quantile.hip, for inputs whose
// knots sit in ties by the thousand); AdaptivePNormDistance's per-column std
// (two-pass) here and its median absolute deviation by radix select
// (abc_select.hip).
//
// Reference:
//   weighted_quantile   pyabc/weighted_statistics.py:27-43 (argsort, cumsum,
//                       np.interp) via QuantileEpsilon._update
//                       pyabc/epsilon/epsilon.py:202-228
//   std / MAD scales    pyabc/distance/scale.py:38-65 via
//                       AdaptivePNormDistance._update distance.py:263-307
// Keys are mapped to order-preserving u64; 8-bit digits, 8 passes, 2048-item
// tiles; stable per-wave ranks by ballot multi-split (radix_scatter_kernel).  Segments (columns) are sorted independently: the
// histogram is laid out [segment][digit][tile], and one global exclusive scan
// over it yields per-segment offsets because every segment holds exactly
// seg_len items.
#include "abc_common.h"

namespace abc {
namespace {

constexpr int RT = 256, RI = 8, RTILE = RT * RI, RBITS = 8, RDIG = 256;

__device__ __forceinline__ uint64_t f2key(double v) {
  if (v == 0.0) v = 0.0;  // -0.0 ties with +0.0, as in numpy's comparisons
  uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key2f(uint64_t k) {
  uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

__global__ void to_keys_kernel(const double* __restrict__ in, int64_t n,
                               uint64_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = f2key(in[i]);
}
// ---- one LSD pass: 8-bit digits, wave multi-split ranking -------------------
// Tile = 2048 items; item i of lane l in wave w sits at tile position
// 512 w + 64 i + l (coalesced loads).  Stable ranks: for each item slot i in
// order, the lanes holding the same digit find each other with 8 ballots
// (one per digit bit); a lane's rank is the running per-wave count of its
// digit (LDS) plus the number of lower lanes with that digit.  Per-wave counts
// then become per-wave prefixes, and the global offset of (segment, digit,
// tile) comes from one exclusive scan over the [segment][digit][tile] table.
constexpr int RW = RT / 64;  // waves per block

__device__ __forceinline__ uint64_t digit_peers(int dg, uint64_t valid) {
  uint64_t peers = valid;
#pragma unroll
  for (int bit = 0; bit < RBITS; ++bit) {
    const uint64_t bal = __ballot((dg >> bit) & 1);
    peers &= ((dg >> bit) & 1) ? bal : ~bal;
  }
  return peers;
}

__global__ __launch_bounds__(RT) void radix_hist_kernel(
    const uint64_t* __restrict__ keys, int64_t seg_len, int64_t tps, int shift,
    int64_t* __restrict__ hist) {
  __shared__ int cnt[RW][RDIG];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  for (int e = t; e < RW * RDIG; e += RT) (&cnt[0][0])[e] = 0;
  __syncthreads();
  const int64_t tile = blockIdx.x;
  const int64_t sgi = tile / tps, tis = tile % tps;
  const int64_t base = sgi * seg_len + tis * RTILE;
  const int64_t lim = seg_len - tis * RTILE;
#pragma unroll
  for (int i = 0; i < RI; ++i) {
    const int64_t o = (int64_t)wave * (64 * RI) + i * 64 + lane;
    if (o < lim) atomicAdd(&cnt[wave][(int)((keys[base + o] >> shift) & (RDIG - 1))], 1);
  }
  __syncthreads();
  for (int dg = t; dg < RDIG; dg += RT) {
    int tot = 0;
#pragma unroll
    for (int w = 0; w < RW; ++w) tot += cnt[w][dg];
    hist[(sgi * RDIG + dg) * tps + tis] = tot;
  }
}

template <bool VALS>
__global__ __launch_bounds__(RT) void radix_scatter_kernel(
    const uint64_t* __restrict__ keys, const double* __restrict__ vals,
    int64_t seg_len, int64_t tps, int shift, const int64_t* __restrict__ off,
    uint64_t* __restrict__ keys_out, double* __restrict__ vals_out) {
  __shared__ int cnt[RW][RDIG];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  for (int e = t; e < RW * RDIG; e += RT) (&cnt[0][0])[e] = 0;
  __syncthreads();
  const int64_t tile = blockIdx.x;
  const int64_t sgi = tile / tps, tis = tile % tps;
  const int64_t base = sgi * seg_len + tis * RTILE;
  const int64_t lim = seg_len - tis * RTILE;
  const uint64_t lt = (1ull << lane) - 1;
  uint64_t kv[RI];
  double vv[RI];
  int dg[RI], pos[RI];
#pragma unroll
  for (int i = 0; i < RI; ++i) {
    const int64_t o = (int64_t)wave * (64 * RI) + i * 64 + lane;
    const bool ok = o < lim;
    kv[i] = ok ? keys[base + o] : 0;
    if (VALS) vv[i] = ok ? vals[base + o] : 0.0;
    dg[i] = (int)((kv[i] >> shift) & (RDIG - 1));
    const uint64_t valid = __ballot(ok);
    const uint64_t peers = digit_peers(dg[i], valid);
    int before = 0;
    if (ok) before = cnt[wave][dg[i]];
    pos[i] = ok ? before + __popcll(peers & lt) : -1;
    if (ok && (peers & lt) == 0) cnt[wave][dg[i]] = before + __popcll(peers);
  }
  __syncthreads();
  // per-wave counts -> global start of each wave's run of each digit
  for (int d = t; d < RDIG; d += RT) {
    int64_t run = off[(sgi * RDIG + d) * tps + tis];
#pragma unroll
    for (int w = 0; w < RW; ++w) {
      const int c = cnt[w][d];
      cnt[w][d] = (int)(run - sgi * seg_len);  // segment-relative (fits int)
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RI; ++i) {
    if (pos[i] >= 0) {
      const int64_t p = sgi * seg_len + cnt[wave][dg[i]] + pos[i];
      keys_out[p] = kv[i];
      if (VALS) vals_out[p] = vv[i];
    }
  }
}

// ---- generic exclusive scan of int64 (3 phases) -----------------------------
constexpr int ST = 256, SI = 8, STILE = ST * SI;

__device__ int64_t block_exscan(int64_t v, int64_t* sh, int64_t& total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < ST; o <<= 1) {
    int64_t add = (t >= o) ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  total = sh[ST - 1];
  int64_t incl = sh[t];
  __syncthreads();
  return incl - v;
}
__global__ __launch_bounds__(ST) void exscan_sums(const int64_t* __restrict__ in,
                                                  int64_t n,
                                                  int64_t* __restrict__ sums) {
  __shared__ int64_t sh[ST];
  const int64_t b = (int64_t)blockIdx.x * STILE + threadIdx.x * SI;
  int64_t s = 0;
  for (int k = 0; k < SI; ++k) if (b + k < n) s += in[b + k];
  int64_t tot;
  block_exscan(s, sh, tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}
__global__ __launch_bounds__(ST) void exscan_top(int64_t* __restrict__ sums,
                                                 int64_t n) {
  __shared__ int64_t sh[ST];
  const int64_t per = (n + ST - 1) / ST;
  const int64_t b0 = threadIdx.x * per;
  int64_t s = 0;
  for (int64_t k = 0; k < per; ++k) if (b0 + k < n) s += sums[b0 + k];
  int64_t tot;
  int64_t off = block_exscan(s, sh, tot);
  for (int64_t k = 0; k < per; ++k)
    if (b0 + k < n) { int64_t v = sums[b0 + k]; sums[b0 + k] = off; off += v; }
}
__global__ __launch_bounds__(ST) void exscan_apply(const int64_t* __restrict__ in,
                                                   int64_t n,
                                                   const int64_t* __restrict__ sums,
                                                   int64_t* __restrict__ out) {
  __shared__ int64_t sh[ST];
  const int64_t b = (int64_t)blockIdx.x * STILE + threadIdx.x * SI;
  int64_t v[SI];
  int64_t s = 0;
  for (int k = 0; k < SI; ++k) { v[k] = (b + k < n) ? in[b + k] : 0; s += v[k]; }
  int64_t tot;
  int64_t run = block_exscan(s, sh, tot) + sums[blockIdx.x];
  for (int k = 0; k < SI; ++k) { if (b + k < n) out[b + k] = run; run += v[k]; }
}

// single-workgroup exclusive scan for histograms up to SCAN1_MAX entries: one
// launch instead of three.  1024 threads, each with S1_PER consecutive
// entries loaded up front (all loads in flight together), wave-shuffle scan of
// the thread sums, LDS across the 16 waves; fixed order, deterministic.
constexpr int S1_T = 1024, S1_PER = 16;
constexpr int64_t SCAN1_MAX = (int64_t)S1_T * S1_PER;
__global__ __launch_bounds__(S1_T) void exscan_single(const int64_t* __restrict__ in,
                                                      int64_t n,
                                                      int64_t* __restrict__ out) {
  __shared__ int64_t wsum[S1_T / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t per = (n + S1_T - 1) / S1_T;  // <= S1_PER
  const int64_t b0 = (int64_t)t * per;
  int64_t v[S1_PER];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < S1_PER; ++k) {
    v[k] = (k < per && b0 + k < n) ? in[b0 + k] : 0;
    s += v[k];
  }
  int64_t incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int64_t run = incl - s;
  for (int w = 0; w < wv; ++w) run += wsum[w];
#pragma unroll
  for (int k = 0; k < S1_PER; ++k)
    if (k < per && b0 + k < n) { out[b0 + k] = run; run += v[k]; }
}

struct SortBufs {
  uint64_t* k0; uint64_t* k1; double* v0; double* v1;
  int64_t* hist; int64_t* off; int64_t* sums;
};

size_t sort_ws_bytes(int64_t nseg, int64_t seg_len, bool vals) {
  const int64_t tps = ceil_div(seg_len > 0 ? seg_len : 1, RTILE);
  const int64_t nh = nseg * RDIG * tps;
  const int64_t n = nseg * seg_len;
  size_t off = 0;
  size_only<uint64_t>(off, (size_t)n);
  size_only<uint64_t>(off, (size_t)n);
  if (vals) { size_only<double>(off, (size_t)n); size_only<double>(off, (size_t)n); }
  size_only<int64_t>(off, (size_t)nh);
  size_only<int64_t>(off, (size_t)nh);
  size_only<int64_t>(off, (size_t)ceil_div(nh, STILE) + 1);
  return off + 256;
}

bool carve_sort(Carver& cv, int64_t nseg, int64_t seg_len, bool vals, SortBufs& b) {
  const int64_t tps = ceil_div(seg_len > 0 ? seg_len : 1, RTILE);
  const int64_t nh = nseg * RDIG * tps;
  const int64_t n = nseg * seg_len;
  b.k0 = cv.take<uint64_t>((size_t)n);
  b.k1 = cv.take<uint64_t>((size_t)n);
  b.v0 = vals ? cv.take<double>((size_t)n) : nullptr;
  b.v1 = vals ? cv.take<double>((size_t)n) : nullptr;
  b.hist = cv.take<int64_t>((size_t)nh);
  b.off = cv.take<int64_t>((size_t)nh);
  b.sums = cv.take<int64_t>((size_t)ceil_div(nh, STILE) + 1);
  return cv.ok;
}

// Sorts keys (already in b.k0, values in b.v0); result lands in b.k0/b.v0
// (8 passes = even number of swaps).
int run_sort(SortBufs& b, int64_t nseg, int64_t seg_len, hipStream_t s) {
  const int64_t tps = ceil_div(seg_len > 0 ? seg_len : 1, RTILE);
  const int64_t ntile = nseg * tps;
  const int64_t nh = nseg * RDIG * tps;
  const int64_t nsum = ceil_div(nh, STILE);
  for (int pass = 0; pass < 64 / RBITS; ++pass) {
    const int shift = pass * RBITS;
    hipLaunchKernelGGL(radix_hist_kernel, dim3((unsigned)ntile), dim3(RT), 0, s, b.k0,
                       seg_len, tps, shift, b.hist);
    ABC_LAUNCHED();
    if (nh <= SCAN1_MAX) {
      hipLaunchKernelGGL(exscan_single, dim3(1), dim3(S1_T), 0, s, b.hist, nh, b.off);
      ABC_LAUNCHED();
    } else {
      hipLaunchKernelGGL(exscan_sums, dim3((unsigned)nsum), dim3(ST), 0, s, b.hist, nh,
                         b.sums);
      ABC_LAUNCHED();
      hipLaunchKernelGGL(exscan_top, dim3(1), dim3(ST), 0, s, b.sums, nsum);
      ABC_LAUNCHED();
      hipLaunchKernelGGL(exscan_apply, dim3((unsigned)nsum), dim3(ST), 0, s, b.hist, nh,
                         b.sums, b.off);
      ABC_LAUNCHED();
    }
    if (b.v0)
      hipLaunchKernelGGL(radix_scatter_kernel<true>, dim3((unsigned)ntile), dim3(RT), 0, s,
                         b.k0, b.v0, seg_len, tps, shift, b.off, b.k1, b.v1);
    else
      hipLaunchKernelGGL(radix_scatter_kernel<false>, dim3((unsigned)ntile), dim3(RT), 0, s,
                         b.k0, b.v0, seg_len, tps, shift, b.off, b.k1, b.v1);
    ABC_LAUNCHED();
    uint64_t* tk = b.k0; b.k0 = b.k1; b.k1 = tk;
    double* tv = b.v0; b.v0 = b.v1; b.v1 = tv;
  }
  return ABC_OK;
}

__global__ void from_keys_kernel(const uint64_t* __restrict__ k, int64_t n,
                                 double* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = key2f(k[i]);
}

// ---- weighted quantile ----------------------------------------------------
// xp_k = (cs_k - w_k/2) / total; np.interp(alpha, xp, sorted points)
// (numpy compiled_base.c arr_interp: j = #(xp <= x) - 1, edges clamp, exact
// knot hit -> fp[j], NaN fallback from the right knot).
__global__ void quantile_pick_kernel(const uint64_t* __restrict__ keys,
                                     const double* __restrict__ w,
                                     const double* __restrict__ cs, int64_t n,
                                     double alpha, double* __restrict__ q) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double total = cs[n - 1];
  auto xp = [&](int64_t k) { return (cs[k] - 0.5 * w[k]) / total; };
  auto fp = [&](int64_t k) { return key2f(keys[k]); };
  if (alpha > xp(n - 1)) { *q = fp(n - 1); return; }
  if (alpha < xp(0)) { *q = fp(0); return; }
  int64_t lo = 0, hi = n;  // first index with xp > alpha
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (xp(mid) > alpha) hi = mid; else lo = mid + 1;
  }
  const int64_t j = lo - 1;
  if (j == n - 1) { *q = fp(j); return; }
  const double xj = xp(j), xj1 = xp(j + 1), yj = fp(j), yj1 = fp(j + 1);
  if (xj == alpha) { *q = yj; return; }
  const double slope = (yj1 - yj) / (xj1 - xj);
  double r = slope * (alpha - xj) + yj;
  if (isnan(r)) {
    r = slope * (alpha - xj1) + yj1;
    if (isnan(r) && yj == yj1) r = yj;
  }
  *q = r;
}

// ---- column std (np.std, two-pass) -------------------------------------------
constexpr int CS_BLOCKS = 256;
__global__ __launch_bounds__(256) void colsum_kernel(const double* __restrict__ X,
                                                     int64_t R, int S,
                                                     const double* __restrict__ mean,
                                                     double* __restrict__ part) {
  // thread -> column (c = threadIdx.x + 256 h), rows strided by block
  // 8 rows in flight per thread (independent partial sums, fixed order)
  constexpr int U = 8;
  const int64_t G = gridDim.x;
  for (int c = threadIdx.x; c < S; c += blockDim.x) {
    double acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = 0.0;
    const double m = mean ? mean[c] : 0.0;
    int64_t r = blockIdx.x;
    for (; r + (U - 1) * G < R; r += U * G) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = X[(r + u * G) * S + c];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += mean ? (v[u] - m) * (v[u] - m) : v[u];
    }
    for (int u = 0; r < R; r += G, ++u) {
      const double v = X[r * S + c];
      acc[u] += mean ? (v - m) * (v - m) : v;
    }
    double sum = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) sum += acc[u];
    part[(int64_t)blockIdx.x * S + c] = sum;
  }
}
__global__ void colsum_final(const double* __restrict__ part, int nblk, int S,
                             int64_t R, double* __restrict__ out, bool sqrt_it) {
  for (int c = threadIdx.x + blockIdx.x * blockDim.x; c < S; c += blockDim.x * gridDim.x) {
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * S + c];
    s /= (double)R;
    out[c] = sqrt_it ? sqrt(s) : s;
  }
}

}  // namespace
}  // namespace abc

namespace abc {
size_t select_ws_bytes(int64_t R, int S);
int column_mad_select(const double* X, int64_t R, int S, double* out, void* ws,
                      size_t ws_bytes, hipStream_t s);
}  // namespace abc

using namespace abc;

extern "C" size_t abc_sort_pairs_workspace(int64_t N) {
  return sort_ws_bytes(1, N, true);
}

extern "C" int abc_sort_pairs_f64(const double* keys, const double* vals,
                                  int64_t N, double* keys_out,
                                  double* vals_out, void* ws, size_t ws_bytes,
                                  void* stream) {
  ABC_CHECK_ARG(N >= 0, "sort: N < 0");
  if (N == 0) return ABC_OK;
  ABC_CHECK_ARG(keys && vals && keys_out && vals_out && ws, "sort: null pointer");
  if (ws_bytes < sort_ws_bytes(1, N, true))
    return set_error(ABC_ERR_WORKSPACE, "sort: workspace too small");
  hipStream_t s = as_stream(stream);
  Carver cv(ws, ws_bytes);
  SortBufs b;
  if (!carve_sort(cv, 1, N, true, b)) return set_error(ABC_ERR_WORKSPACE, "sort: carve");
  hipLaunchKernelGGL(to_keys_kernel, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, s, keys, N, b.k0);
  ABC_LAUNCHED();
  ABC_HIP(hipMemcpyAsync(b.v0, vals, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
  int rc = run_sort(b, 1, N, s);
  if (rc) return rc;
  hipLaunchKernelGGL(from_keys_kernel, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, s, b.k0, N, keys_out);
  ABC_LAUNCHED();
  ABC_HIP(hipMemcpyAsync(vals_out, b.v0, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
  return ABC_OK;
}

extern "C" size_t abc_weighted_quantile_sorted_workspace(int64_t N) {
  size_t off = sort_ws_bytes(1, N, true);
  size_only<double>(off, (size_t)(N > 0 ? N : 1));  // cumsum
  off += abc_scan_workspace(N) + 256;
  return off + 256;
}

extern "C" int abc_weighted_quantile_sorted(const double* points, const double* w,
                                     int64_t N, double alpha, double* q,
                                     void* ws, size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(N >= 1, "quantile: N < 1");
  ABC_CHECK_ARG(points && w && q && ws, "quantile: null pointer");
  if (ws_bytes < abc_weighted_quantile_sorted_workspace(N))
    return set_error(ABC_ERR_WORKSPACE, "quantile: workspace too small");
  hipStream_t s = as_stream(stream);
  Carver cv(ws, ws_bytes);
  SortBufs b;
  if (!carve_sort(cv, 1, N, true, b)) return set_error(ABC_ERR_WORKSPACE, "quantile: carve");
  double* cs = cv.take<double>((size_t)N);
  size_t scan_bytes = abc_scan_workspace(N);
  void* scan_ws = cv.take<char>(scan_bytes);
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "quantile: carve");
  hipLaunchKernelGGL(to_keys_kernel, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, s, points, N, b.k0);
  ABC_LAUNCHED();
  ABC_HIP(hipMemcpyAsync(b.v0, w, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
  int rc = run_sort(b, 1, N, s);
  if (rc) return rc;
  rc = abc_inclusive_scan_f64(b.v0, cs, N, scan_ws, scan_bytes, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(quantile_pick_kernel, dim3(1), dim3(64), 0, s, b.k0, b.v0, cs, N, alpha, q);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" size_t abc_column_stats_workspace(int64_t R, int S) {
  size_t a = select_ws_bytes(R, S);
  size_t off = 0;
  size_only<double>(off, (size_t)CS_BLOCKS * S);
  size_only<double>(off, (size_t)S);
  return (a > off ? a : off) + 256;
}

extern "C" int abc_column_std(const double* X, int64_t R, int S, double* out,
                              void* ws, size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(R >= 1 && S >= 1, "column_std: bad R/S");
  ABC_CHECK_ARG(X && out && ws, "column_std: null pointer");
  if (ws_bytes < abc_column_stats_workspace(R, S))
    return set_error(ABC_ERR_WORKSPACE, "column_std: workspace too small");
  hipStream_t s = as_stream(stream);
  Carver cv(ws, ws_bytes);
  double* part = cv.take<double>((size_t)CS_BLOCKS * S);
  double* mean = cv.take<double>((size_t)S);
  const int nblk = (int)(R < CS_BLOCKS ? R : CS_BLOCKS);
  hipLaunchKernelGGL(colsum_kernel, dim3(nblk), dim3(256), 0, s, X, R, S, (const double*)nullptr, part);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(colsum_final, dim3((unsigned)ceil_div(S, 256)), dim3(256), 0, s, part, nblk, S, R, mean, false);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(colsum_kernel, dim3(nblk), dim3(256), 0, s, X, R, S, (const double*)mean, part);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(colsum_final, dim3((unsigned)ceil_div(S, 256)), dim3(256), 0, s, part, nblk, S, R, out, true);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_column_mad(const double* X, int64_t R, int S, double* out,
                              void* ws, size_t ws_bytes, void* stream) {
  ABC_CHECK_ARG(R >= 1 && S >= 1, "column_mad: bad R/S");
  ABC_CHECK_ARG(X && out && ws, "column_mad: null pointer");
  if (ws_bytes < abc_column_stats_workspace(R, S))
    return set_error(ABC_ERR_WORKSPACE, "column_mad: workspace too small");
  // exact radix select per column (abc_select.hip): median, then the median
  // of |x - median|; no full sort
  return column_mad_select(X, R, S, out, ws, ws_bytes, as_stream(stream));
}
