// k-NN selection of the LocalTransition fit on fp32 MFMA (included by
// abc_local.hip inside its anonymous namespace; uses dist2v from there).
//
// Reference: pyabc/transition/local_transition.py:77-96 (cKDTree.query(X,
// k + 1) per particle, neighbours indices[n, 1:]) and :125-139 (the weighted
// covariance of the neighbour offsets).
//
// Keys.  The exact order is the one of the fp64 squared distances s64 (the
// fma chain of dist2v), ties by index.  The sweeps see fp32 keys
//   s^ = n^_j + n^_n - 2 y^_j . y^_n      (y^ = fp32(X - c), n^ = fp32 |y^|^2)
// computed by v_mfma_f32_16x16x4_f32 from a [rows x K] feature image
// a_j = [y^_j, n^_j, 1] and per-lane particle features b_n = [-2 y^_n, 1,
// n^_n] (K = D + 2 padded to 4 KB): 256 pairs per wave per 16-row tile, the
// MFMA pipe beside the VALU's per-key work.  c is the midrange of the
// population (the bound scales with R^2 = max |y^|^2, not with |X|^2), and
// the MFMA is a k-ordered fmaf chain (cdna_hip_programming.md), so
//   |s^ - s64| <= B(s) = 2 * 1.01 [(4 g_{D+2} + 2 g_D) R^2 + 4 u' R sqrt(s)
//                                   + 4 u'^2 R^2 + (D + 3) 2^-53 s]
// (g_k = k u / (1 - k u), u = 2^-24, u' = u + 2^-52; the leading 2 is a
// safety factor): the expanded products and sums round in fp32 on values up
// to 4 R^2, the inputs y^ are within u' |y| of the true centred
// coordinates, and s64 is itself within (D + 3) 2^-53 s of s.  B increases
// and s - B(s) increases above the tiny s_c = 16 u'^2 R^2, so
//   s^ < V - B(V)  =>  s64 < V,      s^ > V + B(V)  =>  s64 > V.
//
// Per block of 16 particles (one MFMA column tile, 4 waves splitting the
// rows):
//  1. a sorted fp32 distance sample of 512 evenly spaced rows brackets the
//     rank k (the window [lo, hi] of the existing local_select_kernel);
//  2. count sweep: keys below the window counted in registers, keys inside
//     histogrammed in LDS on ~9 bits -> the bin [l, h) holding rank k in
//     fp32 key order;
//  3. collect sweep: T_lo = l - B(l), T_hi = h + B(2h) bracket the exact
//     rank-k key (#{s64 < T_lo} <= #{s^ < l} <= k < #{s^ < h} <=
//     #{s64 < T_hi}); keys certainly below T_lo are counted, keys certainly
//     above T_hi skipped, the rest settled in fp64 and the ones in
//     [T_lo, T_hi) listed (key, index) in LDS; the rank is selected there.
//     For small k ("list mode", every particle's #{s^ < h} + margin fits the
//     list) T_lo = -inf: the list then holds every neighbour, and the block
//     sums the moments of the k + 1 nearest (rank order, fixed-order wave
//     reduction) itself, so no moments sweep runs for those particles.
// A particle whose window misses the rank or whose list overflows is
// flagged (need[n] = 1) and re-selected by local_select_kernel (fp64 radix
// passes, exact for any data).
// Dense k (defer = 1, the moments run on knn_dense_kernel): the kernel stops
// after step 2 and leaves [T_lo, T_hi) in sel_v / sel_jcut; the moments
// sweep does step 3 on its own keys and knn_resolve_kernel step 4
// (abc_local_dense.h), one N^2 sweep fewer.
constexpr int KN_PB = 16;    // particles per block
constexpr int KN_SK = 512;   // sample rows
constexpr int KN_NB = 520;   // window bins
constexpr int KN_CAP = 192;  // list entries per particle (LDS: 4 blocks per CU)
constexpr int KN_MARGIN = 32;
constexpr int KN_PF = 2;     // row-tile groups in flight per sweep (kn_sweep; A/B: 2 best, 1 / 3 / 4 / 6 slower)
// padding tiles past the image's ceil(N / 16) tiles: kn_sweep's last group
// (t0 <= nt - 1) prefetches tiles up to t0 + 2 G + 4 (KN_PF - 1), G = 4 KN_PF,
// i.e. nt - 1 + 12 KN_PF - 4 < nt + 12 KN_PF
constexpr int KN_PAD = 12 * KN_PF;
constexpr int KN_MIN_N = 4 * KN_SK;
constexpr int KN_QCAP = 256; // open pairs per particle queued by the deferred collect
typedef float knf4 __attribute__((ext_vector_type(4)));

template <int D> constexpr int kn_kb() { return (D + 2 + 3) / 4; }
// list mode sums the moments in registers: NM doubles per lane
template <int D> constexpr bool kn_list_capable() { return D <= 8; }

struct KnBound {
  double a0, a1, eta, sc;   // B(s) = a0 + a1 sqrt(s) + eta s, valid above sc
  __device__ double operator()(double s) const { return a0 + a1 * sqrt(s) + eta * s; }
};
template <int D>
__device__ __forceinline__ KnBound kn_bound(double R2) {
  constexpr double u = 5.9604644775390625e-08, up = u + 2.220446049250313e-16;
  constexpr double g2 = (D + 2) * u / (1.0 - (D + 2) * u), g0 = D * u / (1.0 - D * u);
  const double R = sqrt(R2);
  KnBound b;
  b.a0 = 2.0 * 1.01 * ((4.0 * g2 + 2.0 * g0) * R2 + 4.0 * up * up * R2) + 1e-300;
  b.a1 = 2.0 * 1.01 * 4.0 * up * R;
  b.eta = 2.0 * 1.01 * (D + 3) * 1.1102230246251565e-16;
  b.sc = 16.0 * up * up * R2 * 4.0 + 1e-300;
  return b;
}
// fp32 c: s^ < c => s64 < V (-inf when no such cut exists)
__device__ __forceinline__ float kn_cut_below(double V, const KnBound& B) {
  if (!(V > B.sc)) return -INFINITY;
  const double t = V - B(V);
  if (!(t > 0.0)) return -INFINITY;
  if (!(t < 3.0e38)) return 3.0e38f;
  float c = (float)t;
  if ((double)c > t) c = __uint_as_float(__float_as_uint(c) - 1u);
  return c;
}
// fp32 c: s^ > c => s64 > V (+inf for V = +inf)
__device__ __forceinline__ float kn_cut_above(double V, const KnBound& B) {
  const double t = V + B(V > 0.0 ? V : 0.0);
  if (!(t < 3.0e38)) return INFINITY;
  float c = (float)t;
  if ((double)c < t) c = __uint_as_float(__float_as_uint(c) + 1u);
  return c;
}

// c = midrange of each coordinate (one block)
template <int D>
__global__ __launch_bounds__(1024) void knn_center_kernel(const double* __restrict__ X, int64_t N,
                                                          double* __restrict__ cen) {
  __shared__ double smin[16][D], smax[16][D];
  double mn[D], mx[D];
#pragma unroll
  for (int q = 0; q < D; ++q) { mn[q] = INFINITY; mx[q] = -INFINITY; }
  for (int64_t j = threadIdx.x; j < N; j += 1024)
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const double v = X[j * D + q];
      mn[q] = fmin(mn[q], v);
      mx[q] = fmax(mx[q], v);
    }
#pragma unroll
  for (int q = 0; q < D; ++q)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn[q] = fmin(mn[q], __shfl_xor(mn[q], o, 64));
      mx[q] = fmax(mx[q], __shfl_xor(mx[q], o, 64));
    }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < D; ++q) { smin[wv][q] = mn[q]; smax[wv][q] = mx[q]; }
  __syncthreads();
  if (threadIdx.x < D) {
    const int q = threadIdx.x;
    double a = smin[0][q], b = smax[0][q];
    for (int t = 1; t < 16; ++t) { a = fmin(a, smin[t][q]); b = fmax(b, smax[t][q]); }
    cen[q] = 0.5 * a + 0.5 * b;
  }
}

// y^ and n^ of one row: the image and the in-kernel particle features use
// this one function (the same bits)
template <int D>
__device__ __forceinline__ float kn_feat(const double* __restrict__ X, int64_t j,
                                         const double* __restrict__ cen, float (&y)[D]) {
  float n = 0.0f;
#pragma unroll
  for (int q = 0; q < D; ++q) {
    y[q] = (float)(X[j * D + q] - cen[q]);
    n = __builtin_fmaf(y[q], y[q], n);
  }
  return n;
}

// feature image [ceil(N/16)][KB][64]: lane l of k-block kb holds feature
// 4 kb + (l >> 4) of row 16 t + (l & 15) (the A operand of 16x16x4 f32);
// rows >= N: n^ = +inf, everything else 0 (key +inf).  R2 = max |y^|^2
// (bits of a non-negative double, atomic max; zeroed by the caller).
template <int D>
__global__ __launch_bounds__(256) void knn_prep_kernel(const double* __restrict__ X, int64_t N,
                                                       const double* __restrict__ cen,
                                                       float* __restrict__ img,
                                                       unsigned long long* __restrict__ r2bits) {
  constexpr int KB = kn_kb<D>();
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nt = (N + 15) / 16 + KN_PAD;   // + the sweeps' prefetch padding
  double r2 = 0.0;
  if (j < nt * 16) {
    float f[4 * KB];
#pragma unroll
    for (int k = 0; k < 4 * KB; ++k) f[k] = 0.0f;
    if (j < N) {
      float y[D];
      const float n = kn_feat<D>(X, j, cen, y);
#pragma unroll
      for (int q = 0; q < D; ++q) { f[q] = y[q]; r2 += (double)y[q] * (double)y[q]; }
      f[D] = n;
      f[D + 1] = 1.0f;
    } else {
      f[D] = INFINITY;
    }
    const int64_t t = j >> 4;
    const int r = (int)(j & 15);
#pragma unroll
    for (int k = 0; k < 4 * KB; ++k) img[(t * KB + (k >> 2)) * 64 + 16 * (k & 3) + r] = f[k];
  }
  r2 = wave_max(r2);
  if ((threadIdx.x & 63) == 0 && r2 > 0.0)
    atomicMax(r2bits, (unsigned long long)__double_as_longlong(r2 * (1.0 + 1e-6)));
}

// One wave's sweep over its row tiles t = wv, wv + 4, ... (4 waves per
// block): the A fragments of the next KN_PF tiles are loaded while the
// current ones are multiplied and consumed, so a tile's L2 latency hides
// under its predecessors' work (one tile at a time the sweeps were
// latency-bound at 3 waves per SIMD).  body(t, c) gets tile t's keys c
// (lane: rows 16 t + 4 (lane >> 4) + r, particle lane & 15).
// The image carries KN_PAD = 12 KN_PF padding tiles past nt, so the prefetch of the
// last group needs no clamp; tile indices are wave-uniform 32-bit values
// (scalar address arithmetic, the lane offset the only vector part).
template <int KB, class Body>
__device__ __forceinline__ void kn_sweep(const float* __restrict__ img, int nt, int wv,
                                         int lane, const float (&bfr)[KB], Body&& body) {
  // software pipeline over groups of KN_PF tiles: the loads of group g + 2
  // and the MFMAs of group g + 1 are issued before the VALU body of group g,
  // so the matrix pipe, the memory pipe and the VALU work on different groups
  float ld[KN_PF][KB];
  knf4 cn[KN_PF];
  auto load = [&](int t0) {
#pragma unroll
    for (int i = 0; i < KN_PF; ++i) {
      const float* src = img + (size_t)(t0 + 4 * i) * (KB * 64);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) ld[i][kb] = src[kb * 64 + lane];
    }
  };
  // k-block-major order: the KN_PF tiles' MFMAs of one k-block are
  // independent and issue back to back; each accumulator's next k-block
  // comes KN_PF MFMAs later (past the 40-cycle dependent latency)
  auto mfma = [&]() {
#pragma unroll
    for (int i = 0; i < KN_PF; ++i) cn[i] = knf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < KN_PF; ++i)
        cn[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(ld[i][kb], bfr[kb], cn[i], 0, 0, 0);
  };
  constexpr int G = 4 * KN_PF;
  load(wv);
  mfma();
  load(wv + G);
  for (int t0 = wv; t0 < nt; t0 += G) {
    knf4 c[KN_PF];
#pragma unroll
    for (int i = 0; i < KN_PF; ++i) c[i] = cn[i];
    mfma();                 // group t0 + G (its loads were issued a group ago)
    load(t0 + 2 * G);       // <= nt - 1 + 2 G + 4 (KN_PF - 1) < nt + KN_PAD
#pragma unroll
    for (int i = 0; i < KN_PF; ++i)
      if (t0 + 4 * i < nt) body(t0 + 4 * i, c[i]);
  }
}

template <int D>
__global__ __launch_bounds__(256) void knn_select_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t N, int64_t nq,
    const double* __restrict__ cen, const float* __restrict__ img,
    const double* __restrict__ R2p, int list_ok, int defer,
    unsigned long long* __restrict__ sel_v, long long* __restrict__ sel_jcut,
    long long* __restrict__ sel_rank0, int* __restrict__ need, int* __restrict__ done,
    double* __restrict__ lmom, int* __restrict__ counts /* [nfail, ndone] */) {
  constexpr int KB = kn_kb<D>();
  constexpr int NM = 2 + D + D * (D + 1) / 2;
  constexpr int PER = (KN_NB + 15) / 16;     // histogram bins per lane in the scan
  union Lds {
    uint32_t sample[KN_PB][KN_SK];
    struct { uint32_t bins[KN_PB][KN_NB]; uint32_t dummy[64]; } h;
    struct { double key[KN_PB][KN_CAP]; int idx[KN_PB][KN_CAP]; } list;
  };
  __shared__ Lds u;
  __shared__ float s_y[KN_PB][D];
  __shared__ uint32_t s_lo[KN_PB], s_below[KN_PB], s_cnt[KN_PB], s_rank0[KN_PB];
  __shared__ int s_sh[KN_PB], s_fail[KN_PB], s_rank[KN_PB];
  __shared__ double s_tlo[KN_PB], s_thi[KN_PB];
  __shared__ float s_clo[KN_PB], s_chi[KN_PB];
  __shared__ int s_list, s_nest[KN_PB], s_lm[KN_PB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
  const int pl = lane & 15;
  const int64_t p0 = (int64_t)blockIdx.x * KN_PB;
  const int nt = (int)((N + 15) / 16);
  const KnBound Bd = kn_bound<D>(*R2p);

  // ---- particle features (B operand) and the sample's fp32 coordinates
  float bfr[KB];
  double xn[D];
  {
    const int64_t n = p0 + pl < N ? p0 + pl : N - 1;
    float y[D];
    const float nn = kn_feat<D>(X, n, cen, y);
#pragma unroll
    for (int q = 0; q < D; ++q) xn[q] = X[n * D + q];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int k = 4 * kb + (lane >> 4);
      float v = 0.0f;
#pragma unroll
      for (int q = 0; q < D; ++q) if (k == q) v = -2.0f * y[q];
      if (k == D) v = 1.0f;
      if (k == D + 1) v = nn;
      bfr[kb] = v;
    }
    if (tid < KN_PB)
#pragma unroll
      for (int q = 0; q < D; ++q) s_y[tid][q] = y[q];
  }
  if (tid < KN_PB) { s_below[tid] = 0u; s_fail[tid] = 0; s_rank0[tid] = 0xFFFFFFFFu; s_cnt[tid] = 0u; }
  __syncthreads();

  // ---- 1. sample (direct fp32 differences: a guide only), sorted per
  // particle in registers: wave wv takes particles wv, wv + 4, ...; lane
  // holds sample elements 8 lane .. 8 lane + 7 (a bitonic network, partners
  // >= 8 apart through lane shuffles); the sorted sample goes to LDS
  {
    static_assert(KN_SK == 512, "8 sample elements per lane");
    float yq[8][D];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t j = ((2 * (int64_t)(8 * lane + i) + 1) * N) / (2 * KN_SK);
#pragma unroll
      for (int c = 0; c < D; ++c) yq[i][c] = (float)(X[j * D + c] - cen[c]);
    }
#pragma unroll 1
    for (int pi = 0; pi < KN_PB / 4; ++pi) {
      const int p = wv + 4 * pi;
      uint32_t x[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float sv = 0.0f;
#pragma unroll
        for (int c = 0; c < D; ++c) { const float t = yq[i][c] - s_y[p][c]; sv = __builtin_fmaf(t, t, sv); }
        x[i] = __float_as_uint(sv);
      }
#pragma unroll
      for (int size = 2; size <= KN_SK; size <<= 1)
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          if (stride >= 8) {
            const int lm = stride >> 3;
            const bool lower = (lane & lm) == 0;
            const bool asc = ((8 * lane) & size) == 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const uint32_t o = (uint32_t)__shfl_xor((int)x[i], lm, 64);
              const uint32_t mn = x[i] < o ? x[i] : o, mx = x[i] < o ? o : x[i];
              x[i] = (lower == asc) ? mn : mx;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int k = i ^ stride;
              if (k > i) {
                const bool asc = ((8 * lane + i) & size) == 0;
                const uint32_t a = x[i], b = x[k];
                const bool sw = (a > b) == asc;
                x[i] = sw ? b : a;
                x[k] = sw ? a : b;
              }
            }
          }
        }
#pragma unroll
      for (int i = 0; i < 8; ++i) u.sample[p][8 * lane + i] = x[i];
    }
  }
  __syncthreads();
  if (tid < KN_PB) {
    const int p = tid;
    const double pf = (double)(nq - 1) / (double)N;
    const int64_t mrg = 3 + (int64_t)(5.0 * sqrt(KN_SK * pf * (1.0 - pf)));
    const int64_t jk = ((nq - 1) * KN_SK) / N;
    // the smallest NONZERO sampled distance (the particle itself, or an
    // exact duplicate, in the sample would start the window at 0 and bin it
    // by whole binades)
    int z = 0;
    while (z < KN_SK - 1 && u.sample[p][z] == 0u) ++z;
    const uint32_t s0 = u.sample[p][z];
    const uint32_t lo = jk - mrg >= 0 ? u.sample[p][jk - mrg]
                                      : (s0 > (12u << 23) ? s0 - (12u << 23) : 0u);
    uint32_t hi = jk + mrg >= KN_SK ? 0x7F800000u : u.sample[p][jk + mrg];
    if (hi > 0x7F800000u) hi = 0x7F800000u;
    const int L = hi > lo ? 32 - __builtin_clz(hi - lo) : 0;
    const int sh = L > 9 ? L - 9 : 0;
    s_sh[p] = sh;
    s_lo[p] = lo >> sh;
  }
  __syncthreads();   // sample reads done; the LDS becomes the histogram
  for (int e = tid; e < KN_PB * KN_NB; e += 256) (&u.h.bins[0][0])[e] = 0u;
  const int sh = s_sh[pl];
  const uint32_t lor = s_lo[pl];
  __syncthreads();

  // ---- 2. count sweep
  uint32_t below = 0u;
  // per key: the below-window count in a register (branch-free) and an LDS
  // atomic for window keys only (exec-masked: the LDS atomic unit's cost
  // follows the active lanes).  Pad rows (key +inf) can only land in a bin
  // whose upper edge is +inf, and then T_hi = +inf.
  uint32_t* const hrow = &u.h.bins[pl][0];
  kn_sweep<KB>(img, nt, wv, lane, bfr, [&](int, const knf4& c) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t top = __float_as_uint(fmaxf(c[r], 0.0f)) >> sh;
      const uint32_t off = top - lor;
      below += top < lor ? 1u : 0u;
      if (off < (uint32_t)KN_NB) atomicAdd(hrow + off, 1u);
    }
  });
  below += __shfl_xor(below, 16, 64);
  below += __shfl_xor(below, 32, 64);
  if (lane < 16) atomicAdd(&s_below[pl], below);
  __syncthreads();

  // ---- the bin holding rank nq - 1: 16 lanes per particle
  {
    const int p = tid >> 4, l = tid & 15;
    const long long r = nq - 1 - (long long)s_below[p];
    long long v = 0;
    for (int b = l * PER; b < (l + 1) * PER && b < KN_NB; ++b) v += u.h.bins[p][b];
    long long inc = v;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const long long t = __shfl_up(inc, o, 16);
      if (l >= o) inc += t;
    }
    const long long tot = __shfl(inc, 15, 16);
    if (r < 0 || r >= tot) {
      if (l == 0) s_fail[p] = 1;
    } else if (r >= inc - v && r < inc) {
      long long run = inc - v;
      int b = l * PER;
      for (; b < KN_NB; ++b) {
        if (r < run + (long long)u.h.bins[p][b]) break;
        run += u.h.bins[p][b];
      }
      // (this thread's particle is p, not the sweep lane's pl)
      const uint64_t lb = (uint64_t)(s_lo[p] + (uint32_t)b) << s_sh[p];
      const uint64_t hb64 = (uint64_t)(s_lo[p] + (uint32_t)b + 1u) << s_sh[p];
      const double lv = lb >= 0x7F800000ull ? INFINITY : (double)__uint_as_float((uint32_t)lb);
      const double hv = hb64 >= 0x7F800000ull ? INFINITY : (double)__uint_as_float((uint32_t)hb64);
      double tlo = lv - Bd(lv);
      if (!(tlo > Bd.sc)) tlo = -INFINITY;
      const double bh = Bd(2.0 * hv);
      const double thi = (hv < 1e38 && bh <= hv) ? hv + bh : INFINITY;
      s_tlo[p] = tlo;
      s_thi[p] = thi;
      // #{s^ < h}: the list size of list mode, and of the bin in bin mode
      s_nest[p] = (int)min((long long)s_below[p] + run + (long long)u.h.bins[p][b], 1ll << 30);
      s_rank[p] = (int)((long long)u.h.bins[p][b]);
    }
  }
  __syncthreads();
  if (defer) {
    // deferred collect (dense k): the moments sweep classifies every pair
    // against [T_lo, T_hi) itself and queues the open ones
    // (knn_dense_kernel<D, true>, knn_resolve_kernel); the bracket leaves
    // here as two doubles, -inf for a particle whose window missed the rank
    // or whose bin would not fit the queue
    if (tid < KN_PB && p0 + tid < N) {
      const int p = tid;
      const bool bad = s_fail[p] || s_rank[p] + KN_MARGIN > KN_QCAP;
      sel_v[p0 + p] = (unsigned long long)__double_as_longlong(bad ? -INFINITY : s_tlo[p]);
      sel_jcut[p0 + p] = (long long)__double_as_longlong(bad ? -INFINITY : s_thi[p]);
      need[p0 + p] = bad ? 1 : 0;
    }
    return;
  }
  // list mode per particle: every neighbour fits the list
  if (tid < KN_PB)
    s_lm[tid] = (list_ok && kn_list_capable<D>() && !s_fail[tid] &&
                 s_nest[tid] + KN_MARGIN <= KN_CAP) ? 1 : 0;
  if (tid == 0) {
    int any = 0;
    for (int p = 0; p < KN_PB; ++p) any |= s_lm[p];
    s_list = any;
  }
  __syncthreads();
  const bool listm = s_list != 0;     // some particle of the block is listed
  if (tid < KN_PB) {
    const int p = tid;
    if (s_lm[p]) s_tlo[p] = -INFINITY;
    else if (!s_fail[p] && s_rank[p] + KN_MARGIN > KN_CAP) s_fail[p] = 1;
    s_clo[p] = s_fail[p] ? -INFINITY : kn_cut_below(s_tlo[p], Bd);
    s_chi[p] = s_fail[p] ? -INFINITY : kn_cut_above(s_thi[p], Bd);
    s_below[p] = 0u;
  }
  __syncthreads();

  // ---- 3. collect sweep
  {
    const float clo = s_clo[pl], chi = s_chi[pl];
    const double tlo = s_tlo[pl], thi = s_thi[pl];
    const float zc = kn_cut_above(0.0, Bd);       // s^ <= zc: possibly s64 == 0
    uint32_t below2 = 0u;
    // common path branch-free (certain-below count); keys between the cuts
    // ("open": rare) are settled in fp64 behind one wave-uniform branch
    kn_sweep<KB>(img, nt, wv, lane, bfr, [&](int t, const knf4& c) {
      bool open[4], any = false;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sk = c[r];
        const bool bel = sk < clo && sk > zc;
        below2 += bel ? 1u : 0u;
        open[r] = !(sk > chi) && !bel;
        any = any || open[r];
      }
      if (__builtin_amdgcn_ballot_w64(any) == 0ull) return;
      // open rows are queued (index only) and settled in fp64 after the
      // sweep, where their X rows load in parallel instead of stalling it
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * t + 4 * (lane >> 4) + r;
        if (!open[r] || j >= N) continue;
        const uint32_t slot = atomicAdd(&s_cnt[pl], 1u);
        if (slot < (uint32_t)KN_CAP) u.list.idx[pl][slot] = (int)j;
      }
    });
    below2 += __shfl_xor(below2, 16, 64);
    below2 += __shfl_xor(below2, 32, 64);
    if (lane < 16) atomicAdd(&s_below[pl], below2);
  }
  __syncthreads();
  // settle the queued rows in fp64: below T_lo counted, [T_lo, T_hi) kept
  // with their key, the rest (and the counted ones) keyed +inf, which no
  // rank below counts; s_nest = queue length, s_cnt = kept entries (a queue
  // overflow fails the particle)
  if (tid < KN_PB) {
    const uint32_t qn = s_cnt[tid];
    s_nest[tid] = (int)min(qn, (uint32_t)KN_CAP);
    if (qn > (uint32_t)KN_CAP) s_fail[tid] = 1;
    s_cnt[tid] = 0u;
  }
  __syncthreads();
  for (int e = tid; e < KN_PB * KN_CAP; e += 256) {
    const int p = e / KN_CAP, q = e % KN_CAP;
    if (q >= s_nest[p]) continue;
    const int j = u.list.idx[p][q];
    const int64_t n = p0 + p < N ? p0 + p : N - 1;
    double xp[D];
#pragma unroll
    for (int c = 0; c < D; ++c) xp[c] = X[n * D + c];
    const double s64 = dist2<D>(X, j, xp);
    if (s64 == 0.0) atomicMin(&s_rank0[p], (uint32_t)j);
    double kv = INFINITY;
    if (s64 < s_tlo[p]) atomicAdd(&s_below[p], 1u);
    else if (s64 < s_thi[p]) { kv = s64; atomicAdd(&s_cnt[p], 1u); }
    u.list.key[p][q] = kv;
  }
  __syncthreads();
  // ---- 4. select rank nq - 1 in (key, index) order among the list: wave wv
  // takes particles wv, wv + 4, ...; lane holds entries lane + 64 i in
  // registers and counts the smaller (key, index) pairs against broadcast
  // LDS reads of the list
  constexpr int EPL = KN_CAP / 64;
  int myrank[KN_PB / 4][EPL];
#pragma unroll
  for (int pi = 0; pi < KN_PB / 4; ++pi) {
    const int p = wv + 4 * pi;
    const int cnt = s_nest[p];
    const bool ok = !s_fail[p];
    double ke[EPL];
    int je[EPL], less[EPL];
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      const int q = lane + 64 * i;
      ke[i] = q < cnt ? u.list.key[p][q] : INFINITY;
      je[i] = q < cnt ? u.list.idx[p][q] : 0x7FFFFFFF;
      less[i] = 0;
    }
    if (ok)
      for (int f = 0; f < cnt; ++f) {
        const double kf = u.list.key[p][f];
        const int jf = u.list.idx[p][f];
#pragma unroll
        for (int i = 0; i < EPL; ++i) less[i] += (kf < ke[i]) || (kf == ke[i] && jf < je[i]);
      }
    const long long rr = nq - 1 - (long long)s_below[p];
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      const int q = lane + 64 * i;
      myrank[pi][i] = (ok && q < cnt) ? less[i] : -1;
      if (ok && q < cnt && less[i] == rr && p0 + p < N) {
        sel_v[p0 + p] = (unsigned long long)__double_as_longlong(ke[i]);
        sel_jcut[p0 + p] = (long long)je[i] + 1;
        sel_rank0[p0 + p] = s_rank0[p] == 0xFFFFFFFFu ? N : (long long)s_rank0[p];
      }
    }
  }
  __syncthreads();
  if (tid < KN_PB && p0 + tid < N) {
    const int p = tid;
    const long long rr = nq - 1 - (long long)s_below[p];
    const bool bad = s_fail[p] || rr < 0 || rr >= (long long)s_cnt[p];
    need[p0 + p] = bad ? 1 : 0;
    done[p0 + p] = (!bad && s_lm[p]) ? 1 : 0;
    if (bad) atomicAdd(&counts[0], 1);
    else if (s_lm[p]) atomicAdd(&counts[1], 1);
    s_fail[p] = bad ? 1 : 0;
  }
  if constexpr (kn_list_capable<D>()) {
    if (!listm) return;
    __syncthreads();
    // rank -> row index, written over the key array (keys no longer read)
    int* ord = reinterpret_cast<int*>(&u.list.key[0][0]);
#pragma unroll
    for (int pi = 0; pi < KN_PB / 4; ++pi)
#pragma unroll
      for (int i = 0; i < EPL; ++i) {
        const int p = wv + 4 * pi, q = lane + 64 * i;
        if (myrank[pi][i] >= 0 && myrank[pi][i] < nq) ord[p * KN_CAP + myrank[pi][i]] = u.list.idx[p][q];
      }
    __syncthreads();
    // ---- 5. list mode: the neighbours' moments, rank order per lane, then a
    // fixed-order wave reduction (deterministic)
    for (int p = wv; p < KN_PB; p += 4) {
      const int64_t n = p0 + p;
      if (n >= N || s_fail[p] || !s_lm[p]) continue;
      const long long r0 = s_rank0[p] == 0xFFFFFFFFu ? N : (long long)s_rank0[p];
      double xp[D];
#pragma unroll
      for (int q = 0; q < D; ++q) xp[q] = X[n * D + q];
      double m[NM];
#pragma unroll
      for (int t = 0; t < NM; ++t) m[t] = 0.0;
      for (int r = lane; r < nq; r += 64) {
        const int j = ord[p * KN_CAP + r];
        if (j == r0) continue;
        const double lw = w[j];
        double dj[D];
#pragma unroll
        for (int q = 0; q < D; ++q) dj[q] = X[(int64_t)j * D + q] - xp[q];
        m[0] += lw;
        m[1] += lw * lw;
        int c = 2 + D;
#pragma unroll
        for (int a = 0; a < D; ++a) {
          m[2 + a] += lw * dj[a];
#pragma unroll
          for (int b = a; b < D; ++b) { m[c] += lw * dj[a] * dj[b]; ++c; }
        }
      }
#pragma unroll
      for (int t = 0; t < NM; ++t) {
        const double v = wave_sum(m[t]);
        if (lane == 0) lmom[(int64_t)t * N + n] = v;
      }
    }
  }
}

