// MultivariateNormalTransition.pdf, "x3" precision: the whitened cross-term
// GEMM on f16 MFMA (v_mfma_f32_32x32x16_f16) with every operand split into
// three 11-bit limbs, exact-grid accumulation in f32, fused with exp2 and the
// weighted sum over the population.  Result accuracy is that of an f32
// direct-difference evaluation (~1e-7 relative; tested at 2e-6 against the
// fp64 oracle), at f16-MFMA issue rates.
//
// Reference: pyabc/transition/multivariatenormal.py:99-113,
//   dens(x_i) = sum_j w_j N(x_i - X_j; 0, Sigma),
// restated with the fit's fp64 whitening U (U U^T = Sigma^-1; abc_mvn_fit) and the
// log2 scaling folded into the coordinates (q = sqrt(log2 e)):
//   y_j = q (X_j - mu) U,  z_i = q (x_i - mu) U
//   s_ij = c_j - m_i + z_i . y_j              (log2 units, s_ij <= 0)
//   c_j = log2e (log w_j - log w_max) - |y_j|^2 / 2,   m_i = |z_i|^2 / 2
//   dens(x_i) = exp(log_const) * sum_j 2^s_ij,  log_const = log_norm + log w_max
//
// Limbs.  With the grid unit G = 2^(E-11), E chosen per fit on the device
// from the population's largest whitened norm (E = max(3, ceil(log2(1.25
// max|y| + 2 sqrt(r) + 4))), E <= 8), a coordinate v (|v| <= 2^E) is
//   v = a1 G + a2 G 2^-11 + a3 G 2^-22      (a1, a2, a3 integers, |a| <= 2048)
// and every slot value is such an integer times a power of two, so it is an
// exact f16 (subnormal f16 operands and products are exact on gfx950: probe
// tools/probes/mfma_f16_numerics.hip) and every product an exact f32.  Kept
// products (limb indices p, q in 1..3) are the classes p + q <= 4:
//   class 0: v1 w1                      multiples of G^2
//   class 1: v1 w2 + v2 w1              multiples of G^2 2^-11
//   class 2: v1 w3 + v2 w2 + v3 w1      multiples of G^2 2^-22
// c and m are split into five limbs on the grids 2^22 G^2, 2^11 G^2, G^2
// (hi) and G^2 2^-11, G^2 2^-22 (lo).  The K dimension holds, in this order,
//   exact groups : class 0 (r), C0 C1 C2, M0 M1 M2, O  -> r + 7, padded to
//                  whole 8-slot groups (g0 = ceil((r + 7) / 8))
//   lo groups    : class 1 (2r), class 2 (3r), C3 C4, M3 M4 -> 5r + 4
// and is run as KB = ceil((8 g0 + 5r + 4) / 16) v_mfma_f32_32x32x16_f16
// (K = 80 at r = 10: 5 instructions per 32x32 tile pair against the 16x16
// layout's 6 per 2x2 16x16 tiles).  The f16 MFMA sums each group of 8
// products wide and adds the groups to the accumulator in K order with f32
// rounding (probes: tools/probes/mfma_f16_groups.hip for 16x16x32,
// mfma32_f16_sum.hip for 32x32x16 -- K 0-7 then K 8-15, an exact-grid block
// sums exactly), so an exact group must not share an 8-slot group with lo
// terms but may share an MFMA with them.  Every exact-group
// term is a multiple of G^2 and every partial sum is bounded by |c| + |m| + |o| +
// |z||y| < 2^(2E+2) = 2^24 G^2 (norm checks below), so the exact groups sum
// EXACTLY.  O is
// a per-candidate integer offset (B = -o, A = 1): a first pass over the
// chunk runs the exact groups alone (exact s_hi) to find each
// column's max, then o = ceil(max s_hi) is written into the B fragment and
// the main pass leaves s - o <= 1 with the dominant pairs near 0, so the lo
// groups round at 2^-24 |s - o|.  Dropped
// terms (class 3, limb residual) are < 2^(2E-35) per coordinate; numpy
// emulation of this exact scheme: <= 1e-7 relative on the golden vectors.
//
// Layout (HBM): image = 256-byte header (max |y|^2/2, E, ok) + fragments
// [NT][KB][64 lanes][8 halves] of 32-row tiles in the order of
// v_mfma_f32_32x32x16_f16 (lane l holds row l & 31, k = 16 kb + 8 (l >> 5) +
// j); the population image is built once per fit, the candidate image per
// call.  Each lane owns ONE candidate column (l & 31) and sixteen population
// rows of every 32x32 tile (rows (i & 3) + 8 (i >> 2) + 4 (l >> 5)), so the
// sum over the population stays in registers until a final 2-lane
// combine.  Candidates outside the norm bound, and candidates whose density
// underflows 2^-60 relative to max w (all pairs beyond ~11 kernel widths),
// are recomputed in fp64 from the whitened population Y and log2 weights lw
// stored after the fragments (rescue list; empty in practice).
#include "abc_common.h"

namespace abc {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr double LOG2E = 1.4426950408889634074;
constexpr double SQRT_LOG2E = 1.2011224087864498;  // sqrt(log2 e)
constexpr double LN2 = 0.69314718055994530942;
constexpr int MAX_R = 25;       // exact groups r + 7 <= 32
constexpr int E_MIN = 3, E_MAX = 8;
constexpr float O_MIN = -64.f;  // offsets below this: density < 2^-60 -> rescue
constexpr size_t HDR = 256;     // image header bytes
constexpr int X3_PAD = 8;       // pad tiles after the population fragments
constexpr int TR = 32;          // rows (and candidate columns) per tile

struct Header { double maxsq; int E; int ok; };

// exact 8-slot groups, their padded slot count, MFMA instructions per tile
// pair, and the instructions the max pass needs (those holding exact groups)
__host__ __device__ constexpr int x3_g0(int r) { return (r + 7 + 7) / 8; }
__host__ __device__ constexpr int x3_k0pad(int r) { return 8 * x3_g0(r); }
__host__ __device__ constexpr int x3_kb(int r) { return (x3_k0pad(r) + 5 * r + 4 + 15) / 16; }
__host__ __device__ constexpr int x3_kb0(int r) { return (x3_g0(r) + 1) / 2; }
static_assert(x3_kb(10) == 5, "K = 80 at r = 10");

struct Limbs3 { double a1, a2, a3; };  // integers
struct Limbs5 { double c[5]; };        // integers

__device__ __forceinline__ Limbs3 split_coord(double v, int E) {
  Limbs3 L;
  const double G = ldexp(1.0, E - 11);
  L.a1 = rint(v / G);
  double r = v - L.a1 * G;
  L.a2 = rint(ldexp(r / G, 11));
  r -= ldexp(L.a2 * G, -11);
  L.a3 = rint(ldexp(r / G, 22));
  return L;
}

// grid exponent (log2) of scalar limb l: 2E-22 + {22, 11, 0, -11, -22}
__device__ __forceinline__ int scalar_exp(int l, int E) { return 2 * E - 22 + 22 - 11 * l; }

__device__ __forceinline__ Limbs5 split_scalar(double c, int E) {
  Limbs5 L;
  double r = c;
  for (int l = 0; l < 5; ++l) {
    const int e = scalar_exp(l, E);
    L.c[l] = rint(ldexp(r, -e));
    r -= ldexp(L.c[l], e);
  }
  return L;
}

// limb x 2^e as an (exact) f16 operand value
__device__ __forceinline__ float opv(double limb, int e) { return (float)ldexp(limb, e); }

// Value of K slot k for the population side (SIDE 0, A operand: carries c)
// or the candidate side (SIDE 1, B operand: carries -m and the offset).
template <int SIDE>
__device__ __forceinline__ float slot_value(int k, int r, int K0pad, int E,
                                            const Limbs3* L, const Limbs5& S) {
  if (k < K0pad) {
    const int e0 = 2 * (E - 11);
    if (k < r) {  // class 0: a1 b1 G^2
      const int x = e0 >> 1;  // floor
      return opv(L[k].a1, SIDE == 0 ? x : e0 - x);
    }
    const int q = k - r;
    if (q < 6) {  // scalar hi limbs: 0..2 = c (A), 3..5 = m (B)
      const int l = q % 3;
      const int e = scalar_exp(l, E);
      const int x = e > 4 ? 4 : e;  // limb side exponent (|limb| <= 2048)
      const bool limb_side = (q < 3) == (SIDE == 0);
      return limb_side ? opv(S.c[l], x) : opv(1.0, e - x);
    }
    if (q == 6) return SIDE == 0 ? 1.f : 0.f;  // O: B = -o (set in the kernel)
    return 0.f;
  }
  const int q = k - K0pad;
  if (q < 5 * r) {
    const int cls = q / r, dim = q % r;
    // (p, q) limb pairs: (1,2) (2,1) (1,3) (2,2) (3,1)
    const int pa[5] = {1, 2, 1, 2, 3}, pb[5] = {2, 1, 3, 2, 1};
    const int p = SIDE == 0 ? pa[cls] : pb[cls];
    const int etot = 2 * (E - 11) - 11 * (pa[cls] + pb[cls] - 2);
    const int x = etot >> 1;
    const double limb = p == 1 ? L[dim].a1 : (p == 2 ? L[dim].a2 : L[dim].a3);
    return opv(limb, SIDE == 0 ? x : etot - x);
  }
  const int e4 = q - 5 * r;
  if (e4 < 4) {  // scalar lo limbs: 0..1 = c (A), 2..3 = m (B)
    const int l = 3 + (e4 & 1);
    const int e = scalar_exp(l, E);
    const int x = e < -24 ? -24 : e;  // limb side
    const bool limb_side = (e4 < 2) == (SIDE == 0);
    return limb_side ? opv(S.c[l], x) : opv(1.0, e - x);
  }
  return 0.f;
}

// Whitened, log2-scaled point of row `row`; returns |v|^2 / 2.
template <int RR = MAX_R>
__device__ __forceinline__ double whiten(const double* __restrict__ P, int64_t row,
                                         int d, const double* __restrict__ mu,
                                         const double* __restrict__ U, int r,
                                         double* v) {
  double acc[RR];
#pragma unroll
  for (int k = 0; k < RR; ++k) acc[k] = 0.0;
  for (int q = 0; q < d; ++q) {  // each row element loaded once
    const double xq = P[row * d + q] - mu[q];
#pragma unroll
    for (int k = 0; k < RR; ++k)
      if (k < r) acc[k] += xq * U[q * r + k];
  }
  double h = 0.0;
#pragma unroll
  for (int k = 0; k < RR; ++k) {
    if (k < r) {
      const double a = acc[k] * SQRT_LOG2E;
      v[k] = a;
      h += a * a;
    }
  }
  return 0.5 * h;
}

// max |y_j|^2 / 2 over the rows with w > 0 (atomicMax on the bit pattern of
// a non-negative double, which is monotone).  Grid-stride over at most
// POP_RANGE_BLOCKS blocks, one atomic per block: one per wave on the single
// address serialised ~16k atomics per c3 population (0.2 ms).
constexpr int POP_RANGE_BLOCKS = 1024;
__global__ __launch_bounds__(256) void pop_range_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t N,
    int d, const double* __restrict__ mu, const double* __restrict__ U, int r,
    Header* __restrict__ hdr) {
  __shared__ double wm[4];
  double h = 0.0;
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < N;
       row += (int64_t)gridDim.x * blockDim.x) {
    if (w[row] > 0.0) {
      double v[MAX_R];
      h = fmax(h, whiten(X, row, d, mu, U, r, v));
    }
  }
  h = wave_max(h);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    h = fmax(fmax(wm[0], wm[1]), fmax(wm[2], wm[3]));
    if (h > 0.0)
      atomicMax((unsigned long long*)&hdr->maxsq,
                (unsigned long long)__double_as_longlong(h));
  }
}

__global__ void x3_setup_kernel(Header* __restrict__ hdr, int r,
                                double* __restrict__ range) {
  const double ymax = sqrt(2.0 * hdr->maxsq);
  int E = (int)ceil(log2(1.25 * ymax + 2.0 * sqrt((double)r) + 4.0));
  if (E < E_MIN) E = E_MIN;
  hdr->E = E;
  hdr->ok = E <= E_MAX ? 1 : 0;
  if (range) { range[0] = ymax; range[1] = (double)E; }
}

// One thread per image row (population row or candidate column): computes the
// limbs and scatters the K slot values into the fragment image.  R > 0 fixes
// the rank at compile time (limb arrays in registers, slot loop unrolled);
// R = 0 handles any r <= MAX_R with the arrays in scratch.
template <int SIDE, int R>
__global__ __launch_bounds__(128) void pack_x3_kernel(
    const double* __restrict__ P, const double* __restrict__ w, int64_t n,
    int d, const double* __restrict__ mu, const double* __restrict__ U, int r_rt,
    double log_w_shift, int K0pad_rt, int KB_rt, const Header* __restrict__ hdr,
    _Float16* __restrict__ img, int64_t ntiles, int32_t* __restrict__ flags,
    double* __restrict__ Y, double* __restrict__ lw, int64_t Np,
    const int64_t* __restrict__ hint, float* __restrict__ cand_o, int koff,
    const double* __restrict__ shift_dev, const unsigned int* __restrict__ count_dev) {
  // SIDE 0 writes the fp64 whitened population Y [n x r] and its log2
  // weights lw [n] (rescue + hints); SIDE 1 reads them for the hint rows.
  // count_dev (SIDE 1, nullable): only the first *count_dev of the n rows
  // are candidates (a device-sized launch), the rest are padding
  if (count_dev) { const int64_t c = (int64_t)*count_dev; n = c < n ? c : n; }
  constexpr int RR = R > 0 ? R : MAX_R;
  const int r = R > 0 ? R : r_rt;
  const int K0pad = R > 0 ? x3_k0pad(R) : K0pad_rt;
  const int KB = R > 0 ? x3_kb(R) : KB_rt;
  constexpr int NG = R > 0 ? x3_kb(R) * 2 : 0;  // 8-slot groups
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= ntiles * TR) return;
  // tiles wholly past the count are never read (the waves that own them leave)
  if (count_dev && (row / TR) * TR >= n) return;
  const int E = hdr->E;
  const bool ok = hdr->ok != 0;
  const double L2 = ldexp(1.0, 2 * E);  // 2^(2E): bound of |y|^2 and |c|
  double v[RR];
  Limbs3 L[RR];
  double scalar = SIDE == 0 ? -L2 : 0.0;  // padding: c = -2^(2E), m = 0
  bool bad = false;
  float hint_o = O_MIN;
  #pragma unroll
  for (int k = 0; k < RR; ++k) v[k] = 0.0;
  if (row < n) {
    const double h = whiten<RR>(P, row, d, mu, U, r, v);
    if (SIDE == 0) {
      const double wj = w[row];
      bad = !(wj > 0.0) || !(2.0 * h <= L2);
      const double sh = shift_dev ? *shift_dev : log_w_shift;
      const double lwj = wj > 0.0 ? (log(wj) + sh) * LOG2E : -INFINITY;
      scalar = bad ? -L2 : fmax(lwj - h, -L2);
#pragma unroll
      for (int k = 0; k < RR; ++k)
        if (k < r) Y[row * r + k] = v[k];
      lw[row] = lwj;
    } else {
      bad = !ok || !(2.0 * h <= L2);
      scalar = bad ? -L2 : -h;
      if (hint && !bad) {
        // offset from the hint row j (the proposal's ancestor): the exact
        // fp64 exponent s_ij = log2e (log w_j + shift) - |z_i - y_j|^2 / 2,
        // rounded up to an integer, replaces the max pre-pass
        const int64_t j = hint[row];
        if (j < 0 || j >= Np || !(lw[j] > -INFINITY)) {
          bad = true;
        } else {
          double q = 0.0;
#pragma unroll
          for (int k = 0; k < RR; ++k)
            if (k < r) { const double t = v[k] - Y[j * r + k]; q += t * t; }
          hint_o = (float)fmax(ceil(lw[j] - 0.5 * q), (double)O_MIN);
        }
        scalar = bad ? -L2 : -h;
      }
    }
    if (bad)
      #pragma unroll
  for (int k = 0; k < RR; ++k) v[k] = 0.0;
  }
  if (flags && row < n) flags[row] = bad ? 1 : 0;
  if (cand_o) cand_o[row] = hint_o;
#pragma unroll
  for (int k = 0; k < RR; ++k) L[k] = split_coord(v[k], E);
  const Limbs5 S = split_scalar(scalar, E);
  const int64_t t = row / TR;
  const int rl = (int)(row % TR);
  const int Ktot = 16 * KB;
  // 8 consecutive K slots of this row form one lane's 16-byte fragment:
  // assemble them in registers and store them as one vector
#pragma unroll
  for (int g = 0; g < (R > 0 ? NG : 1 << 30); ++g) {
    if (g >= Ktot / 8) break;
    half8 frag;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = g * 8 + j;
      float val = slot_value<SIDE>(k, r, K0pad, E, L, S);
      if (SIDE == 1 && hint && k == koff) val = -hint_o;  // B = -o (A = 1)
      frag[j] = (_Float16)val;
    }
    const int kb = g >> 1, lane = rl + 32 * (g & 1);
    *reinterpret_cast<half8*>(img + (((t * KB + kb) * 64) + lane) * 8) = frag;
  }
}

// ---- the fused limb-split GEMM + exp2 + weighted sum -----------------------
// One wave = CT candidate tiles (32 columns each) x one population chunk;
// block = 4 waves; 1-D grid, block b -> XCD b % 8 owns chunks {xcd, xcd + 8,
// ...} so that the blocks sharing a population chunk share one XCD's L2
// (speed only).
// Pass 1: the exact groups only -> per-column max of s_hi -> integer offset o.
// Pass 2: all groups -> per lane, sum over its population rows of 2^(s - o).
__device__ __forceinline__ float max3(float a, float b, float c) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

__device__ __forceinline__ f32x16 mfma32(const half8& a, const half8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// one wave's work: candidate tiles ct0 .. ct0 + CT - 1 against population
// chunk `chunk`
template <int KB, int CT, bool PASS1>
__device__ __forceinline__ void x3_wave(
    const half8* __restrict__ A, const half8* __restrict__ Bi, int64_t MT,
    int64_t NT, int chunk, int64_t tiles_per_chunk, int64_t ct0, int koff, int kb0,
    double* __restrict__ part_o, double* __restrict__ part_l, int64_t Mpad) {
  const int lane = threadIdx.x & 63;
  // which lanes / instruction / element of the B fragments hold the offset slot
  const bool off_lane = (lane >> 5) == ((koff >> 3) & 1);
  const int off_kb = koff >> 4, off_j = koff & 7;

  half8 b[CT][KB];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int64_t ct = ct0 + c < MT ? ct0 + c : MT - 1;  // clamp: dup work, never stored
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) b[c][kb] = Bi[(ct * KB + kb) * 64 + lane];
  }
  const int64_t t_begin = (int64_t)chunk * tiles_per_chunk;
  const int64_t t_end = t_begin + tiles_per_chunk < NT ? t_begin + tiles_per_chunk : NT;
  const half8* __restrict__ Al = A + lane;
  // prefetches run up to 7 tiles past the chunk end (t_end <= NT); the image
  // carries X3_PAD = 8 pad tiles, so no clamp is needed (pad data is loaded,
  // never used).  A chunk starting at or past NT (small N) loads nothing.
  static_assert(X3_PAD >= 7, "pad must cover the prefetch distance");
  auto tile = [&](int64_t t) { return t * KB; };
  const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f,
                         0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  // ---- pass 1: exact s_hi (offset slot still 0) -> column max -> o.  The
  // instructions holding exact groups (kb < kb0 <= 2) through a ring of 4
  // tiles (prefetch distance 4).
  float o[CT];
  if (PASS1 && t_begin < t_end) {
    float mx[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) mx[c] = -INFINITY;
    half8 ring[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        if (kb < KB) ring[u][kb] = Al[(tile(t_begin + u) + kb) * 64];
    for (int64_t t = t_begin; t < t_end; t += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (t + u < t_end) {
#pragma unroll
          for (int c = 0; c < CT; ++c) {
            f32x16 acc = mfma32(ring[u][0], b[c][0], zero16);
            if (KB > 1 && kb0 > 1) acc = mfma32(ring[u][1], b[c][1 < KB ? 1 : 0], acc);
            float m = mx[c];
#pragma unroll
            for (int i = 0; i < 16; i += 2) m = max3(m, acc[i], acc[i + 1]);
            mx[c] = m;
          }
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          if (kb < KB) ring[u][kb] = Al[(tile(t + u + 4) + kb) * 64];
      }
    }
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const float cm = fmaxf(mx[c], __shfl_xor(mx[c], 32, 64));
      o[c] = fmaxf(ceilf(cm), O_MIN);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
        if (kb == off_kb && off_lane) b[c][kb][off_j] = (_Float16)(-o[c]);
    }
  } else {
#pragma unroll
    for (int c = 0; c < CT; ++c) o[c] = O_MIN;
  }

  // ---- pass 2: full limb-split GEMM, exp2, sums.  Two register buffers of
  // population fragments (prefetch distance 2).  Work runs as a stream of
  // (tile, c) units: the MFMA chain of unit u is issued next to the
  // exp2/sum of unit u-1, so one wave keeps the MFMA and VALU pipes busy.
  double l64[CT];
  float ls[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) { l64[c] = 0.0; ls[c] = 0.f; }
  half8 a0[KB], a1[KB];
  if (t_begin < t_end) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      a0[kb] = Al[(tile(t_begin) + kb) * 64];
      a1[kb] = Al[(tile(t_begin + 1) + kb) * 64];
    }
  }
  auto chain = [&](const half8 (&a)[KB], int c) {
    f32x16 r = mfma32(a[0], b[c][0], zero16);
#pragma unroll
    for (int kb = 1; kb < KB; ++kb) r = mfma32(a[kb], b[c][kb], r);
    return r;
  };
  auto expsum = [&](const f32x16& v) {
    float e[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) e[i] = __builtin_amdgcn_exp2f(v[i]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int i = 0; i < w; ++i) e[i] += e[i + w];
    return e[0];
  };
  // one tile: units (t, 0..CT-1); the exp2/sum of unit c - 1 is issued under
  // the MFMA chain of unit c.  Every candidate slot c sums the same tiles in
  // the same order, so a candidate's bits do not depend on where it sits in
  // the launch (and so not on the sharding over ranks).
  auto do_tile = [&](const half8 (&a)[KB]) {
    f32x16 prev = chain(a, 0);
#pragma unroll
    for (int c = 1; c < CT; ++c) {
      const f32x16 cur = chain(a, c);
      ls[c - 1] += expsum(prev);
      prev = cur;
    }
    ls[CT - 1] += expsum(prev);
  };
  int nflush = 0;
  for (int64_t t = t_begin; t < t_end; t += 2) {
    do_tile(a0);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) a0[kb] = Al[(tile(t + 2) + kb) * 64];
    if (t + 1 < t_end) {
      do_tile(a1);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) a1[kb] = Al[(tile(t + 3) + kb) * 64];
    }
    // f32 partial sums over at most 4 tiles (64 terms per lane), then fp64
    if (++nflush == 2) {
      nflush = 0;
#pragma unroll
      for (int c = 0; c < CT; ++c) { l64[c] += (double)ls[c]; ls[c] = 0.f; }
    }
  }
#pragma unroll
  for (int c = 0; c < CT; ++c) l64[c] += (double)ls[c];
  // lanes l and l ^ 32 hold the same candidate column (same o)
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    double v = l64[c];
    v += __shfl_xor(v, 32, 64);
    const int64_t ct = ct0 + c;
    if (lane < 32 && ct < MT) {
      if (PASS1) part_o[(int64_t)chunk * Mpad + ct * TR + lane] = (double)o[c];
      part_l[(int64_t)chunk * Mpad + ct * TR + lane] = v;
    }
  }
}

// blocks: (groups of 4 waves x CT candidate tiles) x population chunks; a
// device-sized launch (count_dev) covers a few groups and strides over the
// rest, its waves past the candidate count leaving at once (no barrier in
// this kernel); a full launch has every group in the grid (one pass)
template <int KB, int CT, bool PASS1>
__global__ __launch_bounds__(256) void mvn_x3_kernel(
    const half8* __restrict__ A, const half8* __restrict__ Bi, int64_t MT,
    int64_t NT, int nchunk, int64_t tiles_per_chunk, int64_t ngroups, int koff, int kb0,
    double* __restrict__ part_o, double* __restrict__ part_l, int64_t Mpad,
    const unsigned int* __restrict__ count_dev) {
  const int wave = threadIdx.x >> 6;
  const int64_t bid = blockIdx.x;
  const int cpx = nchunk >> 3;
  const int64_t xcd = bid & 7, jb = bid >> 3;
  const int chunk = (int)(xcd + 8 * (jb % cpx));
  const int64_t gstride = (int64_t)gridDim.x / nchunk;
  const int64_t cnt = count_dev ? (int64_t)*count_dev : MT * TR;
  for (int64_t group = jb / cpx; group < ngroups; group += gstride) {
    const int64_t ct0 = (group * 4 + wave) * CT;
    if (ct0 * TR >= cnt) break;
    x3_wave<KB, CT, PASS1>(A, Bi, MT, NT, chunk, tiles_per_chunk, ct0, koff, kb0, part_o,
                           part_l, Mpad);
  }
}

__global__ void x3_combine_kernel(const double* __restrict__ part_o,
                                  const double* __restrict__ part_l, int nchunk,
                                  int64_t M, int64_t Mpad, double log_const,
                                  const int32_t* __restrict__ cflags,
                                  const float* __restrict__ cand_o,
                                  double* __restrict__ out,
                                  int64_t* __restrict__ rescue,
                                  unsigned int* __restrict__ nrescue,
                                  const unsigned int* __restrict__ count_dev) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M || (count_dev && i >= (int64_t)*count_dev)) return;
  double om = -INFINITY;
  double s = 0.0;
  if (cand_o) {  // one offset per candidate (hinted launch): plain sum
    om = (double)cand_o[i];
    for (int c = 0; c < nchunk; ++c) s += part_l[(int64_t)c * Mpad + i];
  } else {
    for (int c = 0; c < nchunk; ++c)
      if (part_l[(int64_t)c * Mpad + i] > 0.0) om = fmax(om, part_o[(int64_t)c * Mpad + i]);
    for (int c = 0; c < nchunk; ++c) {
      const double l = part_l[(int64_t)c * Mpad + i];
      if (l > 0.0) s += l * exp2(part_o[(int64_t)c * Mpad + i] - om);
    }
  }
  const double lg = om + log2(s);  // log2 of sum_j 2^s_ij
  // below 2^-60 (relative to max w) terms flushed at the f32 exp2 floor
  // could matter: recompute in fp64
  // hinted offsets: the dominant terms round at 2^-24 |s - o| <= 2^-24
  // (lg - om); beyond lg - om > 20 (offset far below the true maximum, or
  // > 2^20 comparable terms) recompute in fp64 too
  if (cflags[i] || !(s > 0.0) || !(lg >= -60.0) || (cand_o && lg - om > 20.0)) {
    const unsigned int q = atomicAdd(nrescue, 1u);
    rescue[q] = i;
    out[i] = -INFINITY;
    return;
  }
  out[i] = log_const + LN2 * lg;
}

// Unhinted combine of a device-sized launch (the nested rescue pass: a few
// rows, up to 256 chunks): one wave per row, lanes over the chunks, so the
// row's partials are read in parallel rather than one latency-bound load
// after the other.  Max by a butterfly (exact); the sum adds each lane's
// chunks c, c+64, ... in order and then butterflies in a fixed pattern, so
// a row's bits depend on N (the chunking) only, never on M or its slot.
__global__ __launch_bounds__(256) void x3_combine_rows_kernel(
    const double* __restrict__ part_o, const double* __restrict__ part_l, int nchunk,
    int64_t M, int64_t Mpad, double log_const, const int32_t* __restrict__ cflags,
    double* __restrict__ out, int64_t* __restrict__ rescue,
    unsigned int* __restrict__ nrescue, const unsigned int* __restrict__ count_dev) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= M || i >= (int64_t)*count_dev) return;
  double om = -INFINITY;
  for (int c = lane; c < nchunk; c += 64)
    if (part_l[(int64_t)c * Mpad + i] > 0.0) om = fmax(om, part_o[(int64_t)c * Mpad + i]);
  for (int m = 32; m >= 1; m >>= 1) om = fmax(om, __shfl_xor(om, m, 64));
  double s = 0.0;
  for (int c = lane; c < nchunk; c += 64) {
    const double l = part_l[(int64_t)c * Mpad + i];
    if (l > 0.0) s += l * exp2(part_o[(int64_t)c * Mpad + i] - om);
  }
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (lane) return;
  const double lg = om + log2(s);
  if (cflags[i] || !(s > 0.0) || !(lg >= -60.0)) {
    const unsigned int q = atomicAdd(nrescue, 1u);
    rescue[q] = i;
    out[i] = -INFINITY;
    return;
  }
  out[i] = log_const + LN2 * lg;
}

// Rescue of the listed candidates over the stored whitened population:
// s_ij = lw_j - |z_i - y_j|^2 / 2 (log2 units, the same s as the MFMA path)
// in fp64, accumulated as an online (max, sum) pair in fp64 with f32 exp2 of
// the fp64 difference (1e-7 relative per term).
__device__ __forceinline__ void online_add(double s, double& m, double& l) {
  const double dl = s - m;
  // a new maximum rescales the running sum in fp64 (rare; an f32 factor
  // here compounds over a long scan), terms below it take the f32 exp2
  if (dl > 0.0) { l = l * exp2(-dl) + 1.0; m = s; }
  else l += (double)__builtin_amdgcn_exp2f((float)dl);
}

// Rescue v2: one rescued candidate per lane with its whitened coordinates
// in registers; the population is cut in RS slices that depend on N only
// (so a candidate's summation order -- and its bits -- do not depend on how
// many others are rescued or on the sharding) and streamed through 64-row
// LDS tiles read at broadcast addresses.  Block = one wave = 64 candidates x
// one slice; (max, sum) partials go to pm / pl [slice][q - q0] (the main
// kernel's partial arrays, free after combine), candidates [q0, q0 + cap)
// per launch pair.
constexpr int RS_ROWS = 4096;   // population rows per slice (at least)
constexpr int RS_MAXS = 256;    // slices at most
constexpr int RS_GY = 8;        // candidate-group blocks per slice

__host__ __device__ inline int rescue_slices(int64_t N) {
  const int64_t s = (N + RS_ROWS - 1) / RS_ROWS;
  return (int)(s < 1 ? 1 : (s > RS_MAXS ? RS_MAXS : s));
}

__global__ __launch_bounds__(64) void x3_rescue_kernel(
    const int64_t* __restrict__ rescue, const unsigned int* __restrict__ nrescue,
    int64_t q0, int64_t cap, const double* __restrict__ x, int d,
    const double* __restrict__ mu, const double* __restrict__ U, int r,
    const double* __restrict__ Y, const double* __restrict__ lw, int64_t N,
    double* __restrict__ pm, double* __restrict__ pl) {
  __shared__ double ty[64 * MAX_R];
  __shared__ double tl[64];
  const int64_t n = (int64_t)*nrescue;
  const int64_t nq = n - q0 < cap ? n - q0 : cap;   // this launch's candidates
  const int lane = threadIdx.x;
  const int ns = gridDim.x;
  const int64_t per = (N + ns - 1) / ns;
  const int64_t j0 = (int64_t)blockIdx.x * per;
  const int64_t j1 = j0 + per < N ? j0 + per : N;
  for (int64_t g0 = (int64_t)blockIdx.y * 64; g0 < nq; g0 += (int64_t)gridDim.y * 64) {
    const int64_t q = g0 + lane;
    const bool act = q < nq;
    double z[MAX_R];
    const int64_t i = act ? rescue[q0 + q] : 0;
#pragma unroll
    for (int k = 0; k < MAX_R; ++k) {
      if (k < r) {
        double acc = 0.0;
        for (int cc = 0; cc < d; ++cc) acc += (x[i * d + cc] - mu[cc]) * U[cc * r + k];
        z[k] = acc * SQRT_LOG2E;
      }
    }
    double m = -INFINITY, l = 0.0;
    for (int64_t jt = j0; jt < j1; jt += 64) {
      const int cnt = (int)(j1 - jt < 64 ? j1 - jt : 64);
      __syncthreads();
      for (int e = lane; e < cnt * r; e += 64) ty[e] = Y[jt * r + e];
      if (lane < cnt) tl[lane] = lw[jt + lane];
      __syncthreads();
      for (int t = 0; t < cnt; ++t) {
        const double lwj = tl[t];
        if (!(lwj > -INFINITY)) continue;
        double q2 = 0.0;
#pragma unroll
        for (int k = 0; k < MAX_R; ++k) {
          if (k < r) {
            const double dz = z[k] - ty[t * r + k];
            q2 = fma(dz, dz, q2);
          }
        }
        online_add(lwj - 0.5 * q2, m, l);
      }
    }
    if (act) {
      pm[(int64_t)blockIdx.x * cap + q] = m;
      pl[(int64_t)blockIdx.x * cap + q] = l;
    }
  }
}

__global__ void x3_rescue_final(const int64_t* __restrict__ rescue,
                                const unsigned int* __restrict__ nrescue, int64_t q0,
                                int64_t cap, int nslice, const double* __restrict__ pm,
                                const double* __restrict__ pl, double log_const,
                                double* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)*nrescue;
  if (q >= cap || q0 + q >= n) return;
  double mx = -INFINITY;
  for (int c = 0; c < nslice; ++c)
    if (pl[(int64_t)c * cap + q] > 0.0) mx = fmax(mx, pm[(int64_t)c * cap + q]);
  double t = 0.0;
  for (int c = 0; c < nslice; ++c) {
    const double l = pl[(int64_t)c * cap + q];
    if (l > 0.0) t += l * exp2(pm[(int64_t)c * cap + q] - mx);
  }
  out[rescue[q0 + q]] = t > 0.0 ? log_const + LN2 * (mx + log2(t)) : -INFINITY;
}

template <int SIDE>
void launch_pack(int r, dim3 grid, hipStream_t s, const double* P, const double* w,
                 int64_t n, int d, const double* mu, const double* U,
                 double log_w_shift, int K0pad, int KB, const Header* hdr,
                 _Float16* img, int64_t ntiles, int32_t* flags, double* Y,
                 double* lw, int64_t Np, const int64_t* hint, float* cand_o,
                 int koff, const double* shift_dev = nullptr,
                 const unsigned int* count_dev = nullptr) {
#define ABC_PACK_CASE(RC)                                                          \
  case RC:                                                                         \
    hipLaunchKernelGGL((pack_x3_kernel<SIDE, RC>), grid, dim3(128), 0, s, P, w, n, \
                       d, mu, U, r, log_w_shift, K0pad, KB, hdr, img, ntiles, flags, \
                       Y, lw, Np, hint, cand_o, koff, shift_dev, count_dev);       \
    break;
  switch (r) {
    ABC_PACK_CASE(1) ABC_PACK_CASE(2) ABC_PACK_CASE(3) ABC_PACK_CASE(4)
    ABC_PACK_CASE(5) ABC_PACK_CASE(6) ABC_PACK_CASE(7) ABC_PACK_CASE(8)
    ABC_PACK_CASE(9) ABC_PACK_CASE(10) ABC_PACK_CASE(12) ABC_PACK_CASE(16)
    default: ABC_PACK_CASE(0)
  }
#undef ABC_PACK_CASE
}

// rows of the rescued candidates (x [M x d] -> xs [n x d]) and their
// densities back (outs [n] -> out at the rescued positions)
// (the first min(*nres, cap) list entries: the nested pass's capacity)
__global__ void x3_gather_rescued(const int64_t* __restrict__ rescue,
                                  const unsigned int* __restrict__ nres, int64_t cap,
                                  const double* __restrict__ x, int d,
                                  double* __restrict__ xs) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)*nres < cap ? (int64_t)*nres : cap;
  if (e >= n * d) return;
  xs[e] = x[rescue[e / d] * d + e % d];
}
__global__ void x3_scatter_rescued(const int64_t* __restrict__ rescue,
                                   const unsigned int* __restrict__ nres, int64_t cap,
                                   const double* __restrict__ outs,
                                   double* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < (int64_t)*nres && q < cap) out[rescue[q]] = outs[q];
}

// candidate tiles (32 columns) per wave for KB MFMA instructions per tile
// pair, as dispatch_x3 instantiates them
// (register budget of the hinted pass at 2 waves per SIMD: 4 KB VGPRs per
// candidate tile, 8 KB for the two population buffers, 32 accumulators)
__host__ __device__ constexpr int x3_ct(int KB) {
  return KB <= 3 ? 8 : (KB <= 5 ? 6 : (KB == 6 ? 4 : (KB == 7 ? 3 : 2)));
}

struct PlanX3 {
  int K0pad, KB, KB0, CT, nchunk;
  int64_t MT, NT, MTpad, groups, tiles_per_chunk, Mpad;
};

// fine: the nested rescue pass (few candidates, launched for all M): more,
// shorter population chunks (up to 256, >= 16 tiles each) so its handful of
// candidate waves spread over the chip instead of one wave per 1/32 of the
// population.  Chunking still depends on N only.
PlanX3 make_plan_x3(int64_t M, int64_t N, int r, bool fine = false) {
  PlanX3 p;
  p.K0pad = x3_k0pad(r);
  p.KB = x3_kb(r);
  p.KB0 = x3_kb0(r);
  p.CT = x3_ct(p.KB);
  p.MT = ceil_div(M > 0 ? M : 1, TR);
  p.NT = ceil_div(N > 0 ? N : 1, TR);
  const int64_t waves = ceil_div(p.MT, p.CT);
  p.groups = ceil_div(waves, 4);
  p.MTpad = p.groups * 4 * p.CT;
  p.Mpad = p.MTpad * TR;
  // Population chunks depend on N only (8..32, a multiple of 8 for the
  // XCD map): a candidate's summation order -- and so its bits -- does not
  // depend on M or on its position, which keeps results identical for any
  // candidate sharding over ranks.  32 chunks fill the chip from M ~ 1e4.
  int64_t nc = fine ? ceil_div(ceil_div(p.NT, 16), 8) * 8 : ceil_div(ceil_div(p.NT, 128), 8) * 8;
  nc = nc < 8 ? 8 : (nc > (fine ? 256 : 32) ? (fine ? 256 : 32) : nc);
  p.nchunk = (int)nc;
  p.tiles_per_chunk = ceil_div(p.NT, p.nchunk);
  return p;
}

size_t plan_x3_ws(const PlanX3& p) {
  size_t off = 0;
  size_only<_Float16>(off, (size_t)p.MTpad * p.KB * 64 * 8);  // candidate image
  size_only<int32_t>(off, (size_t)p.Mpad);                     // candidate flags
  size_only<float>(off, (size_t)p.Mpad);                       // hinted offsets
  size_only<double>(off, (size_t)p.nchunk * p.Mpad);           // partial offsets
  size_only<double>(off, (size_t)p.nchunk * p.Mpad);           // partial sums
  size_only<int64_t>(off, (size_t)p.Mpad);                     // rescue list
  size_only<unsigned int>(off, 64);                            // rescue count
  return off + 256;
}

template <int KB, int CT>
void launch_x3(const PlanX3& p, const half8* A, const half8* B, int koff,
               double* po, double* pl, bool pass1, const unsigned int* count_dev,
               hipStream_t s) {
  static_assert(CT == x3_ct(KB), "the plan's tiles per wave must match the instantiation");
  // a device-sized launch strides over its groups with at most 16 in the grid
  const int64_t gg = count_dev && p.groups > 16 ? 16 : p.groups;
  const int64_t blocks = gg * p.nchunk;
  if (pass1)
    hipLaunchKernelGGL((mvn_x3_kernel<KB, CT, true>), dim3((unsigned)blocks),
                       dim3(256), 0, s, A, B, p.MT, p.NT, p.nchunk,
                       p.tiles_per_chunk, p.groups, koff, p.KB0, po, pl, p.Mpad, count_dev);
  else
    hipLaunchKernelGGL((mvn_x3_kernel<KB, CT, false>), dim3((unsigned)blocks),
                       dim3(256), 0, s, A, B, p.MT, p.NT, p.nchunk,
                       p.tiles_per_chunk, p.groups, koff, p.KB0, po, pl, p.Mpad, count_dev);
}

int dispatch_x3(const PlanX3& p, const half8* A, const half8* B, int koff,
                double* po, double* pl, bool pass1, const unsigned int* count_dev,
                hipStream_t s) {
  switch (p.KB) {
#define ABC_X3_CASE(K) \
  case K: launch_x3<K, x3_ct(K)>(p, A, B, koff, po, pl, pass1, count_dev, s); break;
    ABC_X3_CASE(2) ABC_X3_CASE(3) ABC_X3_CASE(4) ABC_X3_CASE(5) ABC_X3_CASE(6)
    ABC_X3_CASE(7) ABC_X3_CASE(8) ABC_X3_CASE(9) ABC_X3_CASE(10) ABC_X3_CASE(11)
#undef ABC_X3_CASE
    default:
      return set_error(ABC_ERR_UNSUPPORTED, "mvn x3: KB=%d unsupported", p.KB);
  }
  return ABC_OK;
}
static_assert(x3_kb(MAX_R) <= 11 && x3_kb(1) >= 2, "dispatch_x3 covers every rank");

}  // namespace

// ---- internal entry points used by abc_mvn.hip ------------------------------
// image = header | fragments [NT][KB][64][8] f16 | Y [N x r] f64 | lw [N] f64
size_t x3_frag_bytes(int64_t N, int r) {
  const int KB = x3_kb(r);
  const int64_t NT = ceil_div(N > 0 ? N : 1, TR) + X3_PAD;
  return align_up((size_t)NT * KB * 64 * 8 * sizeof(_Float16), 256);
}
double* x3_Y(const void* packed, int64_t N, int r) {
  return (double*)((char*)packed + HDR + x3_frag_bytes(N, r));
}
double* x3_lw(const void* packed, int64_t N, int r) {
  return x3_Y(packed, N, r) + align_up((size_t)(N > 0 ? N : 1) * r, 32);
}
size_t x3_packed_bytes(int64_t N, int r) {
  return HDR + x3_frag_bytes(N, r) +
         sizeof(double) * (align_up((size_t)(N > 0 ? N : 1) * r, 32) + (N > 0 ? N : 1));
}

int x3_max_rank() { return MAX_R; }

// kernel 1 = mvn_x3_kernel<KB, CT, *> on v_mfma_f32_32x32x16_f16: K slots
// per pair (16 KB) and 32-column candidate tiles per wave
extern "C" int abc_mvn_x3_layout(int r, int* kslots, int* tiles_per_wave) {
  const int KB = x3_kb(r);
  if (kslots) *kslots = 16 * KB;
  if (tiles_per_wave) *tiles_per_wave = x3_ct(KB);
  return 1;
}

int x3_pack_population(const double* X, const double* w, int64_t N, int d,
                       const double* mu, const double* U, int r,
                       double log_w_shift, const double* shift_dev, void* packed,
                       double* range, hipStream_t s) {
  if (r > MAX_R)
    return set_error(ABC_ERR_UNSUPPORTED, "mvn x3: rank %d > %d", r, MAX_R);
  const int64_t NT = ceil_div(N > 0 ? N : 1, TR);
  Header* hdr = (Header*)packed;
  ABC_HIP(hipMemsetAsync(hdr, 0, HDR, s));
  if (N > 0) {
    const int64_t nb = ceil_div(N, 256);
    hipLaunchKernelGGL(pop_range_kernel,
                       dim3((unsigned)(nb < POP_RANGE_BLOCKS ? nb : POP_RANGE_BLOCKS)), dim3(256),
                       0, s, X, w, N, d, mu, U, r, hdr);
    ABC_LAUNCHED();
  }
  hipLaunchKernelGGL(x3_setup_kernel, dim3(1), dim3(1), 0, s, hdr, r, range);
  ABC_LAUNCHED();
  launch_pack<0>(r, dim3((unsigned)ceil_div(NT * TR, 128)), s, X, w, N, d, mu, U,
                 log_w_shift, x3_k0pad(r), x3_kb(r), (const Header*)hdr,
                 (_Float16*)((char*)packed + HDR), NT, (int32_t*)nullptr,
                 x3_Y(packed, N, r), x3_lw(packed, N, r), N, (const int64_t*)nullptr,
                 (float*)nullptr, 0, shift_dev);
  ABC_LAUNCHED();
  return ABC_OK;
}

// Rows the nested exact pass of a hinted call takes at most (0.04% of the
// candidates are rescued at c3: ~400 of 1e6); list entries past it take the
// fp64 rescue kernel instead.  The nested 'fine' plan keeps up to 256
// population chunks of partials per row, so sizing it for all M reserved
// ~4 GB at M = N = 1e6 for a handful of rows; at this cap it is ~70 MB.
constexpr int64_t X3_NEST_CAP = 16384;
inline int64_t x3_nest_rows(int64_t M) { return M < X3_NEST_CAP ? M : X3_NEST_CAP; }

// the main launch's plan, then (hinted calls) room for the nested exact
// pass over up to X3_NEST_CAP rescued candidates: their rows, results and
// its own plan
size_t x3_logpdf_workspace(int64_t M, int64_t N, int r) {
  const size_t main = plan_x3_ws(make_plan_x3(M, N, r));
  const int64_t m1 = x3_nest_rows(M > 0 ? M : 1);
  size_t nested = 0;
  size_only<double>(nested, (size_t)m1 * 64);           // rows (d <= 64)
  size_only<double>(nested, (size_t)m1);                // results
  size_only<char>(nested, plan_x3_ws(make_plan_x3(m1, N, r, true)));  // the nested plan
  return main + nested + 256;
}

// fp64 rescue of the list entries [q_begin, *nres) (count on the device):
// launch pairs over slot ranges of the main plan's partial arrays (free once
// combined); pairs past the count exit at once
static void x3_rescue_fp64(const PlanX3& p, int64_t q_begin, int64_t M, const double* x, int d,
                    const void* packed, int64_t N, const double* mu, const double* U, int r,
                    double log_const, const int64_t* rescue, const unsigned int* nres,
                    double* po, double* pl, double* out, hipStream_t s) {
  const int ns = rescue_slices(N);
  const int64_t cap = (int64_t)p.nchunk * p.Mpad / ns;
  for (int64_t q0 = q_begin; q0 < M; q0 += cap) {
    hipLaunchKernelGGL(x3_rescue_kernel, dim3((unsigned)ns, (unsigned)RS_GY), dim3(64), 0, s,
                       rescue, nres, q0, cap, x, d, mu, U, r,
                       (const double*)x3_Y(packed, N, r),
                       (const double*)x3_lw(packed, N, r), N, po, pl);
    hipLaunchKernelGGL(x3_rescue_final, dim3((unsigned)ceil_div(cap < M ? cap : M, 256)),
                       dim3(256), 0, s, rescue, nres, q0, cap, ns, po, pl, log_const, out);
  }
}

// count_dev (nullable): a device-sized launch -- only the first *count_dev
// of the M rows of x are candidates (the nested rescue pass below)
int x3_logpdf(const double* x, int64_t M, int d, const void* packed,
              const double* X, const double* w, int64_t N, const double* mu,
              const double* U, int r, double log_const, double log_norm,
              double* out, const int64_t* hint, void* ws, size_t ws_bytes,
              hipStream_t s, int prof_channel, const unsigned int* count_dev) {
  if (r > MAX_R)
    return set_error(ABC_ERR_UNSUPPORTED, "mvn x3: rank %d > %d", r, MAX_R);
  PlanX3 p = make_plan_x3(M, N, r, count_dev != nullptr);
  if (ws_bytes < plan_x3_ws(p))
    return set_error(ABC_ERR_WORKSPACE, "mvn x3: workspace %zu < %zu", ws_bytes,
                     plan_x3_ws(p));
  Carver cv(ws, ws_bytes);
  _Float16* Bimg = cv.take<_Float16>((size_t)p.MTpad * p.KB * 64 * 8);
  int32_t* cflags = cv.take<int32_t>((size_t)p.Mpad);
  float* cand_o = cv.take<float>((size_t)p.Mpad);
  double* po = cv.take<double>((size_t)p.nchunk * p.Mpad);
  double* pl = cv.take<double>((size_t)p.nchunk * p.Mpad);
  int64_t* rescue = cv.take<int64_t>((size_t)p.Mpad);
  unsigned int* nres = cv.take<unsigned int>(64);
  if (!cv.ok) return set_error(ABC_ERR_WORKSPACE, "mvn x3: workspace carve");
  const Header* hdr = (const Header*)packed;
  const half8* Aimg = (const half8*)((const char*)packed + HDR);
  ABC_HIP(hipMemsetAsync(nres, 0, sizeof(unsigned int), s));
  launch_pack<1>(r, dim3((unsigned)ceil_div(p.MTpad * TR, 128)), s, x,
                 (const double*)nullptr, M, d, mu, U, log_norm - log_const, p.K0pad,
                 p.KB, hdr, Bimg, p.MTpad, cflags, x3_Y(packed, N, r),
                 x3_lw(packed, N, r), N, hint, hint ? cand_o : (float*)nullptr, r + 6,
                 (const double*)nullptr, count_dev);
  ABC_LAUNCHED();
  profile_start(s, prof_channel);
  int rc = dispatch_x3(p, Aimg, (const half8*)Bimg, r + 6, po, pl, hint == nullptr,
                       count_dev, s);
  profile_stop(s, prof_channel);
  if (rc) return rc;
  ABC_LAUNCHED();
  if (count_dev && !hint)
    hipLaunchKernelGGL(x3_combine_rows_kernel, dim3((unsigned)ceil_div(M, 4)), dim3(256),
                       0, s, po, pl, p.nchunk, M, p.Mpad, log_const, cflags, out, rescue,
                       nres, count_dev);
  else
    hipLaunchKernelGGL(x3_combine_kernel, dim3((unsigned)ceil_div(M, 256)), dim3(256),
                       0, s, po, pl, p.nchunk, M, p.Mpad, log_const, cflags,
                       hint ? (const float*)cand_o : (const float*)nullptr, out,
                       rescue, nres, count_dev);
  ABC_LAUNCHED();
  if (hint) {
    // Hinted candidates whose ancestor offset was far below their true
    // maximum (or outside the limb range / underflowing) are re-run through
    // the unhinted pass -- exact max pre-pass, still MFMA -- on the gathered
    // rescue list.  The list's length stays on the device: the nested pass
    // is launched for all M and its waves past the count leave at once, so
    // the call never waits for the GPU.  A candidate's result is independent
    // of M, of its slot in the list and of the list's length (chunking by N
    // only), so sharded runs keep identical bits.  The nested pass takes the
    // first X3_NEST_CAP entries; any beyond (more than 16384 rescued rows in
    // one call, never seen on the configs) take the fp64 rescue, equally
    // within the parity bar but not bitwise the nested pass's values.
    const int64_t Mn = x3_nest_rows(M);
    Carver sub(cv.rest(), cv.rest_bytes());
    double* xs = sub.take<double>((size_t)Mn * d);
    double* outs = sub.take<double>((size_t)Mn);
    const size_t need = plan_x3_ws(make_plan_x3(Mn, N, r, true));
    void* ws2 = sub.take<char>(need);
    if (!sub.ok) return set_error(ABC_ERR_WORKSPACE, "mvn x3: nested rescue workspace");
    hipLaunchKernelGGL(x3_gather_rescued, dim3((unsigned)ceil_div(Mn * d, 256)),
                       dim3(256), 0, s, rescue, nres, Mn, x, d, xs);
    ABC_LAUNCHED();
    const int rc2 = x3_logpdf(xs, Mn, d, packed, X, w, N, mu, U, r, log_const, log_norm,
                              outs, nullptr, ws2, need, s, ABC_PROF_RESCUE, nres);
    if (rc2) return rc2;
    hipLaunchKernelGGL(x3_scatter_rescued, dim3((unsigned)ceil_div(Mn, 256)), dim3(256), 0,
                       s, rescue, nres, Mn, outs, out);
    ABC_LAUNCHED();
    if (M > Mn) {
      x3_rescue_fp64(p, Mn, M, x, d, packed, N, mu, U, r, log_const, rescue, nres, po, pl,
                     out, s);
      ABC_LAUNCHED();
    }
    return ABC_OK;
  }
  // fp64 rescue of the listed candidates
  x3_rescue_fp64(p, 0, M, x, d, packed, N, mu, U, r, log_const, rescue, nres, po, pl, out, s);
  ABC_LAUNCHED();
  return ABC_OK;
}

}  // namespace abc
