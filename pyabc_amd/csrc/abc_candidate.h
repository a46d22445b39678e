// Per-candidate device code shared by the stage kernels (abc_sampler.hip) and
// the fused candidate round (abc_fused.hip).
//
// Reference per-candidate closure (pyabc/smc.py:588-724):
//   _generate_valid_proposal (smc.py:610-662): theta = Transition.rvs()
//     (multivariatenormal.py:85-97 / local_transition.py:141-145), re-drawn
//     while the prior density is 0; t == 0: theta = prior.rvs()
//   Model.accept (model.py:163-218) -> summary stats -> PNormDistance
//     (distance/distance.py:79-105) -> UniformAcceptor d <= eps
//     (acceptor/acceptor.py:235-244)
// Every draw is a pure function of (seed, generation, global candidate index,
// slot), so the stage kernels, the fused round and its regeneration of the
// accepted rows compute the same candidate bit for bit: the functions below
// are the single definition all of them inline, and floating-point
// contraction is off (explicit fma() where a fused multiply-add is meant), so
// the compiler cannot fuse differently in different kernels.
#pragma once
#include "abc_common.h"

#pragma clang fp contract(off)

namespace abc {

constexpr double LOG_SQRT_2PI = 0.91893853320467274178;
constexpr uint32_t SLOTS_PER_ATTEMPT = 65536;
constexpr uint32_t SLOT_ANCESTOR = 0;
constexpr uint32_t SLOT_PERTURB = 1;     // 4 normals per slot (after the first two)
constexpr uint32_t SLOT_PRIOR = 32;      // + 512 k + iteration
constexpr uint32_t SLOT_SIM = 0x40000000u;

// normals q .. q+3 of one slot (Box-Muller pairs; only the first `need`
// (1..4) are produced -- the pair the caller does not use is skipped)
__device__ __forceinline__ void normals4(uint64_t g, uint32_t slot, uint32_t gen,
                                         uint64_t seed, double n[4], int need = 4,
                                         const float* tab = BM_TAB) {
  u32x4 r = philox(g, slot, gen, seed);
  box_muller(r.x, r.y, n[0], n[1], tab);
  if (need > 2) box_muller(r.z, r.w, n[2], n[3], tab);
}

// Words of perturbation pair p (normals 2 p, 2 p + 1) of one attempt: pair 0
// takes the ancestor draw's unused second pair (its uniform53 reads x, y);
// pair p >= 1 half (p - 1) & 1 of slot SLOT_PERTURB + (p - 1) / 2, whose
// Philox call the caller makes when (p - 1) is even (into r).  A d = 9 or 10
// proposal then needs 2 perturbation calls instead of 3.
__device__ __forceinline__ void perturb_words(int p, const u32x4& anc, u32x4& r, uint64_t g,
                                              uint32_t s0, uint32_t gen, uint64_t seed,
                                              uint32_t& wa, uint32_t& wb) {
  if (p == 0) {
    wa = anc.z;
    wb = anc.w;
    return;
  }
  const int p1 = p - 1;
  if ((p1 & 1) == 0) r = philox(g, s0 + SLOT_PERTURB + (uint32_t)(p1 >> 1), gen, seed);
  wa = (p1 & 1) ? r.z : r.x;
  wb = (p1 & 1) ? r.w : r.y;
}

// ---- priors (scipy.stats pdf conventions, closed support [a, b]) ----------
__device__ __noinline__ double prior_logpdf1(int kind, const double* p, double x) {
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
    case ABC_PRIOR_HOST:  // lo, hi, c: factor 1 on the support (host adds scipy's)
      return (x >= p[0] && x <= p[1]) ? 0.0 : -INFINITY;
  }
  return NAN;
}

// Prior density > 0 at x (the re-draw test of smc.py:654-656), decided on
// the support alone: exactly the x for which prior_logpdf1 is not -inf / NaN
// (up to overflow of a finite log density), without its transcendentals.
__device__ __forceinline__ bool prior_in_support1(int kind, const double* p, double x) {
  switch (kind) {
    case ABC_PRIOR_FLAT:
      return true;
    case ABC_PRIOR_NORM: {
      double y = (x - p[0]) / p[1];
      return y * y < INFINITY;  // false for NaN
    }
    case ABC_PRIOR_UNIFORM: {
      double y = (x - p[0]) / p[1];
      return y >= 0.0 && y <= 1.0;
    }
    case ABC_PRIOR_EXPON: {
      double y = (x - p[0]) / p[1];
      return y >= 0.0 && y < INFINITY;
    }
    case ABC_PRIOR_LAPLACE: {
      double y = (x - p[0]) / p[1];
      return fabs(y) < INFINITY;
    }
    case ABC_PRIOR_LOGNORM: {
      double y = (x - p[1]) / p[2];
      return y > 0.0 && y < INFINITY;
    }
    case ABC_PRIOR_GAMMA: {
      double y = (x - p[1]) / p[2];
      return (y > 0.0 && y < INFINITY) || (y == 0.0 && p[0] <= 1.0);
    }
    case ABC_PRIOR_BETA: {
      double y = (x - p[2]) / p[3];
      if (!(y >= 0.0 && y <= 1.0)) return false;
      if (y == 0.0 && p[0] > 1.0) return false;
      if (y == 1.0 && p[1] > 1.0) return false;
      return true;
    }
    case ABC_PRIOR_HOST:
      return x >= p[0] && x <= p[1];
  }
  return false;
}

// Marsaglia-Tsang gamma(a, 1) draw; stream = (g, base + iteration)
__device__ inline double gamma_draw(double a, uint64_t g, uint32_t base, uint32_t gen,
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

__device__ __noinline__ double prior_draw1(int kind, const double* p, uint64_t g,
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
    case ABC_PRIOR_HOST:  // a support point; the host writes ppf(u) over it
      return p[2];
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

// The guide-table search split in two: the bracket loads are issued first
// (ancestor_bracket) and the search finished later (ancestor_finish), so
// independent work can run while they are in flight.  Same result as
// ancestor_search.
struct AncestorBracket { int64_t lo, hi; };
__device__ __forceinline__ AncestorBracket ancestor_bracket(const int32_t* __restrict__ guide,
                                                            int64_t N, double total,
                                                            double target) {
  if (guide == nullptr) return {0, N};
  const double step = total / (double)N;
  int64_t k = (int64_t)floor(target / step) - 1;  // t_k < target (one-bin margin)
  k = k < 0 ? 0 : (k > N - 1 ? N - 1 : k);
  const int64_t k3 = k + 3 < N ? k + 3 : N - 1;
  // both loads unconditional (no branch, so no wait at the join)
  const int64_t lo = guide[k];
  const int64_t g3 = guide[k3];
  return {lo, k + 3 < N ? g3 + 1 : N};  // t_{k+3} > target
}
__device__ __forceinline__ int64_t ancestor_finish(const double* __restrict__ cdf, int64_t N,
                                                   double target, AncestorBracket b) {
  int64_t lo = b.lo, hi = b.hi;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cdf[mid] > target) hi = mid; else lo = mid + 1;
  }
  return lo < N ? lo : N - 1;
}

// search of the ancestor table's bracket [lo, hi] (hi inclusive; hi == N:
// past the last row), the scan read from the records (rec[i rs + d] = cdf_i)
__device__ __forceinline__ int64_t table_finish(const double* __restrict__ rec, int rs, int d,
                                                int64_t N, double target, AncestorBracket b) {
  int64_t lo = b.lo, hi = b.hi;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rec[mid * rs + d] > target) hi = mid; else lo = mid + 1;
  }
  return lo < N ? lo : N - 1;
}

// ---- exact support box ------------------------------------------------------
// The support {x : prior_in_support1(kind, p, x)} of every kind is an
// interval of doubles (y = (x - loc) / scale is monotone in x, and so is each
// test on y), so it equals [lo, hi] for two doubles found by bisection over
// the order-preserving integer image of the doubles, evaluating the very
// predicate above.  The per-candidate re-draw test is then two compares.
__device__ __forceinline__ uint64_t dkey(double x) {   // order-preserving
  const uint64_t u = (uint64_t)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}
__device__ __forceinline__ double dval(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & ~(1ull << 63)) : ~k;
  return __longlong_as_double((long long)u);
}
// The bisection runs with the 64 lanes of a wave probing together: each
// step evaluates the predicate at 64 evenly spaced keys of the open bracket
// and keeps the sub-bracket where it turns (the predicate is monotone in
// the key on each side of an interior point c), so a 64-bit bracket closes
// in ~11 steps instead of ~63 dependent ones.  Every lane of the wave must
// call it (uniform arguments); lane 0 writes lo_hi = [lowest, highest
// member] (inf, -inf for an empty support).
__device__ __forceinline__ void support_bounds_wave(int kind, const double* pg, double* lo_hi) {
  const int lane = threadIdx.x & 63;
  double p[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) p[i] = pg[i];
  double c;
  switch (kind) {
    case ABC_PRIOR_UNIFORM: c = p[0] + 0.5 * p[1]; break;
    case ABC_PRIOR_EXPON: c = p[0] + p[1]; break;
    case ABC_PRIOR_LOGNORM: case ABC_PRIOR_GAMMA: c = p[1] + p[2]; break;
    case ABC_PRIOR_BETA: c = p[2] + 0.5 * p[3]; break;
    case ABC_PRIOR_NORM: case ABC_PRIOR_LAPLACE: c = p[0]; break;
    case ABC_PRIOR_HOST: c = p[2]; break;
    default: c = 0.0;
  }
  if (!prior_in_support1(kind, p, c)) {
    if (lane == 0) { lo_hi[0] = INFINITY; lo_hi[1] = -INFINITY; }
    return;
  }
  // first key in (lo, hi] where pred(key) == up (pred(lo) != up, pred(hi) == up)
  auto turn = [&](uint64_t lo, uint64_t hi, bool up) {
    while (hi - lo > 1) {
      const uint64_t span = hi - lo;            // > 1
      const uint64_t step = span / 65 > 0 ? span / 65 : 1;
      const uint64_t m = lo + step * (uint64_t)(lane + 1);
      const bool inside = m < hi;
      const bool pr = inside ? (prior_in_support1(kind, p, dval(m)) == up) : true;
      const unsigned long long bal = __ballot(pr);   // lanes past hi count as "turned"
      if (bal == 0ull) {                             // the turn lies past the last probe
        lo = lo + step * 64ull;
        continue;
      }
      const int f = __ffsll((long long)bal) - 1;     // first turned probe (or a pad)
      const uint64_t mf = lo + step * (uint64_t)(f + 1);
      const uint64_t new_hi = mf < hi ? mf : hi;
      const uint64_t new_lo = f == 0 ? lo : lo + step * (uint64_t)f;
      lo = new_lo;
      hi = new_hi;
    }
    return hi;
  };
  const uint64_t kc = dkey(c);
  uint64_t lo_key;
  if (prior_in_support1(kind, p, -INFINITY)) lo_key = dkey(-INFINITY);
  else lo_key = turn(dkey(-INFINITY), kc, true);       // lowest member
  uint64_t hi_key;
  if (prior_in_support1(kind, p, INFINITY)) hi_key = dkey(INFINITY);
  else hi_key = turn(kc, dkey(INFINITY), false) - 1;   // one below the first non-member
  if (lane == 0) { lo_hi[0] = dval(lo_key); lo_hi[1] = dval(hi_key); }
}

// ---- one proposal ----------------------------------------------------------
struct ProposalArgs {
  const double* X;       // population [N x d] (nullptr: draw from the prior)
  const double* cdf;      // inclusive scan of w [N]
  const int32_t* guide;   // cdf guide table [N] or nullptr
  int64_t N;
  const double* L;        // [d x d] row-major, or [N x d x d] per particle
  const int32_t* kind;    // prior kinds [d]
  const double* params;   // prior params [4 d]
  int d;
  int max_attempts;
  uint64_t seed;
  uint32_t gen;
  // ancestor table (abc_ancestor_table; rec == nullptr: X / cdf / guide)
  const double* rec = nullptr;     // records [N x rs]: X_j, cdf_j, padding
  const int32_t* bguide = nullptr; // exact-bin guide [G + 2]
  int rs = 0;
  int64_t G = 0;
  const double* xmax = nullptr;    // max |X_jk| over the table (its header)
};

// ---- ancestor table -----------------------------------------------------------
// The ancestor draw reads, per candidate, a guide entry, the weight scan near
// the answer and the answer's row.  At c3 sizes (1e6 rows) those are random
// accesses into the Infinity Cache, and the chip serves ~5.5e10 of them per
// second whatever their size (8 B .. 128 B; a 2-MB table that stays in L2
// serves 2.5e11: tools/probes/gather_cost.hip, profiles/r02_gather_probe.txt).
// The table keeps
//   * each row in a 128-byte-aligned record with its scan value (rs = 16
//     doubles for d <= 15): the answer's row and the scan values the search
//     probes are one access;
//   * a guide over G = 4 N bins of the scan, bin(x) = min(floor(x G /
//     total), G), guide[k] = first i with bin(cdf_i) >= k.  bin is monotone
//     and both sides evaluate it identically, so for target t with kt =
//     bin(t), i* = first i with cdf_i > t lies in [guide[kt], guide[kt + 1]]
//     (i < guide[kt]: bin(cdf_i) < kt, so cdf_i < t; bin(cdf_{guide[kt+1]}) >
//     kt, so cdf > t): np.searchsorted's answer, with no probe when the two
//     entries agree (most bins at G = 4 N) and otherwise probes that read the
//     records holding the candidate rows themselves.  Two accesses per draw.
constexpr int ANC_HDR = 256;  // table header bytes
__host__ __device__ inline int anc_rs(int d) { return (d + 1 + 15) / 16 * 16; }
__host__ __device__ inline int64_t anc_bins(int64_t N) {
  const int64_t g = 4 * N;
  return g < (int64_t)0x7FFFFFF0 ? g : (int64_t)0x7FFFFFF0;
}
__device__ __forceinline__ int64_t anc_bin(double x, double inv_step, int64_t G) {
  const double b = x * inv_step;  // x >= 0
  return b >= (double)G ? G : (int64_t)b;
}

// MODE: PROP_MVN (one shared L), PROP_LOCAL (per-particle L), PROP_PRIOR
// (X == nullptr: draw from the prior).  Separate instantiations keep the
// prior draw's calls out of the transition kernels' register allocation.
constexpr int PROP_MVN = 0, PROP_LOCAL = 1, PROP_PRIOR = 2;

// ---- LinearGaussianModel + PNormDistance -----------------------------------
struct SimDistArgs {
  const int32_t* src;     // x_k = a_k theta[src_k] + sigma_k e_k
  const double* a;
  const double* sigma;
  const double* x0;       // observed sum stats [S]
  const double* wf;       // PNorm weights * factors [S]
  double p;
  int S;
};

// Per-block constants in LDS, read at wave-uniform addresses (broadcast).
// Kept out of global memory on purpose: the kernels also store to global
// memory, so the compiler cannot prove these arrays unclobbered and would
// fetch every element with a per-lane vector load (~120 per candidate).
constexpr int SIM_SMAX = 256;     // fused path: S <= SIM_SMAX
constexpr int LT_DMAX = 16;       // shared L staged for d <= 16
struct BlockConsts {
  float bmt[BM_TAB_SIZE];         // Box-Muller tables (BM_TAB)
  double LT[LT_DMAX * LT_DMAX];   // shared L, transposed: LT[q d + k] = L[k d + q]
  double box[2 * 64];             // prior support [lo, hi] per dimension
  double2 as[SIM_SMAX];           // (a_k, sigma_k)
  double2 wx[SIM_SMAX];           // (wf_k, x0_k)
  int32_t src[SIM_SMAX];
  double total;                   // cdf[N - 1]
  double inv_step;                // G / total (ancestor table)
  int lazy;                       // early reject from theta_0..LAZY_KT-1 (lazy_filter_ok)
};

// Fill C (every thread of the block calls it; synchronises).  BOX_FROM_SRC:
// copy the precomputed support box box_src, else bisect here
// (support_bounds_wave; the block size is a multiple of 64).
template <int D, int MODE, bool BOX_FROM_SRC = false>
__device__ __forceinline__ void stage_block_consts(BlockConsts& C, const ProposalArgs& A,
                                                   const SimDistArgs* M,
                                                   const double* box_src) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int d = D > 0 ? D : A.d;
  for (int k = t; k < BM_TAB_SIZE; k += nt) C.bmt[k] = BM_TAB[k];
  if (MODE == PROP_MVN && D > 0 && D <= LT_DMAX)
    for (int e = t; e < d * d; e += nt) C.LT[(e % d) * d + e / d] = A.L[e];
  if (BOX_FROM_SRC) {
    for (int k = t; k < 2 * d; k += nt) C.box[k] = box_src[k];
  } else {
    // one wave per dimension (support_bounds_wave)
    for (int k = t >> 6; k < d; k += nt >> 6)
      support_bounds_wave(A.kind[k], A.params + 4 * k, C.box + 2 * k);
  }
  if (M)
    for (int k = t; k < M->S && k < SIM_SMAX; k += nt) {
      C.as[k] = make_double2(M->a[k], M->sigma[k]);
      C.wx[k] = make_double2(M->wf[k], M->x0[k]);
      C.src[k] = M->src[k];
    }
  if (t == 0) {
    const double total = (MODE != PROP_PRIOR) ? A.cdf[A.N - 1] : 0.0;
    C.total = total;
    C.inv_step = (MODE != PROP_PRIOR && A.rec) ? (double)A.G / total : 0.0;
  }
  __syncthreads();
}

// Candidate g: ancestor j ~ Cat(w), theta = X_j + L_j n (or a prior draw when
// X == nullptr), re-drawn while theta is outside the prior support C.box.
// th holds D (D > 0) or d <= 64 values.  The perturbation is accumulated one
// Box-Muller pair at a time in q order, theta_k = fma(L_kq, n_q, theta_k)
// starting from X_jk (one code copy of the transform).  Returns the attempts
// used, max_attempts + 1 when every attempt fell outside the support (theta
// then holds the last one).
template <int D, int MODE, bool TABLE = false>
__device__ __forceinline__ int propose_one(const ProposalArgs& A, const BlockConsts& C,
                                           uint64_t g, double* th, int64_t& j) {
  constexpr bool LT_LDS = MODE == PROP_MVN && D > 0 && D <= LT_DMAX;
  const int d = D > 0 ? D : A.d;
  j = -1;
  const double total = C.total;
  for (int att = 0; att < A.max_attempts; ++att) {
    const uint32_t s0 = (uint32_t)att * SLOTS_PER_ATTEMPT;
    // an opaque zero offset on the LDS constants: without it the compiler
    // hoists the loop-invariant L / box reads out of the caller's candidate
    // loop into ~100 registers and halves the occupancy
    int oz = 0;
    asm volatile("" : "+s"(oz));
    const double* LT = C.LT + oz;
    const double* box = C.box + oz;
    if (MODE == PROP_PRIOR) {
#pragma unroll
      for (int k = 0; k < (D > 0 ? D : d); ++k)
        th[k] = prior_draw1(A.kind[k], A.params + 4 * k, g,
                            s0 + SLOT_PRIOR + 512u * k, A.gen, A.seed);
    } else {
      // the ancestor's guide bracket is loaded first and the perturbation
      // L n (independent of j) is computed while those loads are in flight;
      // the search and the X_j row come after: theta_k = X_jk + (L n)_k
      const u32x4 ra = philox(g, s0 + SLOT_ANCESTOR, A.gen, A.seed);
      u32x4 r = ra;
      const double target = uniform53(ra.x, ra.y) * total;
      AncestorBracket br;
      if (TABLE) {
        const int64_t kt = anc_bin(target, C.inv_step, A.G);
        br = {A.bguide[kt], A.bguide[kt + 1]};  // answer in [lo, hi]
      } else {
        br = ancestor_bracket(A.guide, A.N, total, target);
      }
#pragma unroll
      for (int k = 0; k < (D > 0 ? D : d); ++k) th[k] = 0.0;
      const double* Lj = A.L;
      if (MODE == PROP_LOCAL) {
        // per-particle factor: needs j first
        j = TABLE ? table_finish(A.rec, A.rs, d, A.N, target, br)
                  : ancestor_finish(A.cdf, A.N, target, br);
        Lj = A.L + j * d * d;
      }
      // L is lower triangular (a Cholesky factor; the ABI contract), so
      // column q only reaches rows k >= q: with D known the pair loop is
      // unrolled and the upper triangle's multiply-adds vanish
      auto pair = [&](int q) {
        uint32_t wa, wb;
        perturb_words(q >> 1, ra, r, g, s0, A.gen, A.seed, wa, wb);
        double n0, n1;
        box_muller(wa, wb, n0, n1, C.bmt);
        const bool two = q + 1 < d;
#pragma unroll
        for (int k = 0; k < (D > 0 ? D : d); ++k) {
          if (k >= q) {
            const double l0 = LT_LDS ? LT[q * d + k] : Lj[k * d + q];
            th[k] = fma(l0, n0, th[k]);
          }
          if (two && k >= q + 1) {
            const double l1 = LT_LDS ? LT[(q + 1) * d + k] : Lj[k * d + q + 1];
            th[k] = fma(l1, n1, th[k]);
          }
        }
      };
#pragma unroll 1
      for (int q = 0; q < d; q += 2) pair(q);
      if (MODE != PROP_LOCAL)
        j = TABLE ? table_finish(A.rec, A.rs, d, A.N, target, br)
                  : ancestor_finish(A.cdf, A.N, target, br);
      const double* Xj = TABLE ? A.rec + j * A.rs : A.X + j * d;
#pragma unroll
      for (int k = 0; k < (D > 0 ? D : d); ++k) th[k] = Xj[k] + th[k];
    }
    bool ok = true;  // branch-free (&& would branch per comparison)
#pragma unroll
    for (int k = 0; k < (D > 0 ? D : d); ++k)
      ok = ok & (box[2 * k] <= th[k]) & (th[k] <= box[2 * k + 1]);
    if (ok) return att + 1;  // prior density > 0 (smc.py:654-656)
  }
  return A.max_attempts + 1;
}

// ---- the lazy early-reject head ---------------------------------------------
// With a lower-triangular L, theta_k depends on normals 0..k only, so the
// first LAZY_KT coordinates of attempt 0 need the ancestor draw's second
// pair, one perturbation Philox call and two Box-Muller pairs instead of
// all d.  lazy_head_group (below)
// evaluates exactly those coordinates with propose_one's operations in
// propose_one's order (same streams, same fma chain, same X_j + (L n)_k), so
// they are the bits propose_one produces whenever attempt 0 is the accepted
// proposal.
constexpr int LAZY_KT = 4;

// Attempt 0 is the accepted proposal for EVERY candidate whose first LAZY_KT
// coordinates lie in the support, when the support box of every coordinate
// k >= LAZY_KT contains the whole range theta_k can take:
//   |theta_k| <= max_jk |X_jk| + 7.6 sum_q |L_kq|
// (every Box-Muller normal has |n| <= sqrt(2 * 41 ln 2) < 7.54, the 41-bit
// u1 of box_muller; a relative margin covers the roundings).  Also the early-reject statistics 0..3 must
// read theta_src with src < LAZY_KT.  Decided per block from its LDS
// constants (thread 0; the caller synchronises before C.lazy is read).
template <int D, int MODE>
__device__ __forceinline__ bool lazy_filter_ok(const BlockConsts& C, const ProposalArgs& A,
                                               const SimDistArgs& M) {
  if constexpr (MODE != PROP_MVN || D <= LAZY_KT || D > LT_DMAX) {
    return false;
  } else {
    if (A.xmax == nullptr || M.S <= 4) return false;
    bool ok = true;
    for (int k = 0; k < 4; ++k) ok = ok && C.src[k] >= 0 && C.src[k] < LAZY_KT;
    const double xm = *A.xmax;
    for (int k = LAZY_KT; k < D; ++k) {
      double ls = 0.0;
      for (int q = 0; q <= k; ++q) ls += fabs(C.LT[q * D + k]);
      const double b = (xm + 7.6 * ls) * 1.000001 + 1e-300;
      ok = ok && (C.box[2 * k] <= -b) && (b <= C.box[2 * k + 1]);  // NaN: false
    }
    return ok;
  }
}

// (contraction is off for the whole header, line 20; restated in each of
// these three so that no include order or later edit can let the compiler
// turn s + v * v into an fma in one kernel and not in another: the round's
// accept bit and the regenerated / staged distance must be the same bits)
__device__ __forceinline__ double pterm(double v, double p) {
#pragma clang fp contract(off)
  return (p == 1.0) ? v : (p == 2.0 ? v * v : pow(v, p));
}
// running p-norm state s (sum of |.|^p, or max for p = inf); order = k order.
// PK = 2: p == 2 known at compile time (the same operations as the runtime
// p == 2 branch, so the same bits); PK = 0: any p.  A kernel that can meet a
// general p carries pow's constants in registers for its whole candidate loop
// (~30 VGPRs), so the hot kernels are instantiated for p == 2 separately.
template <int PK = 0>
__device__ __forceinline__ double pnorm_acc(double s, double v, double p) {
#pragma clang fp contract(off)
  if constexpr (PK == 2) return s + v * v;
  return isinf(p) ? fmax(s, v) : s + pterm(v, p);
}
template <int PK = 0>
__device__ __forceinline__ double pnorm_finish(double s, double p) {
#pragma clang fp contract(off)
  if constexpr (PK == 2) return sqrt(s);
  return isinf(p) ? s : ((p == 1.0) ? s : (p == 2.0 ? sqrt(s) : pow(s, 1.0 / p)));
}
// one simulated statistic (simulate_lg_kernel's formula)
__device__ __forceinline__ double lg_stat(double a, double sigma, double th_src, double e) {
  return a * th_src + sigma * e;
}

// Simulate statistics [q0, q1) (q0 even, q1 <= SIM_SMAX) of candidate g and
// fold them into the p-norm state s in k order; x (nullable) receives the
// row.  Statistic k uses normal k of the candidate's simulation stream (slot
// SLOT_SIM + k/4).  theta_{src_k} is read from tsrc[src_k * tstride] (a
// theta row in memory; sim_pnorm_regs below for theta in registers); x[k -
// xoff] receives statistic k.
template <int PK = 0>
__device__ __forceinline__ double sim_pnorm_range(const SimDistArgs& M, const BlockConsts& C,
                                                  const double* tsrc, int tstride,
                                                  uint64_t g, uint32_t gen,
                                                  uint64_t seed, int q0, int q1,
                                                  double s, double* x, int xoff = 0) {
  u32x4 r;
  if (q0 < q1 && (q0 & 3)) r = philox(g, SLOT_SIM + (uint32_t)(q0 >> 2), gen, seed);
#pragma unroll 1
  for (int q = q0; q < q1; q += 2) {
    if ((q & 3) == 0) r = philox(g, SLOT_SIM + (uint32_t)(q >> 2), gen, seed);
    double n2[2];
    box_muller((q & 2) ? r.z : r.x, (q & 2) ? r.w : r.y, n2[0], n2[1], C.bmt);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = q + t;
      if (k < q1) {
        const double2 as = C.as[k], wx = C.wx[k];
        const double xv = lg_stat(as.x, as.y, tsrc[C.src[k] * tstride], n2[t]);
        if (x) x[k - xoff] = xv;
        s = pnorm_acc<PK>(s, fabs(wx.x * (xv - wx.y)), M.p);
      }
    }
  }
  return s;
}

// sim_pnorm_range with theta in registers (D > 0): src_k is block-uniform, so
// th[src_k] is a register-indexed read with an SGPR index (readfirstlane of
// the LDS value) instead of an LDS slab of every thread's theta, which would
// cost 8 D bytes of LDS per thread and halve the occupancy.
template <int D, int PK = 0>
__device__ __forceinline__ double sim_pnorm_regs(const SimDistArgs& M, const BlockConsts& C,
                                                 const double (&th)[D], uint64_t g,
                                                 uint32_t gen, uint64_t seed, int q0, int q1,
                                                 double s, double* x, int xoff = 0) {
  u32x4 r;
  if (q0 < q1 && (q0 & 3)) r = philox(g, SLOT_SIM + (uint32_t)(q0 >> 2), gen, seed);
#pragma unroll 1
  for (int q = q0; q < q1; q += 2) {
    if ((q & 3) == 0) r = philox(g, SLOT_SIM + (uint32_t)(q >> 2), gen, seed);
    double n2[2];
    box_muller((q & 2) ? r.z : r.x, (q & 2) ? r.w : r.y, n2[0], n2[1], C.bmt);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = q + t;
      if (k < q1) {
        const double2 as = C.as[k], wx = C.wx[k];
        const int sk = __builtin_amdgcn_readfirstlane(C.src[k]);
        const double xv = lg_stat(as.x, as.y, th[sk], n2[t]);
        if (x) x[k - xoff] = xv;
        s = pnorm_acc<PK>(s, fabs(wx.x * (xv - wx.y)), M.p);
      }
    }
  }
  return s;
}

// The lazy early reject for CG candidates at once: theta_0..LAZY_KT-1 of
// attempt 0 (propose_one's operations in propose_one's order: same streams,
// same fma chain, same X_j + (L n)_k) and statistics 0..3 (sim_pnorm_regs's
// operations), in stages so that the memory accesses of the CG candidates
// overlap with each other and with arithmetic: the guide loads of all CG
// are issued, their perturbation normals computed (independent of the
// ancestor), the searches finished and the X heads loaded (the record line
// the search probes), the simulation normals computed, then theta, the
// statistics and the partial p-norm.  keep[c]: candidate c may be accepted (its head left the
// support, or its partial distance is <= eps).
template <int D, int PK, int CG>
__device__ __forceinline__ void lazy_head_group(const ProposalArgs& A, const SimDistArgs& M,
                                                const BlockConsts& C, const uint64_t (&g)[CG],
                                                double eps, bool (&keep)[CG]) {
  constexpr int KT = LAZY_KT;
  static_assert(D > KT, "lazy_head_group: D > LAZY_KT");
  int oz = 0;
  asm volatile("" : "+s"(oz));
  const double* LT = C.LT + oz;
  const double* box = C.box + oz;
  double target[CG];
  int32_t glo[CG], ghi[CG];
  uint32_t az[CG], aw[CG];   // the ancestor draw's second pair: normals 0, 1
#pragma unroll
  for (int c = 0; c < CG; ++c) {
    const u32x4 r = philox(g[c], SLOT_ANCESTOR, A.gen, A.seed);
    target[c] = uniform53(r.x, r.y) * C.total;
    az[c] = r.z;
    aw[c] = r.w;
    const int64_t kt = anc_bin(target[c], C.inv_step, A.G);
    glo[c] = A.bguide[kt];
    ghi[c] = A.bguide[kt + 1];
  }
  double th[CG][KT];
#pragma unroll
  for (int c = 0; c < CG; ++c) {
#pragma unroll
    for (int k = 0; k < KT; ++k) th[c][k] = 0.0;
    const u32x4 r = philox(g[c], SLOT_PERTURB, A.gen, A.seed);
#pragma unroll
    for (int q = 0; q < KT; q += 2) {
      // (perturb_words: pair 0 from the ancestor draw, pair 1 from x, y)
      double n0, n1;
      box_muller(q == 0 ? az[c] : r.x, q == 0 ? aw[c] : r.y, n0, n1, C.bmt);
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        if (k >= q) th[c][k] = fma(LT[q * D + k], n0, th[c][k]);
        if (k >= q + 1) th[c][k] = fma(LT[(q + 1) * D + k], n1, th[c][k]);
      }
    }
  }
  const double* xh[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) {
    const int64_t j = table_finish(A.rec, A.rs, D, A.N, target[c],
                                   AncestorBracket{(int64_t)glo[c], (int64_t)ghi[c]});
    xh[c] = A.rec + j * A.rs;
  }
  double xv4[CG][KT];
#pragma unroll
  for (int c = 0; c < CG; ++c)
#pragma unroll
    for (int k = 0; k < KT; ++k) xv4[c][k] = xh[c][k];
  double e[CG][4];
#pragma unroll
  for (int c = 0; c < CG; ++c) {
    const u32x4 r = philox(g[c], SLOT_SIM, A.gen, A.seed);
    box_muller(r.x, r.y, e[c][0], e[c][1], C.bmt);
    box_muller(r.z, r.w, e[c][2], e[c][3], C.bmt);
  }
#pragma unroll
  for (int c = 0; c < CG; ++c) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      th[c][k] = xv4[c][k] + th[c][k];
      ok = ok & (box[2 * k] <= th[c][k]) & (th[c][k] <= box[2 * k + 1]);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 as = C.as[k], wx = C.wx[k];
      const int sk = __builtin_amdgcn_readfirstlane(C.src[k]);
      const double xv = lg_stat(as.x, as.y, th[c][sk], e[c][k]);
      s = pnorm_acc<PK>(s, fabs(wx.x * (xv - wx.y)), M.p);
    }
    keep[c] = !ok || !(pnorm_finish<PK>(s, M.p) > eps);
  }
}

}  // namespace abc
