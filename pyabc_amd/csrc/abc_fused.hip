// Fused candidate round: one launch runs the whole per-candidate closure of
// pyabc/smc.py:588-724 for B candidates -- proposal with prior re-draw
// (smc.py:610-662), LinearGaussianModel simulation (model.py:89-116),
// PNormDistance (distance/distance.py:79-105) and the UniformAcceptor test
// d <= eps (acceptor/acceptor.py:235-244) -- and keeps nothing per candidate
// but one accept bit.  The sampler loop it serves is
// sampler/singlecore.py:20-38 / multicore_evaluation_parallel.py:92-150
// (draw until n accepted, keep the first n by evaluation index).
//
// Because every draw is keyed by (seed, generation, global index, slot), the
// rows of the few accepted candidates are not stored by the round: the
// regeneration kernel recomputes theta, prior log-density, ancestor, sum
// stats and distance for the kept indices with the same device functions
// (abc_candidate.h), bit for bit.  Per rejected candidate the round moves
// ~1/8 byte to HBM instead of ~440 B for the staged pipeline.
//
// Filter mode (low acceptance): phase A proposes every candidate of a tile
// and simulates only its first group of 4 statistics; the p-norm partial sum
// of nonnegative terms can only grow, so a partial distance > eps rejects the
// candidate exactly.  Survivors are queued in LDS and phase B evaluates them
// in full, dense across the block's waves (no lane idles behind an early
// exit).
#include "abc_candidate.h"

namespace abc {
namespace {

constexpr int FR_T = 256;                // threads per block
constexpr int FR_CPT = 8;                // candidates per thread and tile
constexpr int FR_TILE = FR_T * FR_CPT;   // candidates per block
constexpr int FR_WORDS = FR_TILE / 64;   // 64-bit accept words per tile
constexpr int FR_CG = 2;                 // lazy early reject: candidates in flight per thread

struct RoundArgs {
  ProposalArgs P;
  SimDistArgs M;
  const double* box;  // prior support [d x (lo, hi)] (support_box_kernel)
  const double* eps_dev;   // nullable: threshold *eps_dev * eps_scale
  double eps_scale;
};

// Full evaluation of candidate g: proposal + simulation + distance.  Returns
// the distance (NaN when the proposal gave up on the prior support: never
// accepted, even at eps = +inf), the attempts and the ancestor through the
// references; x (nullable) gets the row.
template <int D, int MODE, int PK>
__device__ __forceinline__ double evaluate_full(const RoundArgs& A, const BlockConsts& C,
                                                uint64_t g,
                                                double* th, int64_t& j, int& att, double* x) {
  att = propose_one<D, MODE, true>(A.P, C, g, th, j);
  double s;
  if constexpr (D > 0) {
    s = sim_pnorm_regs<D, PK>(A.M, C, *reinterpret_cast<const double(*)[D]>(th), g, A.P.gen,
                          A.P.seed, 0, A.M.S, 0.0, x);
  } else {
    s = sim_pnorm_range<PK>(A.M, C, th, 1, g, A.P.gen, A.P.seed, 0, A.M.S, 0.0, x);
  }
  const double dist = pnorm_finish<PK>(s, A.M.p);
  return att <= A.P.max_attempts ? dist : NAN;
}

// Rows written through LDS: one group = FR_T candidates (one per thread)
// whose sum-stat rows are out[0 .. nvalid) (S doubles each, consecutive).
// Each chunk of XCH statistics goes to an LDS tile [FR_T][XCH + 1] and then
// leaves the block as row segments, XCH consecutive doubles per row, instead
// of one 8-byte store per thread and statistic into FR_T different rows.
// The p-norm state runs through the chunks in k order (the same bits as one
// pass).  Used by the regeneration of kept rows (c4, S = 256: 565 -> 480 us
// per call); in the round's record_rejected path the barriers and the LDS
// cost more than the stores save (1.03 -> 1.59 ms per round at c4).
// Every thread of the block calls it (barriers inside); `valid` false only
// keeps the thread in step.  Returns the distance as evaluate_full.
constexpr int XCH = 16;  // multiple of 4: chunks start on a Philox slot
template <int D, int MODE, int PK>
__device__ __forceinline__ double evaluate_staged(const RoundArgs& A, const BlockConsts& C,
                                                  uint64_t g, bool valid, double* th,
                                                  int64_t& j, int& att, double* out,
                                                  int nvalid, double (*stage)[XCH + 1]) {
  const int t = threadIdx.x;
  const int S = A.M.S;
  att = valid ? propose_one<D, MODE, true>(A.P, C, g, th, j) : A.P.max_attempts + 1;
  double s = 0.0;
  for (int k0 = 0; k0 < S; k0 += XCH) {
    const int k1 = k0 + XCH < S ? k0 + XCH : S;
    if (valid) {
      if constexpr (D > 0) {
        s = sim_pnorm_regs<D, PK>(A.M, C, *reinterpret_cast<const double(*)[D]>(th), g,
                                  A.P.gen, A.P.seed, k0, k1, s, stage[t], k0);
      } else {
        s = sim_pnorm_range<PK>(A.M, C, th, 1, g, A.P.gen, A.P.seed, k0, k1, s, stage[t], k0);
      }
    }
    __syncthreads();
    const int w = k1 - k0;
    for (int e = t; e < FR_T * w; e += FR_T) {
      const int r = e / w, c = e - r * w;
      if (r < nvalid) out[(int64_t)r * S + k0 + c] = stage[r][c];
    }
    __syncthreads();
  }
  const double dist = pnorm_finish<PK>(s, A.M.p);
  return att <= A.P.max_attempts ? dist : NAN;
}

template <int D, int MODE, bool FILTER, int PK>
__device__ __forceinline__ void round_body(
    RoundArgs A, int64_t idx0, int64_t B, double eps_host,
    uint64_t* __restrict__ bits, int64_t* __restrict__ tile_cnt,
    double* __restrict__ rec_x) {
  // the threshold read on the device (the host's float(q) * multiplier, one
  // IEEE product either way)
  const double eps = A.eps_dev ? (*A.eps_dev) * A.eps_scale : eps_host;
  constexpr bool filter = FILTER;
  constexpr int DM = D > 0 ? D : 64;
  __shared__ BlockConsts C;
  stage_block_consts<D, MODE, true>(C, A.P, &A.M, A.box);
  __shared__ uint32_t tbits[FR_TILE / 32];
  __shared__ uint16_t queue[FR_TILE];
  __shared__ int qn;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int d = D > 0 ? D : A.P.d;
  const int64_t tile0 = (int64_t)blockIdx.x * FR_TILE;
  if (tid < FR_TILE / 32) tbits[tid] = 0u;
  if (tid == 0) {
    qn = 0;
    if (FILTER) C.lazy = lazy_filter_ok<D, MODE>(C, A.P, A.M) ? 1 : 0;
  }
  __syncthreads();
  double th[DM];
  int64_t j;
  int att;
  if (FILTER) {
    // phase A: proposal + first group of 4 statistics; an exact early reject
    bool lazy_done = false;
    if constexpr (MODE == PROP_MVN && D > LAZY_KT && D <= LT_DMAX) {
      if (C.lazy) {
        // lazy head: theta_0..3 of attempt 0 and statistics 0..3 only, FR_CG
        // candidates at a time (lazy_head_group); a head outside the
        // support (attempt 0 may be re-drawn) survives
#pragma unroll 1
        for (int it = 0; it < FR_CPT; it += FR_CG) {
          uint64_t gs[FR_CG];
          bool keep[FR_CG];
#pragma unroll
          for (int c = 0; c < FR_CG; ++c) gs[c] = (uint64_t)(idx0 + tile0 + (it + c) * FR_T + tid);
          lazy_head_group<D, PK, FR_CG>(A.P, A.M, C, gs, eps, keep);
#pragma unroll
          for (int c = 0; c < FR_CG; ++c) {
            const int loc = (it + c) * FR_T + tid;
            if (keep[c] && tile0 + loc < B) {
              const int pos = atomicAdd(&qn, 1);
              queue[pos] = (uint16_t)loc;
            }
          }
        }
        lazy_done = true;
      }
    }
#pragma unroll 1
    for (int it = 0; it < (lazy_done ? 0 : FR_CPT); ++it) {
      const int loc = it * FR_T + tid;
      const int64_t b = tile0 + loc;
      if (b < B) {
        const uint64_t g = (uint64_t)(idx0 + b);
        att = propose_one<D, MODE, true>(A.P, C, g, th, j);
        double s;
        if constexpr (D > 0) {
          s = sim_pnorm_regs<D, PK>(A.M, C, *reinterpret_cast<const double(*)[D]>(th), g,
                                A.P.gen, A.P.seed, 0, 4, 0.0, nullptr);
        } else {
          s = sim_pnorm_range<PK>(A.M, C, th, 1, g, A.P.gen, A.P.seed, 0, 4, 0.0, nullptr);
        }
        if (att <= A.P.max_attempts && !(pnorm_finish<PK>(s, A.M.p) > eps)) {
          const int pos = atomicAdd(&qn, 1);
          queue[pos] = (uint16_t)loc;
        }
      }
    }
    __syncthreads();
  }
  // full evaluation: every candidate of the tile, or the phase-A survivors
  // (dense over the block's waves)
  const int n = filter ? qn : FR_TILE;
#pragma unroll 1
  for (int i = tid; i < n; i += FR_T) {
    const int loc = filter ? (int)queue[i] : i;
    const int64_t b = tile0 + loc;
    if (b < B) {
      double* xr = rec_x ? rec_x + b * A.M.S : nullptr;
      const double dist = evaluate_full<D, MODE, PK>(A, C, (uint64_t)(idx0 + b), th, j, att,
                                                  xr);
      if (dist <= eps) atomicOr(&tbits[loc >> 5], 1u << (loc & 31));
    }
  }
  __syncthreads();
  // accept words of the tile + its count (wave 0)
  if (wave == 0) {
    int c = 0;
    if (lane < FR_WORDS) {
      const uint64_t w = (uint64_t)tbits[2 * lane] | ((uint64_t)tbits[2 * lane + 1] << 32);
      const int64_t word = tile0 / 64 + lane;
      if (word * 64 < B) bits[word] = w;
      c = __popcll(w);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) tile_cnt[blockIdx.x] = c;
  }
}

// the plain and the early-reject round as separate kernels (a runtime
// switch would give both the register allocation of the larger one), each
// for p == 2 and for any p (pnorm_acc)
#define ABC_ROUND_KERNEL(NAME, FILTER, PK, REC)                                       \
  template <int D, int MODE>                                                          \
  __global__ __launch_bounds__(FR_T) void NAME(RoundArgs A, int64_t idx0, int64_t B,  \
                                               double eps, uint64_t* bits,            \
                                               int64_t* tile_cnt, double* rec_x) {    \
    round_body<D, MODE, FILTER, PK>(A, idx0, B, eps, bits, tile_cnt,                  \
                                    REC ? rec_x : nullptr);                           \
  }
ABC_ROUND_KERNEL(fused_round_plain, false, 0, true)
ABC_ROUND_KERNEL(fused_round_plain_p2, false, 2, true)
ABC_ROUND_KERNEL(fused_round_filter, true, 0, false)
ABC_ROUND_KERNEL(fused_round_filter_p2, true, 2, false)
#undef ABC_ROUND_KERNEL

// one wave per dimension (support_bounds_wave): ~1 us instead of the ~40 us
// of one thread's 126 dependent bisection steps
__global__ __launch_bounds__(64) void support_box_kernel(const int32_t* __restrict__ kind,
                                                         const double* __restrict__ params,
                                                         int d, double* __restrict__ box) {
  const int k = blockIdx.x;
  if (k < d) support_bounds_wave(kind[k], params + 4 * k, box + 2 * k);
}

// ---- order-preserving compaction of the accept bits -----------------------
// exclusive scan of the tile counts in place, total -> *count: per block of
// SC_N tiles a local scan (scan_partial: block sums), one block scans the
// block sums (scan_top), then each block adds its offset (scan_apply)
constexpr int SC_T = 256, SC_PER = 4, SC_N = SC_T * SC_PER;

__device__ __forceinline__ int64_t block_exscan(int64_t v, int64_t* sh, int64_t& total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < SC_T; o <<= 1) {
    const int64_t add = (t >= o) ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  total = sh[SC_T - 1];
  const int64_t ex = sh[t] - v;
  __syncthreads();
  return ex;
}

__global__ __launch_bounds__(SC_T) void scan_partial(const int64_t* __restrict__ cnt,
                                                     int64_t n, int64_t* __restrict__ bsum) {
  __shared__ int64_t sh[SC_T];
  const int64_t b0 = (int64_t)blockIdx.x * SC_N + threadIdx.x * SC_PER;
  int64_t v = 0;
#pragma unroll
  for (int k = 0; k < SC_PER; ++k)
    if (b0 + k < n) v += cnt[b0 + k];
  int64_t tot;
  block_exscan(v, sh, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SC_T) void scan_top(int64_t* __restrict__ bsum, int64_t nb,
                                                 int64_t* __restrict__ count) {
  __shared__ int64_t sh[SC_T];
  const int64_t per = (nb + SC_T - 1) / SC_T;
  const int64_t b0 = threadIdx.x * per;
  int64_t v = 0;
  for (int64_t k = 0; k < per; ++k)
    if (b0 + k < nb) v += bsum[b0 + k];
  int64_t tot;
  int64_t off = block_exscan(v, sh, tot);
  for (int64_t k = 0; k < per; ++k)
    if (b0 + k < nb) { const int64_t x = bsum[b0 + k]; bsum[b0 + k] = off; off += x; }
  if (threadIdx.x == 0) *count = tot;
}

__global__ __launch_bounds__(SC_T) void scan_apply(int64_t* __restrict__ cnt, int64_t n,
                                                   const int64_t* __restrict__ boff) {
  __shared__ int64_t sh[SC_T];
  const int64_t b0 = (int64_t)blockIdx.x * SC_N + threadIdx.x * SC_PER;
  int64_t c[SC_PER];
  int64_t v = 0;
#pragma unroll
  for (int k = 0; k < SC_PER; ++k) {
    c[k] = b0 + k < n ? cnt[b0 + k] : 0;
    v += c[k];
  }
  int64_t tot;
  int64_t off = block_exscan(v, sh, tot) + boff[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SC_PER; ++k)
    if (b0 + k < n) { cnt[b0 + k] = off; off += c[k]; }
}

// one lane per 64-bit word: positions of the set bits, in increasing order,
// for output slots < cap
__global__ __launch_bounds__(256) void bits_write_kernel(
    const uint64_t* __restrict__ bits, int64_t nwords,
    const int64_t* __restrict__ tile_off, int64_t cap, int64_t* __restrict__ idx) {
  const int64_t wd = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  uint64_t w = wd < nwords ? bits[wd] : 0ull;
  // exclusive popcount prefix among the FR_WORDS words of this tile
  // (tiles are FR_WORDS = 32 aligned words: half a wave)
  int c = __popcll(w);
  int incl = c;
#pragma unroll
  for (int o = 1; o < FR_WORDS; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if ((lane & (FR_WORDS - 1)) >= o) incl += v;
  }
  if (wd >= nwords || w == 0ull) return;
  int64_t pos = tile_off[wd / FR_WORDS] + (incl - c);
  while (w != 0ull && pos < cap) {
    const int bit = __ffsll((long long)w) - 1;
    idx[pos++] = wd * 64 + bit;
    w &= w - 1;
  }
}

// ---- regeneration of kept rows ----------------------------------------------
template <int D, int MODE>
__global__ __launch_bounds__(256) void fused_regen_kernel(
    RoundArgs A, int64_t idx0, const int64_t* __restrict__ idx, int64_t n,
    const int64_t* __restrict__ n_dev, double* __restrict__ theta, double* __restrict__ lp,
    int64_t* __restrict__ anc, double* __restrict__ x, double* __restrict__ dist) {
  constexpr int DM = D > 0 ? D : 64;
  __shared__ BlockConsts C;
  __shared__ double stage[FR_T][XCH + 1];
  // device-sized launch: blocks past the round's count leave at once
  // (uniform per block, before any barrier)
  if (n_dev && *n_dev < n) n = *n_dev > 0 ? *n_dev : 0;
  if ((int64_t)blockIdx.x * FR_T >= n) return;
  stage_block_consts<D, MODE>(C, A.P, &A.M, nullptr);
  const int d = D > 0 ? D : A.P.d;
  const int64_t i0 = (int64_t)blockIdx.x * FR_T;
  const int64_t i = i0 + threadIdx.x;
  const bool valid = i < n;
  const int nvalid = n - i0 < FR_T ? (int)(n - i0) : FR_T;
  double th[DM];
  int64_t j = -1;
  int att;
  // the kept rows x[i] (consecutive) leave through LDS (evaluate_staged)
  const double dd = evaluate_staged<D, MODE, 0>(A, C, valid ? (uint64_t)(idx0 + idx[i]) : 0ull,
                                                valid, th, j, att, x + i0 * A.M.S, nvalid, stage);
  if (!valid) return;
#pragma unroll
  for (int k = 0; k < (D > 0 ? D : d); ++k) theta[i * d + k] = th[k];
  lp[i] = att <= A.P.max_attempts ? prior_logpdf(A.P.kind, A.P.params, d, th) : -INFINITY;
  if (anc) anc[i] = j;
  dist[i] = dd;
}

// ---- proposals only (the staged path of models without a fused simulator) --
// Rows [0, B) of candidates idx0 + b: theta, prior log-density, ancestor,
// attempts.  The same propose_one as the round and the regeneration (the
// ancestor table, the support box computed once), so the staged path's
// proposals are the fused path's bits; each block proposes FP_CPT groups of
// FR_T candidates with its constants staged once.
constexpr int FP_CPT = 4;
template <int D, int MODE>
__global__ __launch_bounds__(256) void fused_propose_kernel(
    RoundArgs A, int64_t idx0, int64_t B, double* __restrict__ theta,
    double* __restrict__ lp, int64_t* __restrict__ anc, int32_t* __restrict__ att_out) {
  constexpr int DM = D > 0 ? D : 64;
  __shared__ BlockConsts C;
  stage_block_consts<D, MODE, true>(C, A.P, nullptr, A.box);
  const int d = D > 0 ? D : A.P.d;
  // rows stored straight from registers: a wave's d stores cover its 64 rows'
  // 64 d contiguous doubles, which L2 merges into whole lines (an LDS
  // transposition with two barriers per 256 rows ran at 1.2e10 rows/s)
  for (int c = 0; c < FP_CPT; ++c) {
    const int64_t i = ((int64_t)blockIdx.x * FP_CPT + c) * FR_T + threadIdx.x;
    if (i >= B) break;
    double th[DM];
    int64_t j = -1;
    const int att = propose_one<D, MODE, true>(A.P, C, (uint64_t)(idx0 + i), th, j);
    double* row = theta + i * d;
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) row[k] = th[k];
    if (lp) lp[i] = att <= A.P.max_attempts ? prior_logpdf(A.P.kind, A.P.params, d, th) : -INFINITY;
    if (anc) anc[i] = j;
    if (att_out) att_out[i] = att;
  }
}

// ---- the accept tail of user simulators ---------------------------------------
// A VectorizedModel without a fused simulator hands the sampler its sum stats
// x [B x S]; one pass over them computes PNormDistance (distance.py:79-105)
// and the UniformAcceptor test d <= eps (acceptor.py:235-244) and leaves only
// the accept bits + per-tile counts of the fused round, whose scan and
// bits_write turn them into the positions of the first `cap` accepted: no
// distance array is written and re-read.  The arithmetic per row is
// pnorm_row_kernel's (S <= 32: thread per row, k order) or pnorm_wave_kernel's
// (wide rows: lane-strided partials then the wave tree), so the decision is
// the one dist <= eps of abc_pnorm's value would give, and the kept rows'
// distances recomputed by abc_pnorm are those bits.  A proposal that gave up
// on the prior support (attempts > max_attempts) is never accepted, as
// abc_mask_gave_up's NaN.
constexpr int PA_ROWS = 8;    // rows in flight per wave (wide path)
// rows per LDS chunk of the row path: 256, fewer when 256 padded rows of S
// doubles would pass 64 KB (S = 32: 248); even, so chunks stay 16-B aligned
__host__ __device__ constexpr int pa_chunk_rows(int S) {
  return (65536 / ((S + 1) * 8)) >= FR_T ? FR_T : ((65536 / ((S + 1) * 8)) & ~1);
}
template <bool WIDE>
__global__ __launch_bounds__(FR_T) void pnorm_accept_kernel(
    const double* __restrict__ x, int64_t B, int S, const double* __restrict__ x0,
    const double* __restrict__ wf, double p, double eps, const int32_t* __restrict__ att,
    int max_attempts, uint64_t* __restrict__ bits, int64_t* __restrict__ tile_cnt) {
  __shared__ uint32_t tbits[FR_TILE / 32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t tile0 = (int64_t)blockIdx.x * FR_TILE;
  if (tid < FR_TILE / 32) tbits[tid] = 0u;
  __syncthreads();
  const bool inf = isinf(p);
  auto finish = [&](double t) {
    return inf ? t : ((p == 1.0) ? t : (p == 2.0 ? sqrt(t) : pow(t, 1.0 / p)));
  };
  auto ok = [&](int64_t b) { return att == nullptr || att[b] <= max_attempts; };
  if (!WIDE) {
    // chunks of RC rows (pa_chunk_rows: 256, or what 64 KB of LDS holds):
    // the chunk's RC * S contiguous doubles come in with 16-B coalesced loads
    // (the next chunk's held in registers while this one is summed), land in
    // LDS rows of stride S + 1 (2-way banked reads), and each thread sums its
    // row in k order as abc_pnorm does
    extern __shared__ double pa_rows[];
    const int S1 = S + 1;
    const int RC = pa_chunk_rows(S);
    const int n16 = RC * S / 2;                   // 16-B pieces per chunk (RC even)
    const int per = (n16 + FR_T - 1) / FR_T;      // <= 16 for S <= 32
    double2 hold[16];
    auto fetch = [&](int it) {
      const int64_t e0 = (tile0 + (int64_t)it * RC) * S;   // first double of the chunk
      const int64_t eend = B * S;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q >= per) break;
        const int piece = q * FR_T + tid;
        const int64_t e = e0 + 2 * (int64_t)piece;
        if (piece < n16 && e + 1 < eend) {
          hold[q] = *reinterpret_cast<const double2*>(x + e);
        } else if (piece < n16 && e < eend) {
          hold[q] = double2{x[e], 0.0};
        }
      }
    };
    auto stash = [&]() {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q >= per) break;
        const int piece = q * FR_T + tid;
        if (piece < n16) {
          const int e = 2 * piece;
          const int r0 = e / S, k0 = e - r0 * S;
          pa_rows[r0 * S1 + k0] = hold[q].x;
          const int r1 = (e + 1) / S, k1 = e + 1 - r1 * S;
          pa_rows[r1 * S1 + k1] = hold[q].y;
        }
      }
    };
    const int64_t rows = B - tile0 < FR_TILE ? B - tile0 : FR_TILE;
    const int nchunk = (int)((rows + RC - 1) / RC);
    fetch(0);
#pragma unroll 1
    for (int it = 0; it < nchunk; ++it) {
      __syncthreads();                 // the previous chunk's rows are read
      stash();
      __syncthreads();
      if (it + 1 < nchunk) fetch(it + 1);
      const int loc = it * RC + tid;
      const int64_t b = tile0 + loc;
      if (tid < RC && loc < FR_TILE && b < B) {
        const double* xr = pa_rows + tid * S1;
        double s = 0.0;
        if (inf) {
          for (int k = 0; k < S; ++k) s = fmax(s, fabs(wf[k] * (xr[k] - x0[k])));
        } else {
          for (int k = 0; k < S; ++k) s += pterm(fabs(wf[k] * (xr[k] - x0[k])), p);
        }
        if (finish(s) <= eps && ok(b)) atomicOr(&tbits[loc >> 5], 1u << (loc & 31));
      }
    }
  } else {
    // wave w takes rows w * PA_ROWS + 4 PA_ROWS i of the tile
#pragma unroll 1
    for (int r0 = wave * PA_ROWS; r0 < FR_TILE; r0 += 4 * PA_ROWS) {
      const int64_t b0 = tile0 + r0;
      if (b0 >= B) break;  // wave-uniform
      double sr[PA_ROWS];
#pragma unroll
      for (int r = 0; r < PA_ROWS; ++r) sr[r] = 0.0;
      for (int k = lane; k < S; k += 64) {
        const double wk = wf[k], ck = x0[k];
        double v[PA_ROWS];
#pragma unroll
        for (int r = 0; r < PA_ROWS; ++r) v[r] = b0 + r < B ? x[(b0 + r) * S + k] : ck;
#pragma unroll
        for (int r = 0; r < PA_ROWS; ++r) {
          const double a = fabs(wk * (v[r] - ck));
          sr[r] = inf ? fmax(sr[r], a) : sr[r] + pterm(a, p);
        }
      }
#pragma unroll
      for (int r = 0; r < PA_ROWS; ++r) {
        const double t = inf ? wave_max(sr[r]) : wave_sum(sr[r]);
        const int loc = r0 + r;
        if (lane == 0 && b0 + r < B && finish(t) <= eps && ok(b0 + r))
          atomicOr(&tbits[loc >> 5], 1u << (loc & 31));
      }
    }
  }
  __syncthreads();
  if (wave == 0) {
    int c = 0;
    if (lane < FR_WORDS) {
      const uint64_t w = (uint64_t)tbits[2 * lane] | ((uint64_t)tbits[2 * lane + 1] << 32);
      const int64_t word = tile0 / 64 + lane;
      if (word * 64 < B) bits[word] = w;
      c = __popcll(w);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) tile_cnt[blockIdx.x] = c;
  }
}

// accept bits + tile counts -> exclusive tile offsets, *count, and the first
// cap positions (the fused round's compaction)
int compact_accept_bits(const uint64_t* bits, int64_t* tcnt, int64_t nt, int64_t* bsum,
                        int64_t B, int64_t cap, int64_t* idx, int64_t* count, hipStream_t s) {
  const int64_t nb = ceil_div(nt, SC_N);
  hipLaunchKernelGGL(scan_partial, dim3((unsigned)nb), dim3(SC_T), 0, s, tcnt, nt, bsum);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(scan_top, dim3(1), dim3(SC_T), 0, s, bsum, nb, count);
  ABC_LAUNCHED();
  hipLaunchKernelGGL(scan_apply, dim3((unsigned)nb), dim3(SC_T), 0, s, tcnt, nt, bsum);
  ABC_LAUNCHED();
  if (cap > 0) {
    const int64_t nwords = ceil_div(B, 64);
    hipLaunchKernelGGL(bits_write_kernel, dim3((unsigned)ceil_div(nwords, 256)), dim3(256), 0,
                       s, bits, nwords, tcnt, cap, idx);
    ABC_LAUNCHED();
  }
  return ABC_OK;
}

// ---- ancestor table (abc_candidate.h) ---------------------------------------
__global__ __launch_bounds__(256) void anc_records_kernel(const double* __restrict__ X,
                                                          const double* __restrict__ cdf,
                                                          int64_t N, int d, int rs,
                                                          double* __restrict__ rec) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= N * rs) return;
  const int64_t i = e / rs;
  const int k = (int)(e - i * rs);
  rec[e] = k < d ? X[i * d + k] : (k == d ? cdf[i] : 0.0);
}

// max |X_jk| into the table header (lazy_filter_ok): a grid-stride pass
// with one atomic per block (one per wave on a single address serialised
// ~250k atomics per c3 table, ~3 ms); the bits of a non-negative double
// order like the value (a NaN sorts above +inf and disables the lazy head)
constexpr int XMAX_BLOCKS = 512;
__global__ __launch_bounds__(256) void anc_xmax_kernel(const double* __restrict__ X,
                                                       int64_t n,
                                                       unsigned long long* __restrict__ xmax_bits) {
  __shared__ unsigned long long wm[4];
  unsigned long long a = 0ull;  // bits of |x|: order like the values, NaN on top
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(fabs(X[e]));
    a = b > a ? b : a;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long b = __shfl_xor(a, o, 64);
    a = b > a ? b : a;
  }
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0ull;
    for (int w = 0; w < 4; ++w) m = wm[w] > m ? wm[w] : m;
    atomicMax(xmax_bits, m);
  }
}

// guide[k] = first i with anc_bin(cdf_i) >= k (N if none), k = 0 .. G + 1
__global__ __launch_bounds__(256) void anc_guide_kernel(const double* __restrict__ cdf,
                                                        int64_t N, int64_t G,
                                                        int32_t* __restrict__ guide) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k > G + 1) return;
  const double inv_step = (double)G / cdf[N - 1];  // as stage_block_consts
  int64_t lo = 0, hi = N;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (anc_bin(cdf[mid], inv_step, G) >= k) hi = mid; else lo = mid + 1;
  }
  guide[k] = (int32_t)lo;
}

// table layout: header (ANC_HDR) | records [N x rs] doubles | guide int32 [G + 2]
struct AncTable { const double* rec; const int32_t* guide; int rs; int64_t G; const double* xmax; };
inline AncTable anc_table_view(const void* t, int64_t N, int d) {
  AncTable v;
  v.xmax = static_cast<const double*>(t);  // header word 0
  v.rs = anc_rs(d);
  v.G = anc_bins(N);
  v.rec = reinterpret_cast<const double*>(static_cast<const char*>(t) + ANC_HDR);
  v.guide = reinterpret_cast<const int32_t*>(v.rec + N * v.rs);
  return v;
}

RoundArgs round_args(const abc_candidate_spec* s, const double* box) {
  RoundArgs A;
  A.box = box;
  A.eps_dev = nullptr;
  A.eps_scale = 1.0;
  A.P = ProposalArgs{s->X, s->cdf, s->guide, s->N, s->L, s->prior_kind,
                     s->prior_params, s->d, s->max_attempts, s->seed, s->generation};
  if (s->X && s->anc_table) {
    const AncTable v = anc_table_view(s->anc_table, s->N, s->d);
    A.P.rec = v.rec;
    A.P.bguide = v.guide;
    A.P.rs = v.rs;
    A.P.G = v.G;
    A.P.xmax = v.xmax;
  }
  A.M = SimDistArgs{s->src, s->a, s->sigma, s->x0, s->wf, s->p, s->S};
  return A;
}

int check_spec(const abc_candidate_spec* s) {
  ABC_CHECK_ARG(s != nullptr, "candidates: null spec");
  ABC_CHECK_ARG(s->d >= 1 && s->d <= 64 && s->S >= 1, "candidates: bad d/S");
  if (s->S > SIM_SMAX)
    return set_error(ABC_ERR_UNSUPPORTED, "candidates: S > %d (use the staged kernels)",
                     SIM_SMAX);
  ABC_CHECK_ARG(s->max_attempts >= 1 && s->max_attempts < (1 << 15),
                "candidates: bad max_attempts");
  ABC_CHECK_ARG(s->prior_kind && s->prior_params && s->src && s->a && s->sigma && s->x0 &&
                s->wf, "candidates: null pointer");
  ABC_CHECK_ARG(s->X == nullptr || (s->cdf && s->L && s->N >= 1),
                "candidates: population needs cdf, L, N");
  ABC_CHECK_ARG(s->p >= 1.0, "candidates: p < 1");
  ABC_CHECK_ARG(s->X == nullptr || s->anc_table, "candidates: population needs anc_table");
  return ABC_OK;
}

#define ABC_FUSED_DISPATCH(KERNEL, GRID, STREAM, ...)                          \
  do {                                                                         \
    const int mode_ = spec->X == nullptr ? PROP_PRIOR                          \
                      : (spec->per_particle_L ? PROP_LOCAL : PROP_MVN);        \
    switch (spec->d) {                                                         \
      ABC_FUSED_CASE(KERNEL, 1, GRID, STREAM, __VA_ARGS__)                     \
      ABC_FUSED_CASE(KERNEL, 2, GRID, STREAM, __VA_ARGS__)                     \
      ABC_FUSED_CASE(KERNEL, 3, GRID, STREAM, __VA_ARGS__)                     \
      ABC_FUSED_CASE(KERNEL, 4, GRID, STREAM, __VA_ARGS__)                     \
      ABC_FUSED_CASE(KERNEL, 5, GRID, STREAM, __VA_ARGS__)                     \
      ABC_FUSED_CASE(KERNEL, 6, GRID, STREAM, __VA_ARGS__)                     \
      ABC_FUSED_CASE(KERNEL, 8, GRID, STREAM, __VA_ARGS__)                     \
      ABC_FUSED_CASE(KERNEL, 10, GRID, STREAM, __VA_ARGS__)                    \
      ABC_FUSED_CASE(KERNEL, 12, GRID, STREAM, __VA_ARGS__)                    \
      ABC_FUSED_CASE(KERNEL, 16, GRID, STREAM, __VA_ARGS__)                    \
      default:                                                                 \
        ABC_FUSED_CASE_BODY(KERNEL, 0, GRID, STREAM, __VA_ARGS__)              \
    }                                                                          \
  } while (0)
#define ABC_FUSED_CASE_BODY(KERNEL, DD, GRID, STREAM, ...)                     \
  if (mode_ == PROP_MVN)                                                       \
    hipLaunchKernelGGL((KERNEL<DD, PROP_MVN>), GRID, dim3(256), 0, STREAM,     \
                       __VA_ARGS__);                                           \
  else if (mode_ == PROP_LOCAL)                                                \
    hipLaunchKernelGGL((KERNEL<DD, PROP_LOCAL>), GRID, dim3(256), 0, STREAM,   \
                       __VA_ARGS__);                                           \
  else                                                                         \
    hipLaunchKernelGGL((KERNEL<DD, PROP_PRIOR>), GRID, dim3(256), 0, STREAM,   \
                       __VA_ARGS__);                                           \
  break;
#define ABC_FUSED_CASE(KERNEL, DD, GRID, STREAM, ...)                          \
  case DD: { ABC_FUSED_CASE_BODY(KERNEL, DD, GRID, STREAM, __VA_ARGS__) }

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" size_t abc_candidates_workspace(int64_t B) {
  const int64_t nt = ceil_div(B > 0 ? B : 1, FR_TILE);
  size_t off = 0;
  size_only<uint64_t>(off, (size_t)nt * FR_WORDS);  // accept bits
  size_only<int64_t>(off, (size_t)nt);              // tile counts / offsets
  size_only<double>(off, 128);                      // prior support box
  size_only<int64_t>(off, (size_t)ceil_div(nt, SC_N));  // scan block sums
  return off + 256;
}

extern "C" int64_t abc_ancestor_table_bytes(int64_t N, int d) {
  if (N < 1 || d < 1) return 0;
  return ANC_HDR + N * anc_rs(d) * (int64_t)sizeof(double) +
         (anc_bins(N) + 2) * (int64_t)sizeof(int32_t);
}

extern "C" int abc_ancestor_table(const double* X, const double* cdf, int64_t N, int d,
                                  void* table, size_t table_bytes, void* stream) {
  ABC_CHECK_ARG(N >= 1 && N < (1ll << 31) && d >= 1 && d <= 64,
                "ancestor_table: bad N/d");
  ABC_CHECK_ARG(X && cdf && table, "ancestor_table: null pointer");
  ABC_CHECK_ARG(((uintptr_t)table & 127) == 0, "ancestor_table: table not 128-B aligned");
  if ((int64_t)table_bytes < abc_ancestor_table_bytes(N, d))
    return set_error(ABC_ERR_WORKSPACE, "ancestor_table: buffer too small");
  const AncTable v = anc_table_view(table, N, d);
  hipStream_t s = as_stream(stream);
  ABC_HIP(hipMemsetAsync(table, 0, ANC_HDR, s));
  hipLaunchKernelGGL(anc_records_kernel, dim3((unsigned)ceil_div(N * v.rs, 256)), dim3(256), 0,
                     s, X, cdf, N, d, v.rs, const_cast<double*>(v.rec));
  ABC_LAUNCHED();
  const int64_t nx = N * (int64_t)d;
  const int64_t xb = ceil_div(nx, 256) < XMAX_BLOCKS ? ceil_div(nx, 256) : XMAX_BLOCKS;
  hipLaunchKernelGGL(anc_xmax_kernel, dim3((unsigned)xb), dim3(256), 0, s, X, nx,
                     static_cast<unsigned long long*>(table));
  ABC_LAUNCHED();
  hipLaunchKernelGGL(anc_guide_kernel, dim3((unsigned)ceil_div(v.G + 2, 256)), dim3(256), 0, s,
                     cdf, N, v.G, const_cast<int32_t*>(v.guide));
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_candidates_round(const abc_candidate_spec* spec, int64_t idx0,
                                    int64_t B, double eps, const double* eps_dev,
                                    double eps_scale, int filter, int64_t cap,
                                    int64_t* idx, int64_t* count, double* rec_x,
                                    void* ws, size_t ws_bytes, void* stream) {
  const int rc = check_spec(spec);
  if (rc != ABC_OK) return rc;
  ABC_CHECK_ARG(B >= 0 && cap >= 0 && count, "candidates_round: bad B/cap/count");
  ABC_CHECK_ARG(B < (1ll << 40), "candidates_round: B too large");
  ABC_CHECK_ARG(cap == 0 || idx, "candidates_round: null idx");
  if (ws_bytes < abc_candidates_workspace(B))
    return set_error(ABC_ERR_WORKSPACE, "candidates_round: workspace too small");
  hipStream_t s = as_stream(stream);
  if (B == 0) {
    ABC_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), s));
    return ABC_OK;
  }
  // the filter is exact for p in {1, 2, inf} only (monotone finish) and
  // pointless when the first group of 4 statistics is all of them
  const double p = spec->p;
  const int filt = (filter && rec_x == nullptr && spec->S > 4 &&
                    (p == 1.0 || p == 2.0 || p == INFINITY)) ? 1 : 0;
  const int64_t nt = ceil_div(B, FR_TILE);
  Carver c(ws, ws_bytes);
  uint64_t* bits = c.take<uint64_t>((size_t)nt * FR_WORDS);
  int64_t* tcnt = c.take<int64_t>((size_t)nt);
  double* box = c.take<double>(128);
  int64_t* bsum = c.take<int64_t>((size_t)ceil_div(nt, SC_N));
  if (!c.ok) return set_error(ABC_ERR_WORKSPACE, "candidates_round: workspace");
  hipLaunchKernelGGL(support_box_kernel, dim3((unsigned)spec->d), dim3(64), 0, s,
                     spec->prior_kind, spec->prior_params, spec->d, box);
  ABC_LAUNCHED();
  RoundArgs A = round_args(spec, box);
  A.eps_dev = eps_dev;
  A.eps_scale = eps_scale;
  ABC_CHECK_ARG(nt < (1ll << 31), "candidates_round: too many tiles");
  profile_start(s, ABC_PROF_CANDIDATES);
  const bool p2 = p == 2.0;
  if (filt && p2)
    ABC_FUSED_DISPATCH(fused_round_filter_p2, dim3((unsigned)nt), s, A, idx0, B, eps, bits,
                       tcnt, rec_x);
  else if (filt)
    ABC_FUSED_DISPATCH(fused_round_filter, dim3((unsigned)nt), s, A, idx0, B, eps, bits, tcnt,
                       rec_x);
  else if (p2)
    ABC_FUSED_DISPATCH(fused_round_plain_p2, dim3((unsigned)nt), s, A, idx0, B, eps, bits,
                       tcnt, rec_x);
  else
    ABC_FUSED_DISPATCH(fused_round_plain, dim3((unsigned)nt), s, A, idx0, B, eps, bits, tcnt,
                       rec_x);
  profile_stop(s, ABC_PROF_CANDIDATES);
  ABC_LAUNCHED();
  return compact_accept_bits(bits, tcnt, nt, bsum, B, cap, idx, count, s);
}

extern "C" int abc_pnorm_accept(const double* x, int64_t B, int S, const double* x0,
                                const double* wf, double p, double eps,
                                const int32_t* attempts, int max_attempts, int64_t cap,
                                int64_t* idx, int64_t* count, void* ws, size_t ws_bytes,
                                void* stream) {
  ABC_CHECK_ARG(S >= 1 && B >= 0 && p >= 1.0 && cap >= 0, "pnorm_accept: bad S/B/p/cap");
  ABC_CHECK_ARG(B < (1ll << 40), "pnorm_accept: B too large");
  ABC_CHECK_ARG(count && (cap == 0 || idx), "pnorm_accept: null pointer");
  if (ws_bytes < abc_candidates_workspace(B))
    return set_error(ABC_ERR_WORKSPACE, "pnorm_accept: workspace too small");
  hipStream_t s = as_stream(stream);
  if (B == 0) {
    ABC_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), s));
    return ABC_OK;
  }
  ABC_CHECK_ARG(x && x0 && wf, "pnorm_accept: null pointer");
  const int64_t nt = ceil_div(B, FR_TILE);
  ABC_CHECK_ARG(nt < (1ll << 31), "pnorm_accept: too many tiles");
  Carver c(ws, ws_bytes);
  uint64_t* bits = c.take<uint64_t>((size_t)nt * FR_WORDS);
  int64_t* tcnt = c.take<int64_t>((size_t)nt);
  c.take<double>(128);
  int64_t* bsum = c.take<int64_t>((size_t)ceil_div(nt, SC_N));
  if (!c.ok) return set_error(ABC_ERR_WORKSPACE, "pnorm_accept: workspace");
  // the same row / wave split as abc_pnorm (the same bits per row)
  if (S <= 32)
    hipLaunchKernelGGL(pnorm_accept_kernel<false>, dim3((unsigned)nt), dim3(FR_T),
                       (size_t)pa_chunk_rows(S) * (S + 1) * sizeof(double), s, x, B, S, x0, wf, p, eps,
                       attempts, max_attempts, bits, tcnt);
  else
    hipLaunchKernelGGL(pnorm_accept_kernel<true>, dim3((unsigned)nt), dim3(FR_T), 0, s, x, B,
                       S, x0, wf, p, eps, attempts, max_attempts, bits, tcnt);
  ABC_LAUNCHED();
  return compact_accept_bits(bits, tcnt, nt, bsum, B, cap, idx, count, s);
}

extern "C" size_t abc_candidates_propose_workspace() { return 128 * sizeof(double) + 256; }

extern "C" int abc_candidates_propose(const abc_candidate_spec* spec, int64_t idx0, int64_t B,
                                      double* theta, double* prior_logpdf, int64_t* ancestor,
                                      int32_t* attempts, void* ws, size_t ws_bytes,
                                      void* stream) {
  const int rc = check_spec(spec);
  if (rc != ABC_OK) return rc;
  ABC_CHECK_ARG(B >= 0 && B < (1ll << 40), "candidates_propose: bad B");
  if (B == 0) return ABC_OK;
  ABC_CHECK_ARG(theta, "candidates_propose: null pointer");
  if (ws_bytes < abc_candidates_propose_workspace())
    return set_error(ABC_ERR_WORKSPACE, "candidates_propose: workspace too small");
  hipStream_t s = as_stream(stream);
  Carver c(ws, ws_bytes);
  double* box = c.take<double>(128);
  hipLaunchKernelGGL(support_box_kernel, dim3((unsigned)spec->d), dim3(64), 0, s,
                     spec->prior_kind, spec->prior_params, spec->d, box);
  ABC_LAUNCHED();
  const RoundArgs A = round_args(spec, box);
  const int64_t nb = ceil_div(B, (int64_t)FR_T * FP_CPT);
  ABC_CHECK_ARG(nb < (1ll << 31), "candidates_propose: too many blocks");
  ABC_FUSED_DISPATCH(fused_propose_kernel, dim3((unsigned)nb), s, A, idx0, B, theta,
                     prior_logpdf, ancestor, attempts);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_candidates_regen(const abc_candidate_spec* spec, int64_t idx0,
                                    const int64_t* idx, int64_t n, const int64_t* n_dev,
                                    double* theta, double* prior_logpdf, int64_t* ancestor,
                                    double* x, double* dist, void* stream) {
  const int rc = check_spec(spec);
  if (rc != ABC_OK) return rc;
  ABC_CHECK_ARG(n >= 0, "candidates_regen: n < 0");
  if (n == 0) return ABC_OK;
  ABC_CHECK_ARG(idx && theta && prior_logpdf && x && dist, "candidates_regen: null pointer");
  const RoundArgs A = round_args(spec, nullptr);  // box: per block, in LDS
  hipStream_t s = as_stream(stream);
  profile_start(s, ABC_PROF_REGEN);
  ABC_FUSED_DISPATCH(fused_regen_kernel, dim3((unsigned)ceil_div(n, 256)), s, A, idx0, idx, n,
                     n_dev, theta, prior_logpdf, ancestor, x, dist);
  profile_stop(s, ABC_PROF_REGEN);
  ABC_LAUNCHED();
  return ABC_OK;
}
