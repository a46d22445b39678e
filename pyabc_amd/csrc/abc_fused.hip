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

// One tile of the round: candidates tile0 + [0, cpt * FR_T) (cpt per thread,
// FR_CPT or FR_CPT_TAIL), its accept words into bits.  The block's constants
// C are staged; every thread calls it (barriers inside).
struct TileLds {
  uint32_t* tbits;   // [FR_TILE / 32]
  uint16_t* queue;   // [FR_TILE] (early-reject mode)
  int& qn;
};
template <int D, int MODE, bool FILTER, int PK>
__device__ __forceinline__ void tile_body(const RoundArgs& A, const BlockConsts& C, double eps,
                                          int64_t idx0, int64_t B, int64_t tile0, int cpt,
                                          uint64_t* __restrict__ bits,
                                          double* __restrict__ rec_x, TileLds T) {
  constexpr int DM = D > 0 ? D : 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tn = cpt * FR_T;                  // candidates of the tile
  if (tid < tn / 32) T.tbits[tid] = 0u;
  if (tid == 0) T.qn = 0;
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
        for (int it = 0; it < cpt; it += FR_CG) {
          uint64_t gs[FR_CG];
          bool keep[FR_CG];
#pragma unroll
          for (int c = 0; c < FR_CG; ++c) gs[c] = (uint64_t)(idx0 + tile0 + (it + c) * FR_T + tid);
          lazy_head_group<D, PK, FR_CG>(A.P, A.M, C, gs, eps, keep);
#pragma unroll
          for (int c = 0; c < FR_CG; ++c) {
            const int loc = (it + c) * FR_T + tid;
            if (keep[c] && tile0 + loc < B) {
              const int pos = atomicAdd(&T.qn, 1);
              T.queue[pos] = (uint16_t)loc;
            }
          }
        }
        lazy_done = true;
      }
    }
#pragma unroll 1
    for (int it = 0; it < (lazy_done ? 0 : cpt); ++it) {
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
          const int pos = atomicAdd(&T.qn, 1);
          T.queue[pos] = (uint16_t)loc;
        }
      }
    }
    __syncthreads();
  }
  // full evaluation: every candidate of the tile, or the phase-A survivors
  // (dense over the block's waves)
  const int n = FILTER ? T.qn : tn;
#pragma unroll 1
  for (int i = tid; i < n; i += FR_T) {
    const int loc = FILTER ? (int)T.queue[i] : i;
    const int64_t b = tile0 + loc;
    if (b < B) {
      double* xr = rec_x ? rec_x + b * A.M.S : nullptr;
      const double dist = evaluate_full<D, MODE, PK>(A, C, (uint64_t)(idx0 + b), th, j, att,
                                                  xr);
      if (dist <= eps) atomicOr(&T.tbits[loc >> 5], 1u << (loc & 31));
    }
  }
  __syncthreads();
  // accept words of the tile (wave 0)
  if (wave == 0 && lane < tn / 64) {
    const uint64_t w = (uint64_t)T.tbits[2 * lane] | ((uint64_t)T.tbits[2 * lane + 1] << 32);
    const int64_t word = tile0 / 64 + lane;
    if (word * 64 < B) bits[word] = w;
  }
}

// ---- the round: tiles handed out by a ticket counter -------------------------
// Blocks are placed on the 8 XCDs round-robin by block index, so a grid of
// one tile per block gives every XCD the same number of tiles however fast
// it runs: a block-level trace of round 5's kernel
// (profiles/r06_fused_block_trace.log) shows the XCDs' median tile times
// 99-104 us at c3's shape and their last tiles ending up to 450 us apart
// (5% of a full round), and at 3.4e7 candidates (a rank's share of c3 on
// 8 GPUs) the last block-wave another 6.5%.  Here a resident grid of blocks
// takes tiles from a counter until none are left, so faster XCDs take more;
// the last tiles are FR_CPT_TAIL candidates per thread (a quarter tile), so
// the blocks run out of work within a short tile of each other.  The
// tickets are exact -- ntiles + grid grabs per launch, one failing grab per
// block -- so the counter wraps back to zero at the last grab (atomicInc):
// no reset between launches.  Tile t covers the same candidates whichever
// block takes it; the accept bits do not depend on the schedule.
constexpr int FR_CPT_TAIL = 2;
constexpr int FR_TILE_TAIL = FR_T * FR_CPT_TAIL;

struct TilePlan {
  int64_t nbig, ntiles;        // full tiles first, then tail tiles
  unsigned int grid;
};
__host__ __device__ inline void tile_span(int64_t t, int64_t nbig, int64_t& tile0, int& cpt) {
  if (t < nbig) { tile0 = t * FR_TILE; cpt = FR_CPT; }
  else { tile0 = nbig * FR_TILE + (t - nbig) * FR_TILE_TAIL; cpt = FR_CPT_TAIL; }
}

template <int D, int MODE, bool FILTER, int PK>
__device__ __forceinline__ void round_body(RoundArgs A, int64_t idx0, int64_t B,
                                           double eps_host, uint64_t* __restrict__ bits,
                                           unsigned int* __restrict__ ticket,
                                           int64_t nbig, int64_t ntiles,
                                           double* __restrict__ rec_x) {
  // the threshold read on the device (the host's float(q) * multiplier, one
  // IEEE product either way)
  const double eps = A.eps_dev ? (*A.eps_dev) * A.eps_scale : eps_host;
  __shared__ BlockConsts C;
  __shared__ uint32_t tbits[FR_TILE / 32];
  __shared__ uint16_t queue[FR_TILE];
  __shared__ int qn;
  __shared__ int64_t s_tile;
  const TileLds T{tbits, queue, qn};
  stage_block_consts<D, MODE, true>(C, A.P, &A.M, A.box);
  if (FILTER) {
    if (threadIdx.x == 0) C.lazy = lazy_filter_ok<D, MODE>(C, A.P, A.M) ? 1 : 0;
  }
  const unsigned int limit = (unsigned int)(ntiles + gridDim.x - 1);
#pragma unroll 1
  for (;;) {
    if (threadIdx.x == 0) s_tile = (int64_t)atomicInc(ticket, limit);
    __syncthreads();
    const int64_t t = s_tile;
    if (t >= ntiles) break;            // block-uniform: one failing grab per block
    int64_t tile0;
    int cpt;
    tile_span(t, nbig, tile0, cpt);
    tile_body<D, MODE, FILTER, PK>(A, C, eps, idx0, B, tile0, cpt, bits, rec_x, T);
    __syncthreads();                   // s_tile and the tile's LDS are reused
  }
}

// The plain round's tile loop flattened into its candidate loop (one loop:
// a tile boundary is a block-uniform branch in it).  With the tile loop
// nested around the candidate loop the compiler keeps ~20 more VGPRs live
// (101 vs 80 at d = 10: 4 instead of 6 waves per SIMD).
template <int D, int MODE, int PK>
__device__ __forceinline__ void round_plain_body(RoundArgs A, int64_t idx0, int64_t B,
                                                 double eps_host, uint64_t* __restrict__ bits,
                                                 unsigned int* __restrict__ ticket,
                                                 int64_t nbig, int64_t ntiles,
                                                 double* __restrict__ rec_x) {
  const double eps = A.eps_dev ? (*A.eps_dev) * A.eps_scale : eps_host;
  constexpr int DM = D > 0 ? D : 64;
  __shared__ BlockConsts C;
  __shared__ uint32_t tbits[FR_TILE / 32];
  __shared__ int64_t s_tile;
  stage_block_consts<D, MODE, true>(C, A.P, &A.M, A.box);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned int limit = (unsigned int)(ntiles + gridDim.x - 1);
  int64_t tile0 = 0;
  int cpt = 0, it = 0;
  bool started = false;
#pragma unroll 1
  for (;;) {
    if (it == cpt) {                      // block-uniform: the tile is done
      __syncthreads();
      if (started && wave == 0 && lane < cpt * (FR_T / 64)) {
        const uint64_t w = (uint64_t)tbits[2 * lane] | ((uint64_t)tbits[2 * lane + 1] << 32);
        const int64_t word = tile0 / 64 + lane;
        if (word * 64 < B) bits[word] = w;
      }
      if (tid == 0) s_tile = (int64_t)atomicInc(ticket, limit);
      __syncthreads();                    // tbits read, s_tile written
      // the ticket into scalar registers (an LDS read is a per-lane value)
      const int64_t t = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(
                                       (int)(s_tile >> 32)) << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile));
      if (t >= ntiles) break;             // one failing grab per block
      tile_span(t, nbig, tile0, cpt);
      if (tid < FR_TILE / 32) tbits[tid] = 0u;
      __syncthreads();
      it = 0;
      started = true;
    }
    const int loc = it * FR_T + tid;
    const int64_t b = tile0 + loc;
    if (b < B) {
      double th[DM];
      int64_t j;
      int att;
      double* xr = rec_x ? rec_x + b * A.M.S : nullptr;
      const double dist = evaluate_full<D, MODE, PK>(A, C, (uint64_t)(idx0 + b), th, j, att, xr);
      if (dist <= eps) atomicOr(&tbits[loc >> 5], 1u << (loc & 31));
    }
    ++it;
  }
}

// Minimum waves per SIMD the compiler must allow (__launch_bounds__' second
// argument): the plain p = 2 round at d = 10 with a population (c2 / c3 / c5
// shapes) takes 100 VGPRs unconstrained (4 waves) but fits 80 (6 waves, as in
// round 5's one-tile-per-block kernel) without spilling; every other
// instantiation is left to the compiler (a bound there spills).
__host__ __device__ constexpr int fr_min_waves(bool filter, int D, int MODE, int PK) {
  return (!filter && PK == 2 && D == 10 && MODE != PROP_PRIOR) ? 6 : 1;
}

#define ABC_ROUND_KERNEL(NAME, FILTER, PK)                                                \
  template <int D, int MODE>                                                              \
  __global__ __launch_bounds__(FR_T, fr_min_waves(FILTER, D, MODE, PK))                   \
  void NAME(RoundArgs A, int64_t idx0, int64_t B,                                         \
                                               double eps, uint64_t* bits,                \
                                               unsigned int* ticket, int64_t nbig,        \
                                               int64_t ntiles, double* rec_x) {           \
    if (FILTER)                                                                           \
      round_body<D, MODE, true, PK>(A, idx0, B, eps, bits, ticket, nbig, ntiles, nullptr);\
    else                                                                                  \
      round_plain_body<D, MODE, PK>(A, idx0, B, eps, bits, ticket, nbig, ntiles, rec_x);  \
  }
ABC_ROUND_KERNEL(fused_round_plain, false, 0)
ABC_ROUND_KERNEL(fused_round_plain_p2, false, 2)
ABC_ROUND_KERNEL(fused_round_filter, true, 0)
ABC_ROUND_KERNEL(fused_round_filter_p2, true, 2)
#undef ABC_ROUND_KERNEL

// ---- accept words -> ordered positions -------------------------------------
// The accept words are cut into ranges of whole words (<= RG_MAX ranges);
// each range's accepted count goes to rtot[range], and bits_write_ranges
// (one wave per range) sums the counts of the ranges before its own --
// at most RG_MAX reads per wave, from L2 -- and writes the positions of its
// set bits; the wave of the last range writes the round's total.  One short
// launch after the producer when the producer is the plain round (it counts
// its own ranges), two otherwise; round 5 ran a three-kernel scan of
// per-tile counts and a per-word writer after it.
constexpr int RG_MAX = 2048;    // ranges at most
constexpr int RG_T = 256;

// range totals of accept words written by another kernel (the early-reject
// round, the user-model tail): one block per range of wpr words
__global__ __launch_bounds__(RG_T) void bits_range_sum_kernel(
    const uint64_t* __restrict__ bits, int64_t nwords, int64_t wpr,
    int64_t* __restrict__ rtot) {
  __shared__ int ws[RG_T / 64];
  const int64_t w0 = (int64_t)blockIdx.x * wpr;
  const int64_t w1 = w0 + wpr < nwords ? w0 + wpr : nwords;
  int c = 0;
  for (int64_t w = w0 + threadIdx.x; w < w1; w += RG_T) c += __popcll(bits[w]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t tot = 0;
    for (int q = 0; q < RG_T / 64; ++q) tot += ws[q];
    rtot[blockIdx.x] = tot;
  }
}

// One wave per range: its offset (the totals of the ranges before it), then
// the range's words loaded up front (WB per lane in flight) and taken 64 at
// a time -- popcount prefix across the lanes, the set bits' positions
// written while below cap.
constexpr int WB = 32;
__global__ __launch_bounds__(256) void bits_write_ranges(
    const uint64_t* __restrict__ bits, int64_t nwords, int64_t wpr, int nranges,
    const int64_t* __restrict__ rtot, int64_t cap, int64_t* __restrict__ idx,
    int64_t* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nranges) return;
  int64_t off = 0;
  for (int q = lane; q < r; q += 64) off += rtot[q];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) off += __shfl_xor(off, o, 64);
  const int64_t mine = rtot[r];
  if (r == nranges - 1 && lane == 0) *count = off + mine;
  if (off >= cap || mine == 0) return;    // wave-uniform
  const int64_t w0 = (int64_t)r * wpr;
  const int64_t w1 = w0 + wpr < nwords ? w0 + wpr : nwords;
  for (int64_t b0 = w0; b0 < w1 && off < cap; b0 += 64 * WB) {
    uint64_t w[WB];
#pragma unroll
    for (int q = 0; q < WB; ++q) {
      const int64_t wd = b0 + 64 * q + lane;
      w[q] = wd < w1 ? bits[wd] : 0ull;
    }
#pragma unroll
    for (int q = 0; q < WB; ++q) {
      if (b0 + 64 * q >= w1 || off >= cap) break;   // wave-uniform
      const int c = __popcll(w[q]);
      int incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
      }
      int64_t pos = off + (incl - c);
      uint64_t m = w[q];
      const int64_t wd = b0 + 64 * q + lane;
      while (m != 0ull && pos < cap) {
        idx[pos++] = wd * 64 + (__ffsll((long long)m) - 1);
        m &= m - 1;
      }
      off += __shfl(incl, 63, 64);
    }
  }
}

// one wave per dimension (support_bounds_wave): ~1 us instead of the ~40 us
// of one thread's 126 dependent bisection steps
__global__ __launch_bounds__(64) void support_box_kernel(const int32_t* __restrict__ kind,
                                                         const double* __restrict__ params,
                                                         int d, double* __restrict__ box) {
  const int k = blockIdx.x;
  if (k < d) support_bounds_wave(kind[k], params + 4 * k, box + 2 * k);
}

struct Ranges { int64_t nwords, wpr; int n; };
// nwords accept words in at most `most` ranges of at least `least` words
inline Ranges make_ranges(int64_t B, int64_t most, int64_t least) {
  Ranges r;
  r.nwords = ceil_div(B, 64);
  if (most > RG_MAX) most = RG_MAX;
  int64_t n = ceil_div(r.nwords, least);
  n = n < most ? n : most;
  n = n < 1 ? 1 : n;
  r.wpr = ceil_div(r.nwords, n);
  r.n = (int)ceil_div(r.nwords, r.wpr);
  return r;
}

// the round's tile schedule: full tiles, then tail tiles for about two
// resident block-waves; the grid is the resident capacity (at most one
// block per tile)
inline TilePlan plan_tiles(int64_t B, int resident) {
  TilePlan p;
  const int64_t tail = 2 * (int64_t)resident * FR_TILE_TAIL;
  p.nbig = B > tail ? (B - tail) / FR_TILE : 0;
  p.ntiles = p.nbig + ceil_div(B - p.nbig * FR_TILE, FR_TILE_TAIL);
  p.grid = (unsigned int)(p.ntiles < resident ? p.ntiles : resident);
  return p;
}

template <int D, int MODE>
void launch_round(bool filt, bool p2, const RoundArgs& A, int64_t idx0, int64_t B, double eps,
                  uint64_t* bits, unsigned int* ticket, double* rec_x, hipStream_t s) {
  auto k = filt ? (p2 ? fused_round_filter_p2<D, MODE> : fused_round_filter<D, MODE>)
                : (p2 ? fused_round_plain_p2<D, MODE> : fused_round_plain<D, MODE>);
  const TilePlan p = plan_tiles(B, resident_blocks(k, FR_T));
  hipLaunchKernelGGL(k, dim3(p.grid), dim3(FR_T), 0, s, A, idx0, B, eps, bits, ticket, p.nbig,
                     p.ntiles, rec_x);
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

// ---- the multi-rank cutoff on the device -------------------------------------
// keep[0] = how many of this rank's accepted candidates the round keeps: the
// first `need` accepted in global order (ranks in order), counts gathered
// from every rank (dd.cutoff on the host computes the same numbers)
__global__ void round_keep_kernel(const int64_t* __restrict__ counts, int rank, int64_t need,
                                  int64_t* __restrict__ keep) {
  if (threadIdx.x != 0) return;
  int64_t left = need > 0 ? need : 0, k = 0;
  for (int q = 0; q <= rank; ++q) {
    const int64_t c = counts[q] > 0 ? counts[q] : 0;
    const int64_t take = c < left ? c : left;
    if (q == rank) k = take;
    left -= take;
  }
  *keep = k;
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
    int max_attempts, uint64_t* __restrict__ bits) {
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
  if (wave == 0 && lane < FR_WORDS) {
    const uint64_t w = (uint64_t)tbits[2 * lane] | ((uint64_t)tbits[2 * lane + 1] << 32);
    const int64_t word = tile0 / 64 + lane;
    if (word * 64 < B) bits[word] = w;
  }
}

// *count and the positions of the first cap accepted from the range totals
int write_ranges(const uint64_t* bits, const Ranges& rg, const int64_t* rtot, int64_t cap,
                 int64_t* idx, int64_t* count, hipStream_t s) {
  hipLaunchKernelGGL(bits_write_ranges, dim3((unsigned)ceil_div(rg.n, 4)), dim3(256), 0, s,
                     bits, rg.nwords, rg.wpr, rg.n, rtot, cap, idx, count);
  ABC_LAUNCHED();
  return ABC_OK;
}

// accept words written by another kernel -> *count and the first cap
// positions (range sums, then the writer)
int compact_accept_bits(const uint64_t* bits, int64_t* rtot, int64_t B, int64_t cap,
                        int64_t* idx, int64_t* count, hipStream_t s) {
  const Ranges rg = make_ranges(B, RG_MAX, RG_T);
  hipLaunchKernelGGL(bits_range_sum_kernel, dim3((unsigned)rg.n), dim3(RG_T), 0, s, bits,
                     rg.nwords, rg.wpr, rtot);
  ABC_LAUNCHED();
  return write_ranges(bits, rg, rtot, cap, idx, count, s);
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

// the same dispatch for a host launcher template FN<D, MODE>(args...)
#define ABC_FUSED_CALL(FN, ...)                                                \
  do {                                                                         \
    const int mode_ = spec->X == nullptr ? PROP_PRIOR                          \
                      : (spec->per_particle_L ? PROP_LOCAL : PROP_MVN);        \
    switch (spec->d) {                                                         \
      ABC_FUSED_CALL_CASE(FN, 1, __VA_ARGS__)                                  \
      ABC_FUSED_CALL_CASE(FN, 2, __VA_ARGS__)                                  \
      ABC_FUSED_CALL_CASE(FN, 3, __VA_ARGS__)                                  \
      ABC_FUSED_CALL_CASE(FN, 4, __VA_ARGS__)                                  \
      ABC_FUSED_CALL_CASE(FN, 5, __VA_ARGS__)                                  \
      ABC_FUSED_CALL_CASE(FN, 6, __VA_ARGS__)                                  \
      ABC_FUSED_CALL_CASE(FN, 8, __VA_ARGS__)                                  \
      ABC_FUSED_CALL_CASE(FN, 10, __VA_ARGS__)                                 \
      ABC_FUSED_CALL_CASE(FN, 12, __VA_ARGS__)                                 \
      ABC_FUSED_CALL_CASE(FN, 16, __VA_ARGS__)                                 \
      default:                                                                 \
        ABC_FUSED_CALL_BODY(FN, 0, __VA_ARGS__)                                \
    }                                                                          \
  } while (0)
#define ABC_FUSED_CALL_BODY(FN, DD, ...)                                       \
  if (mode_ == PROP_MVN) FN<DD, PROP_MVN>(__VA_ARGS__);                        \
  else if (mode_ == PROP_LOCAL) FN<DD, PROP_LOCAL>(__VA_ARGS__);               \
  else FN<DD, PROP_PRIOR>(__VA_ARGS__);                                        \
  break;
#define ABC_FUSED_CALL_CASE(FN, DD, ...)                                       \
  case DD: { ABC_FUSED_CALL_BODY(FN, DD, __VA_ARGS__) }

}  // namespace
}  // namespace abc

using namespace abc;

// workspace: tile ticket (zero before the first call; every round leaves it
// zero) | range totals | prior support box | accept bits
struct RoundWs {
  unsigned int* ticket; int64_t* rtot; double* box; uint64_t* bits; bool ok;
};
inline RoundWs carve_round_ws(void* ws, size_t ws_bytes, int64_t B) {
  Carver c(ws, ws_bytes);
  RoundWs w;
  w.ticket = c.take<unsigned int>(64);
  w.rtot = c.take<int64_t>(RG_MAX);
  w.box = c.take<double>(128);
  w.bits = c.take<uint64_t>((size_t)ceil_div(B > 0 ? B : 1, FR_TILE) * FR_WORDS);
  w.ok = c.ok;
  return w;
}

extern "C" size_t abc_candidates_workspace(int64_t B) {
  size_t off = 0;
  size_only<unsigned int>(off, 64);
  size_only<int64_t>(off, RG_MAX);
  size_only<double>(off, 128);
  size_only<uint64_t>(off, (size_t)ceil_div(B > 0 ? B : 1, FR_TILE) * FR_WORDS);
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
  ABC_CHECK_ARG(nt < (1ll << 31), "candidates_round: too many tiles");
  const RoundWs w = carve_round_ws(ws, ws_bytes, B);
  if (!w.ok) return set_error(ABC_ERR_WORKSPACE, "candidates_round: workspace");
  const double* box = spec->support_box;
  if (!box) {
    hipLaunchKernelGGL(support_box_kernel, dim3((unsigned)spec->d), dim3(64), 0, s,
                       spec->prior_kind, spec->prior_params, spec->d, w.box);
    ABC_LAUNCHED();
    box = w.box;
  }
  RoundArgs A = round_args(spec, box);
  A.eps_dev = eps_dev;
  A.eps_scale = eps_scale;
  profile_start(s, ABC_PROF_CANDIDATES);
  ABC_FUSED_CALL(launch_round, filt != 0, p == 2.0, A, idx0, B, eps, w.bits, w.ticket, rec_x, s);
  profile_stop(s, ABC_PROF_CANDIDATES);
  ABC_LAUNCHED();
  return compact_accept_bits(w.bits, w.rtot, B, cap, idx, count, s);
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
  const RoundWs w = carve_round_ws(ws, ws_bytes, B);
  if (!w.ok) return set_error(ABC_ERR_WORKSPACE, "pnorm_accept: workspace");
  uint64_t* bits = w.bits;
  // the same row / wave split as abc_pnorm (the same bits per row)
  if (S <= 32)
    hipLaunchKernelGGL(pnorm_accept_kernel<false>, dim3((unsigned)nt), dim3(FR_T),
                       (size_t)pa_chunk_rows(S) * (S + 1) * sizeof(double), s, x, B, S, x0, wf, p, eps,
                       attempts, max_attempts, bits);
  else
    hipLaunchKernelGGL(pnorm_accept_kernel<true>, dim3((unsigned)nt), dim3(FR_T), 0, s, x, B,
                       S, x0, wf, p, eps, attempts, max_attempts, bits);
  ABC_LAUNCHED();
  return compact_accept_bits(bits, w.rtot, B, cap, idx, count, s);
}

extern "C" int abc_prior_support_box(const int32_t* prior_kind, const double* prior_params,
                                     int d, double* box, void* stream) {
  ABC_CHECK_ARG(d >= 1 && d <= 64, "prior_support_box: bad d");
  ABC_CHECK_ARG(prior_kind && prior_params && box, "prior_support_box: null pointer");
  hipLaunchKernelGGL(support_box_kernel, dim3((unsigned)d), dim3(64), 0, as_stream(stream),
                     prior_kind, prior_params, d, box);
  ABC_LAUNCHED();
  return ABC_OK;
}

extern "C" int abc_round_keep(const int64_t* counts, int nranks, int rank, int64_t need,
                              int64_t* keep, void* stream) {
  ABC_CHECK_ARG(counts && keep && nranks >= 1 && rank >= 0 && rank < nranks,
                "round_keep: bad arguments");
  hipLaunchKernelGGL(round_keep_kernel, dim3(1), dim3(64), 0, as_stream(stream), counts, rank,
                     need, keep);
  ABC_LAUNCHED();
  return ABC_OK;
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
  if (spec->support_box) {
    box = const_cast<double*>(spec->support_box);
  } else {
    hipLaunchKernelGGL(support_box_kernel, dim3((unsigned)spec->d), dim3(64), 0, s,
                       spec->prior_kind, spec->prior_params, spec->d, box);
    ABC_LAUNCHED();
  }
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
