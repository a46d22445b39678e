// Dense-neighbourhood moments of the LocalTransition fit (k a sizeable
// fraction of N, the default k = N/4) on f16 MFMA, fed by fp32 expanded-form
// keys (included by abc_local.hip after mm_finish_kernel; the membership
// bound is abc_local_knn.h's kn_bound).
//
// Reference: pyabc/transition/local_transition.py:125-139 (weighted
// covariance of the k neighbours' offsets).
//
// The raw sums S_n,f = sum_j m_nj F_j,f are the [particles x rows] x [rows x
// features] product of mm_moments_kernel (same exact 11-bit limb image of
// F, same fp64 flushes, same mm_finish_kernel), with two changes that
// matter at k = N/4, where every row of every wave has members:
//  * the membership key is the k-NN select's s^ = n^_j + n^_n - 2 y^_j . y^_n
//    on the same centred fp32 features, formed by v_mfma_f32_16x16x4_f32
//    (the select's k-ordered chain, so kn_bound covers it) from a row
//    fragment image in the step's k-slot order: 2 x KB MFMAs per 32-row step
//    where the VALU spent D fma + 1 add per pair (round 5: 21.6 VALU
//    lane-instructions per pair); the keys are decided against the fp32 cuts
//    of v* and settled exactly in fp64 between them;
//  * both operand streams reach LDS by global_load_lds (16 B per lane, no
//    staging registers), double-buffered per DM_SB 32-row steps, so the
//    wave's registers go to its 2 x 7 accumulator tiles.
constexpr int DM_W = 4;                    // waves per block
constexpr int DM_G = 1;                    // particle tiles per wave
constexpr int DM_T = DM_W * 64;
constexpr int DM_PB = DM_W * DM_G * 16;    // particles per block
constexpr int DM_SB = 2;                   // 32-row steps per LDS stage
// Row fragments of one 32-row step: 2 tiles h x KB k-blocks x 64 lanes
// (floats); lane l of (h, kb) holds feature 4 kb + (l >> 4) of the step's
// row dm_row(h, l & 15), features [y^ (D), n^, 1, 0...] (rows >= N: n^ =
// +inf, the rest 0).  The MFMA returns tile h's keys at lane l for rows
// dm_row(h, 4 (l >> 4) + r), r < 4 -- with dm_row(h, i) = 8 (i >> 2) +
// (i & 3) + 4 h those are rows 8 (l >> 4) + 4 h + r: the k-slots of the
// moments MFMA's A fragment (lane l: rows 8 (l >> 4) + u, u < 8), so the
// keys become the fragment without a lane exchange.  Reads are one float per
// lane at consecutive addresses (no bank conflicts).
template <int D> constexpr int dm_rstep() { return 2 * kn_kb<D>() * 64; }
__host__ __device__ constexpr int dm_row(int h, int i) { return 8 * (i >> 2) + (i & 3) + 4 * h; }

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)g,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// the row fragment image (one thread per row; rows past N key +inf)
template <int D>
__global__ __launch_bounds__(256) void knn_rows_kernel(const double* __restrict__ X, int64_t N,
                                                       int64_t nrows,
                                                       const double* __restrict__ cen,
                                                       float* __restrict__ rows) {
  constexpr int KB = kn_kb<D>();
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= nrows) return;
  const int r = (int)(j & 31);
  const int h = (r >> 2) & 1, i = 4 * (r >> 3) + (r & 3);   // dm_row(h, i) == r
  float* dst = rows + (j >> 5) * dm_rstep<D>() + h * KB * 64 + i;
  float f[4 * KB];
#pragma unroll
  for (int k = 0; k < 4 * KB; ++k) f[k] = 0.0f;
  if (j < N) {
    float y[D];
    const float n = kn_feat<D>(X, j, cen, y);
#pragma unroll
    for (int q = 0; q < D; ++q) f[q] = y[q];
    f[D] = n;
    f[D + 1] = 1.0f;
  } else {
    f[D] = INFINITY;
  }
#pragma unroll
  for (int k = 0; k < 4 * KB; ++k) dst[(k >> 2) * 64 + 16 * (k & 3)] = f[k];
}

// DEFER (the deferred collect, see knn_select_kernel): sel_v / sel_jcut hold
// the bracket [T_lo, T_hi) of the rank-k key as doubles instead of the
// selected key; pairs certainly below T_lo are members (and counted into
// cbelow), pairs between the cuts are not summed here but queued (qcnt,
// qidx: KN_QCAP per particle) for knn_resolve_kernel, which selects the rank
// among them and adds the members' limbs.  Queue slots come from an LDS
// queue per block (DQ_L per particle), flushed to the global queue at the
// end with one atomic per particle; a full LDS queue spills by global atomics.
constexpr int DQ_L = 16;
template <int D, bool DEFER>
__global__ __launch_bounds__(DM_T) void knn_dense_kernel(
    const double* __restrict__ X, const double* __restrict__ cen,
    const double* __restrict__ R2p, const float* __restrict__ rows,
    const half8* __restrict__ img, int64_t N, int64_t nsteps,
    const unsigned long long* __restrict__ sel_v, const long long* __restrict__ sel_jcut,
    const long long* __restrict__ sel_rank0, double* __restrict__ part,
    int* __restrict__ qcnt, int* __restrict__ qidx, int* __restrict__ cbelow) {
  constexpr int KB = kn_kb<D>();
  constexpr int RSTEP = dm_rstep<D>();
  constexpr int NT = mm_nt<D>(), NCP = 16 * NT;
  constexpr int BP = DM_SB * NT * 64;              // B pieces (16 B) per stage
  constexpr int RP = DM_SB * RSTEP / 4;            // row pieces per stage
  constexpr int SP = BP + RP;
  static_assert(BP % 64 == 0 && RSTEP % 4 == 0, "B stream: whole wave-instructions");
  constexpr int PW = ((SP + 63) / 64 + DM_W - 1) / DM_W;  // wave-instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char stage[2][SP * 16];
  __shared__ int s_qn[DEFER ? DM_PB : 1], s_q[DEFER ? DM_PB * DQ_L : 1];
  if constexpr (DEFER) {
    for (int e = threadIdx.x; e < DM_PB; e += DM_T) s_qn[e] = 0;
    // (the first stage's barrier orders these stores before any queue use)
  }
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int RS = gridDim.y;
  const int64_t s0 = (nsteps * (int64_t)blockIdx.y) / RS;
  const int64_t s1 = (nsteps * ((int64_t)blockIdx.y + 1)) / RS;
  const int64_t p0 = ((int64_t)blockIdx.x * DM_W + wv) * (DM_G * 16);
  const int kq = lane >> 4;
  const KnBound Bd = kn_bound<D>(*R2p);
  const float zc = kn_cut_above(0.0, Bd);

  // the lane's particle in each tile: its key features (the B operand of
  // the key MFMA: feature 4 kb + (lane >> 4) of [-2 y^_n, 1, n^_n]) and the
  // fp32 cuts of v*
  float bfr[DM_G][KB], cin[DM_G], cout[DM_G];
#pragma unroll
  for (int g = 0; g < DM_G; ++g) {
    const int64_t pn = p0 + 16 * g + (lane & 15);
    const int64_t pe = pn < N ? pn : N - 1;
    float y[D];
    const float nn = kn_feat<D>(X, pe, cen, y);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int k = 4 * kb + (lane >> 4);
      float v = 0.0f;
#pragma unroll
      for (int q = 0; q < D; ++q) if (k == q) v = -2.0f * y[q];
      if (k == D) v = 1.0f;
      if (k == D + 1) v = nn;
      bfr[g][kb] = v;
    }
    if constexpr (DEFER) {
      cin[g] = kn_cut_below(__longlong_as_double((long long)sel_v[pe]), Bd);
      cout[g] = kn_cut_above(__longlong_as_double(sel_jcut[pe]), Bd);
    } else {
      const double v = key_val(sel_v[pe]);
      cin[g] = kn_cut_below(v, Bd);
      cout[g] = kn_cut_above(v, Bd);
    }
  }
  uint32_t nin[DM_G];   // DEFER: certain members counted per lane
#pragma unroll
  for (int g = 0; g < DM_G; ++g) nin[g] = 0u;
  f32x4 acc[DM_G][NT];
#pragma unroll
  for (int g = 0; g < DM_G; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool first = true;
  int since = 0;
  auto flush = [&]() {
#pragma unroll
    for (int g = 0; g < DM_G; ++g)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int c = 16 * t + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t n = p0 + 16 * g + 4 * kq + r;
          if (n < N) {
            double* dst = part + ((int64_t)blockIdx.y * NCP + c) * N + n;
            *dst = (first ? 0.0 : *dst) + (double)acc[g][t][r];
          }
        }
        acc[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    first = false;
    since = 0;
  };
  // one stage: the B image of DM_SB steps, then their rows (both streams
  // padded by DM_SB steps past nsteps, so a partial last stage loads safely)
  auto issue = [&](int buf, int64_t sb) {
    const char* bsrc = reinterpret_cast<const char*>(img + sb * NT * 64);
    const char* rsrc = reinterpret_cast<const char*>(rows + sb * RSTEP);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int wi = wv * PW + i;              // wave-instruction index (uniform)
      const int e = wi * 64 + lane;
      if (e < SP) {                            // the rows' last instruction is partial
        const char* src = e < BP ? bsrc + (size_t)e * 16 : rsrc + (size_t)(e - BP) * 16;
        glds16(src, &stage[buf][(size_t)wi * 64 * 16]);
      }
    }
  };
  if (s0 < s1) issue(0, s0);
  int buf = 0;
  for (int64_t sb = s0; sb < s1; sb += DM_SB, buf ^= 1) {
    __syncthreads();                 // stage sb landed (vmcnt(0) + barrier); buf ^ 1 free
    if (sb + DM_SB < s1) issue(buf ^ 1, sb + DM_SB);
    const half8* bs = reinterpret_cast<const half8*>(&stage[buf][0]);
    const float* rs = reinterpret_cast<const float*>(&stage[buf][(size_t)BP * 16]);
    const int nk = (int)((s1 - sb) < DM_SB ? (s1 - sb) : DM_SB);
    for (int k = 0; k < nk; ++k) {
      half8 a[DM_G];
      uint32_t openm = 0u, inm = 0u;   // bit 8 g + u: pair (tile g, row 8 kq + u)
      // the step's keys: tile h gives rows 8 kq + 4 h + r (r < 4)
      const float* rf = rs + k * RSTEP + lane;
      float af[2][KB];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) af[h][kb] = rf[(h * KB + kb) * 64];
#pragma unroll
      for (int g = 0; g < DM_G; ++g) {
        knf4 c[2] = {knf4{0.f, 0.f, 0.f, 0.f}, knf4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            c[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[h][kb], bfr[g][kb], c[h], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float sk = c[u >> 2][u & 3];
          const bool in = sk < cin[g] && sk > zc;
          openm |= (!in && !(sk > cout[g])) ? (1u << (8 * g + u)) : 0u;
          inm |= in ? (1u << (8 * g + u)) : 0u;
        }
      }
#pragma unroll
      for (int g = 0; g < DM_G; ++g)
#pragma unroll
        for (int u = 0; u < 8; ++u)
          a[g][u] = ((inm >> (8 * g + u)) & 1u) ? (_Float16)1.0f : (_Float16)0.0f;
      if constexpr (DEFER) {
#pragma unroll
        for (int g = 0; g < DM_G; ++g) nin[g] += __builtin_popcount((inm >> (8 * g)) & 0xFFu);
      }
      if (DEFER && __builtin_amdgcn_ballot_w64(openm != 0u) != 0ull) {
        // queue the open pairs (their a stays 0): one LDS atomic per lane
        // reserves its slots
#pragma unroll
        for (int g = 0; g < DM_G; ++g) {
          const int64_t pn = p0 + 16 * g + (lane & 15);
          const int pl = (wv * DM_G + g) * 16 + (lane & 15);
          const int64_t jb = 32 * (sb + k) + 8 * kq;
          uint32_t om = (openm >> (8 * g)) & 0xFFu;
          if (jb + 8 > N) om &= N > jb ? (1u << (uint32_t)(N - jb)) - 1u : 0u;
          if (pn >= N) om = 0u;
          if (om) {
            int slot = atomicAdd(&s_qn[pl], __builtin_popcount(om));
            while (om) {
              const int j = (int)jb + __builtin_ctz(om);
              om &= om - 1u;
              if (slot < DQ_L) {
                s_q[pl * DQ_L + slot] = j;
              } else {
                const int gs = atomicAdd(&qcnt[pn], 1);
                if (gs < KN_QCAP) qidx[pn * KN_QCAP + gs] = j;
              }
              ++slot;
            }
          }
        }
      } else if (!DEFER && __builtin_amdgcn_ballot_w64(openm != 0u) != 0ull) {
        // rare: settle the open pairs in fp64 (rank-0 row excluded)
#pragma unroll
        for (int g = 0; g < DM_G; ++g) {
          if (!((openm >> (8 * g)) & 0xFFu)) continue;
          const int64_t pn = p0 + 16 * g + (lane & 15);
          const int64_t pe = pn < N ? pn : N - 1;
          double xp[D];
#pragma unroll
          for (int q = 0; q < D; ++q) xp[q] = X[pe * D + q];
          const unsigned long long vs = sel_v[pe];
          const long long jc = sel_jcut[pe], r0 = sel_rank0[pe];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int64_t j = 32 * (sb + k) + 8 * kq + u;
            if (!((openm >> (8 * g + u)) & 1u) || j >= N) continue;
            const unsigned long long key = (unsigned long long)__double_as_longlong(dist2<D>(X, j, xp));
            const bool member = (key < vs || (key == vs && j < jc)) && j != r0;
            a[g][u] = member ? (_Float16)1.0f : (_Float16)0.0f;
          }
        }
      }
      const half8* b = bs + k * NT * 64 + lane;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const half8 bt = b[t * 64];
#pragma unroll
        for (int g = 0; g < DM_G; ++g)
          acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[g], bt, acc[g][t], 0, 0, 0);
      }
      if (++since == MM_FLUSH) flush();
    }
  }
  if (since > 0 || first) flush();
  if constexpr (DEFER) {
#pragma unroll
    for (int g = 0; g < DM_G; ++g) {
      uint32_t c = nin[g];
      c += __shfl_xor(c, 16, 64);
      c += __shfl_xor(c, 32, 64);
      const int64_t pn = p0 + 16 * g + (lane & 15);
      if (lane < 16 && pn < N && c) atomicAdd(&cbelow[pn], (int)c);
    }
    __syncthreads();   // every wave's LDS queue entries are in
    for (int pl = threadIdx.x; pl < DM_PB; pl += DM_T) {
      const int64_t pn = (int64_t)blockIdx.x * DM_PB + pl;
      const int m = s_qn[pl] < DQ_L ? s_qn[pl] : DQ_L;
      if (pn >= N || m == 0) continue;
      const int base = atomicAdd(&qcnt[pn], m);
      for (int i = 0; i < m; ++i)
        if (base + i < KN_QCAP) qidx[pn * KN_QCAP + base + i] = s_q[pl * DQ_L + i];
    }
  }
}

// The deferred collect's settle step, one wave per particle: the queued open
// pairs get their exact fp64 keys; those below T_lo join the certain-below
// count, those in [T_lo, T_hi) are ranked in (key, index) order, and rank
// nq - 1 - #below is the selected neighbour (as in knn_select_kernel's
// steps 3-4).  The members among the queue (below T_lo, or ranked at most
// the selected one; the rank-0 row excluded) are put in index order -- the
// queue's order comes from atomics, index order makes the sum deterministic
// -- and lanes 0..NM-1 each sum one fp64 moment feature over them into
// `extra` (mm_finish_kernel adds it to the limb sums of the certain members).
// A particle flagged by the select, with an overflowing queue or with the
// rank outside the kept set counts into nfail (the host then reruns the fit
// with the in-kernel collect).  Queueing in knn_dense_kernel reserves a
// lane's slots with one LDS atomic (popcount of its open pairs).
template <int D>
__global__ __launch_bounds__(256) void knn_resolve_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t N, int64_t nq,
    const int* __restrict__ need, unsigned long long* __restrict__ sel_v,
    long long* __restrict__ sel_jcut, long long* __restrict__ sel_rank0,
    const int* __restrict__ qcnt, const int* __restrict__ qidx,
    const int* __restrict__ cbelow, const double* __restrict__ bnd,
    double* __restrict__ part, double* __restrict__ extra, int* __restrict__ nfail) {
  constexpr int E = KN_QCAP / 64;
  constexpr int NC = mm_nc<D>();
  constexpr int CPL = (NC + 63) / 64;
  __shared__ double s_key[4][KN_QCAP];
  __shared__ int s_idx[4][KN_QCAP];
  __shared__ int s_ord[4][KN_QCAP];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 4 + wv;
  const bool live = n < N;
  const int64_t ne = live ? n : N - 1;
  const int cnt = qcnt[ne];
  bool ok = live && !need[ne] && cnt <= KN_QCAP;
  const double tlo = __longlong_as_double((long long)sel_v[ne]);
  const double thi = __longlong_as_double(sel_jcut[ne]);
  double xn[D];
#pragma unroll
  for (int q = 0; q < D; ++q) xn[q] = X[ne * D + q];
  double key[E], s64[E];
  int jj[E];
  int nbelow = 0, nkeep = 0, r0 = 0x7FFFFFFF;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int q = lane + 64 * i;
    jj[i] = (ok && q < cnt) ? qidx[ne * KN_QCAP + q] : -1;
    s64[i] = INFINITY;
    key[i] = INFINITY;
    if (jj[i] >= 0) {
      s64[i] = dist2<D>(X, jj[i], xn);
      if (s64[i] == 0.0) r0 = min(r0, jj[i]);
      if (s64[i] < tlo) ++nbelow;
      else if (s64[i] < thi) { key[i] = s64[i]; ++nkeep; }
    }
    if (q < KN_QCAP) { s_key[wv][q] = key[i]; s_idx[wv][q] = jj[i]; }
  }
  __syncthreads();
  int less[E];
#pragma unroll
  for (int i = 0; i < E; ++i) less[i] = 0;
  if (ok)
    for (int f = 0; f < cnt; ++f) {
      const double kf = s_key[wv][f];
      const int jf = s_idx[wv][f];
#pragma unroll
      for (int i = 0; i < E; ++i) less[i] += (kf < key[i]) || (kf == key[i] && jf < jj[i]);
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nbelow += __shfl_xor(nbelow, o, 64);
    nkeep += __shfl_xor(nkeep, o, 64);
    r0 = min(r0, __shfl_xor(r0, o, 64));
  }
  const long long rr = nq - 1 - ((long long)cbelow[ne] + nbelow);
  if (!(rr >= 0 && rr < nkeep)) ok = false;
  const long long r0l = r0 == 0x7FFFFFFF ? (long long)N : (long long)r0;
  bool mem[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const bool kept = key[i] < INFINITY;
    mem[i] = ok && jj[i] >= 0 && (long long)jj[i] != r0l &&
             (s64[i] < tlo || (kept && less[i] <= rr));
    if (ok && kept && less[i] == rr) {
      sel_v[n] = (unsigned long long)__double_as_longlong(s64[i]);
      sel_jcut[n] = (long long)jj[i] + 1;
      sel_rank0[n] = r0l;
    }
  }
  if (live && !ok && lane == 0) atomicAdd(nfail, 1);
  // members in index order (a deterministic summation order: the queue's
  // order comes from atomics), their NM features summed in fp64 into extra
  // (mm_finish_kernel adds it to the limb sums)
  __syncthreads();                       // the ranking's LDS reads are done
#pragma unroll
  for (int i = 0; i < E; ++i) s_idx[wv][lane + 64 * i] = mem[i] ? jj[i] : 0x7FFFFFFF;
  __syncthreads();
  int pos[E], nmem = 0;
#pragma unroll
  for (int i = 0; i < E; ++i) { pos[i] = 0; nmem += mem[i] ? 1 : 0; }
  if (ok)
    for (int f = 0; f < cnt; ++f) {
      const int jf = s_idx[wv][f];
#pragma unroll
      for (int i = 0; i < E; ++i) pos[i] += jf < jj[i] ? 1 : 0;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nmem += __shfl_xor(nmem, o, 64);
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (mem[i]) s_ord[wv][pos[i]] = jj[i];
  __syncthreads();
  constexpr int NM = local_nm<D>();
  double sum = 0.0, sabs = 0.0;
  if (ok && lane < NM)
    for (int q = 0; q < nmem; ++q) {
      const int j = s_ord[wv][q];
      double y[D];
#pragma unroll
      for (int a = 0; a < D; ++a) y[a] = X[(int64_t)j * D + a] - X[a];
      const double f = mm_feature<D>(lane, w[j], y);
      sum += f;
      sabs += fabs(f);
    }
  // the sum and its rounding bound: a sequential fp64 sum of nmem terms is
  // off by at most (nmem - 1) u sum |f| (mm_finish_kernel adds eps x this)
  if (ok && lane < NM) {
    extra[(int64_t)lane * N + n] = sum;
    extra[(int64_t)(NM + lane) * N + n] = (double)nmem * sabs;
  }
  (void)bnd; (void)part;
}
