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
//  * the membership key is s^ = n^_n + sum_q y^_jq (-2 y^_nq) + n^_j on the
//    centred fp32 rows of knn_prep_kernel (D fma + 1 add per pair instead of
//    D sub + D fma; any evaluation order is inside kn_bound), decided
//    against the fp32 cuts of v* and settled exactly in fp64 between them;
//  * both operand streams reach LDS by global_load_lds (16 B per lane, no
//    staging registers), double-buffered per DM_SB 32-row steps, so the
//    wave's registers go to its 2 x 7 accumulator tiles.
constexpr int DM_W = 4;                    // waves per block
constexpr int DM_G = 1;                    // particle tiles per wave
constexpr int DM_T = DM_W * 64;
constexpr int DM_PB = DM_W * DM_G * 16;    // particles per block
constexpr int DM_SB = 2;                   // 32-row steps per LDS stage
constexpr int DM_ROWF = 8;                 // floats per staged row: y^ (D <= 7), n^
// rows image: per 32-row step 32 rows of DM_ROWF floats with 4 pad floats
// after every 8 rows, so the 4 lane groups (rows 8 kq + u) read 4 different
// bank quads of the staged copy (unpadded, the rows lay 64 words apart: one
// bank quad, a 4-way conflict on every row read)
constexpr int DM_RSTEP = 32 * DM_ROWF + 16;     // floats per 32-row step
__host__ __device__ constexpr int dm_row_off(int r) { return r * DM_ROWF + (r >> 3) * 4; }

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)g,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// rows [y^_0 .. y^_{D-1}, n^, 0...] per row (rows >= N: n^ = +inf, key +inf)
template <int D>
__global__ __launch_bounds__(256) void knn_rows_kernel(const double* __restrict__ X, int64_t N,
                                                       int64_t nrows,
                                                       const double* __restrict__ cen,
                                                       float* __restrict__ rows) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= nrows) return;
  float* dst = rows + (j >> 5) * DM_RSTEP + dm_row_off((int)(j & 31));
  float f[DM_ROWF];
#pragma unroll
  for (int k = 0; k < DM_ROWF; ++k) f[k] = 0.0f;
  if (j < N) {
    float y[D];
    const float n = kn_feat<D>(X, j, cen, y);
#pragma unroll
    for (int q = 0; q < D; ++q) f[q] = y[q];
    f[D] = n;
  } else {
    f[D] = INFINITY;
  }
#pragma unroll
  for (int k = 0; k < DM_ROWF; ++k) dst[k] = f[k];
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
  static_assert(D + 1 <= DM_ROWF, "staged row holds y^ and n^");
  constexpr int NT = mm_nt<D>(), NCP = 16 * NT;
  constexpr int BP = DM_SB * NT * 64;              // B pieces (16 B) per stage
  constexpr int RP = DM_SB * DM_RSTEP / 4;         // row pieces per stage
  constexpr int SP = BP + RP;
  static_assert(BP % 64 == 0 && DM_RSTEP % 4 == 0, "B stream: whole wave-instructions");
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

  // the lane's particle in each tile: -2 y^_n, n^_n and the fp32 cuts of v*
  float m2y[DM_G][D], nn[DM_G], cin[DM_G], cout[DM_G];
#pragma unroll
  for (int g = 0; g < DM_G; ++g) {
    const int64_t pn = p0 + 16 * g + (lane & 15);
    const int64_t pe = pn < N ? pn : N - 1;
    float y[D];
    nn[g] = kn_feat<D>(X, pe, cen, y);
#pragma unroll
    for (int q = 0; q < D; ++q) m2y[g][q] = -2.0f * y[q];
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
    const char* rsrc = reinterpret_cast<const char*>(rows + sb * DM_RSTEP);
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
      uint32_t openm = 0u, inm = 0u;   // bit 8 g + u: pair (tile g, row u)
      // rows one at a time (not unrolled: the 8 rows' features would
      // otherwise be loaded up front and cost the occupancy)
#pragma unroll 2
      for (int u = 0; u < 8; ++u) {
        const float* rf = rs + k * DM_RSTEP + dm_row_off(8 * kq + u);
        const f32x4 r0 = *reinterpret_cast<const f32x4*>(rf);
        const f32x4 r1 = *reinterpret_cast<const f32x4*>(rf + 4);
        float y[8] = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
#pragma unroll
        for (int g = 0; g < DM_G; ++g) {
          float sk = nn[g];
#pragma unroll
          for (int q = 0; q < D; ++q) sk = __builtin_fmaf(y[q], m2y[g][q], sk);
          sk += y[D];
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
