/*
 * libabcgpu -- C ABI of the MI355X (gfx950) batched ABC-SMC generation engine.
 *
 * Drop-in boundary for pyABC 0.10.5's hot path.  pyABC has no FFI of its own
 * (it is pure Python); these entry points are what its plugin
 * classes bind through ctypes (INTEGRATION.md shows the binding).  Each group
 * cites the reference interface it replaces.
 *
 * Conventions
 *   - Every pointer is DEVICE memory owned by the caller (torch tensors in the
 *     Python layer), except where a parameter says "host".
 *   - Parameters are row-major [rows x d] float64, columns in the reference's
 *     order (sorted parameter names, pyabc/storage/history.py:307); summary
 *     statistics in x_0 key order (pyabc/distance/distance.py:113-125).
 *   - `stream` is a hipStream_t (NULL = default stream).  Calls are
 *     stream-ordered and asynchronous unless stated; nothing allocates device
 *     memory inside a call: scratch comes from a caller workspace whose size
 *     the matching *_workspace() query returns.
 *   - Return 0 on success, a negative ABC_ERR_* code otherwise; the message is
 *     in abc_last_error() (thread-local).  No C++ exception crosses the ABI.
 */
#ifndef ABCGPU_H
#define ABCGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ABC_OK 0
#define ABC_ERR_INVALID (-1)
#define ABC_ERR_HIP (-2)
#define ABC_ERR_WORKSPACE (-3)
#define ABC_ERR_NOT_ENOUGH_PARTICLES (-4)
#define ABC_ERR_UNSUPPORTED (-5)
#define ABC_ERR_COMM (-6)      /* RCCL missing or a collective failed */

/* Largest parameter dimension d the proposal, prior-density, weighted-
 * moments, direct MVN density and LocalTransition entry points accept (one
 * cap for all of them; the runtime-d LocalTransition fit stages a member row
 * of d + 1 doubles in LDS, abc_local_wide.hip).  The fused candidate round,
 * the MVN pack / MFMA density and abc_mvn_fit take d <= 64. */
#define ABC_MAX_D 2048

/* Precision of the transition-density kernel. */
#define ABC_PREC_F64 0 /* f64 MFMA cross term: parity mode (default)   */
#define ABC_PREC_F32 1 /* f32 MFMA cross term: fast mode (~3e-5 rel.)  */
#define ABC_PREC_X3 2  /* f16 MFMA on 3-limb split operands: f32-grade
                          (~1e-7 rel.), fastest; r <= 25 */

/* Prior distribution kinds (scipy.stats names, loc/scale convention). */
#define ABC_PRIOR_FLAT (-1)  /* no prior: density 1 everywhere (plain rvs) */
#define ABC_PRIOR_NORM 0    /* params: loc, scale                       */
#define ABC_PRIOR_UNIFORM 1 /* params: loc, scale -> U[loc, loc+scale]  */
#define ABC_PRIOR_EXPON 2   /* params: loc, scale                       */
#define ABC_PRIOR_LAPLACE 3 /* params: loc, scale                       */
#define ABC_PRIOR_LOGNORM 4 /* params: s, loc, scale                    */
#define ABC_PRIOR_GAMMA 5   /* params: a, loc, scale                    */
#define ABC_PRIOR_BETA 6    /* params: a, b, loc, scale                 */
/* any other scipy.stats family: the device knows only its support [lo, hi]
 * (re-draw test) and a point c inside it (the t = 0 draw, which the host
 * replaces by ppf(u) of abc_prior_uniforms); density factor 1 on the
 * support -- the host adds the scipy log density of the kept rows.
 * params: lo, hi, c */
#define ABC_PRIOR_HOST 7

const char* abc_last_error(void);
int abc_version(void);

/* Timing of the dominant kernel (the transition-density GEMM launch inside
 * abc_mvn_logpdf): between begin and end, HIP events are recorded on the
 * launch stream directly around each such launch; end synchronises on them
 * and returns the summed elapsed time and the number of launches. */
int abc_profile_begin(void);
int abc_profile_end(double* total_ms, int64_t* launches);
/* The other timing channels of the last begin/end window: ABC_PROF_DENSITY
 * (what abc_profile_end returns), ABC_PROF_CANDIDATES (the fused candidate
 * round kernel), ABC_PROF_REGEN (regeneration of kept rows),
 * ABC_PROF_RESCUE (the exact density pass over rescued candidates). */
#define ABC_PROF_DENSITY 0
#define ABC_PROF_CANDIDATES 1
#define ABC_PROF_REGEN 2
#define ABC_PROF_RESCUE 3
int abc_profile_channel(int channel, double* total_ms, int64_t* launches);

/* ---- reductions used by the fits ------------------------------------------
 * Replaces the numpy work in MultivariateNormalTransition.fit
 * (pyabc/transition/multivariatenormal.py:72-83, smart_cov util.py:4-16):
 * out[0] = sum w, out[1] = sum w^2, out[2 .. 2+d) = weighted mean
 * (sum w x / sum w), out[2+d .. 2+d+d*d) = sum w (x-mean)(x-mean)^T / sum w,
 * out[2+d+d*d] = max w (out holds 3 + d + d*d doubles).
 * Deterministic two-pass fp64 (per-block partials, fixed-order combine);
 * d <= ABC_MAX_D (above 64: one column / one covariance entry per thread). */
size_t abc_weighted_moments_workspace(int64_t N, int d);
int abc_weighted_moments(const double* X, const double* w, int64_t N, int d,
                         double* out, void* ws, size_t ws_bytes, void* stream);

/* Inclusive prefix sum (fp64), the cumulative weights behind
 * np.random.choice(p=w) in MultivariateNormalTransition.rvs
 * (multivariatenormal.py:85-91). */
size_t abc_scan_workspace(int64_t N);
int abc_inclusive_scan_f64(const double* in, double* out, int64_t N, void* ws,
                           size_t ws_bytes, void* stream);

/* Population._normalize_weights (pyabc/population.py:123-145, one model) and
 * effective_sample_size (pyabc/weighted_statistics.py:73-83): w /= sum w in
 * place; stats[0] = sum w (before), stats[1] = ESS = (sum w)^2 / sum w^2,
 * stats[2] = sum w^2 (before). */
size_t abc_normalize_weights_workspace(int64_t N);
int abc_normalize_weights(double* w, int64_t N, double* stats, void* ws,
                          size_t ws_bytes, void* stream);

/* ---- MultivariateNormalTransition.pdf (multivariatenormal.py:99-113) -----
 * density(x_i) = sum_j w_j N(x_i - X_j; 0, Sigma).  The caller supplies the
 * fp64 whitening of Sigma (scipy _PSD semantics; abc_mvn_fit computes it on
 * the device): U [d x r], mean mu [d].
 * pack: builds the MFMA A-operand image of the population once per fit:
 *   y_j = (X_j - mu) U,  c_j = log(w_j) + log_w_shift - |y_j|^2 / 2
 * (log_w_shift = -log max w keeps every exponent <= 0; log_w_shift_dev,
 * device, nullable, X3 only: read the shift from there instead, e.g.
 * abc_mvn_fit's stats[3], so the fit needs no host read).  `range` (device,
 * 2 doubles, nullable; X3 only) receives max_j |y_j| in the log2-scaled
 * units of the X3 kernel (sqrt(log2 e) y) and the limb grid exponent E the
 * image was built with; the X3 image is accurate to ~1e-7 for E <= 8 (use
 * F64 otherwise).
 * logpdf: out[i] = log(sum_j w_j exp(-|(x_i - X_j) U|^2 / 2)) + log_const,
 *   log_const = -(r log 2pi + log pdet)/2 - log_w_shift.  prec selects the
 *   f64-MFMA, f32-MFMA or limb-split f16-MFMA (X3) kernel.  The X3 image
 *   also stores the fp64 whitened population and log2 weights: candidates
 *   outside its range (or whose density underflows 2^-60 relative to max w)
 *   are recomputed from them in fp64 on the device (X, w may be NULL for
 *   X3).  r <= 59 (X3: r <= 25).
 *   hint_rows (device int64 [M], nullable; X3 only): for each candidate a
 *   population row near it -- the proposal's ancestor in the sampler.  Its
 *   exact fp64 log-kernel value becomes the candidate's exponent offset, which
 *   replaces the X3 kernel's max pre-pass over the population (a quarter of
 *   its MFMA work).  Invalid rows (outside [0, N) or w <= 0) send the
 *   candidate to the fp64 rescue path.  With hints, candidates whose hinted
 *   offset proves too far below their maximum are re-run through the exact
 *   (unhinted) pass on a gathered subset, launched device-sized (waves past
 *   the subset's device-side count leave): no host read. */
size_t abc_mvn_packed_bytes(int64_t N, int r, int prec);
int abc_mvn_pack_population(const double* X, const double* w, int64_t N, int d,
                            const double* mu, const double* U, int r,
                            double log_w_shift, const double* log_w_shift_dev,
                            int prec, void* packed, double* range, void* stream);
/* The host half of MultivariateNormalTransition.fit on the device
 * (multivariatenormal.py:72-83 and scipy's _PSD behind its frozen
 * multivariate_normal): from abc_weighted_moments' output `moments`
 * [sum w, sum w^2, mean (d), biased cov (d x d), max w] of normalised
 * weights, cov = np.cov(X, aweights=w) * bw^2 * scaling with bw the
 * bandwidth rule of the effective sample size 1 / sum w^2 (bw_rule 0 =
 * silverman_rule_of_thumb :27-37, 1 = scott_rule_of_thumb :14-24); its
 * eigen-decomposition (parallel Jacobi, fp64) with eigenvalues `evals` (d,
 * decreasing) and vectors `evec` (d x d, columns); the whitening U (d x d:
 * columns of the eigenvalues above 1e6 eps max|s| scaled by 1/sqrt(s), the
 * others zero); the lower sampling factor L (L L^T = cov, semidefinite
 * Cholesky); stats (8) = [rank, log pdet, support tol, -log max w, bw,
 * min s, max s, ok (0: cov not positive semidefinite)].  All device, one
 * single-workgroup launch, no host read; d <= 64.  A full-rank covariance
 * whose smallest eigenvalue is certified above the cut-off (1 / |L^-1|_F^2 >
 * 4e6 eps trace) is whitened by U = L^-T instead, with no eigen-
 * decomposition: evals / evec are then NaN and stats[5], stats[6] the
 * eigenvalue bounds used. */
int abc_mvn_fit(const double* moments, int d, double scaling, int bw_rule,
                double* cov, double* evec, double* evals, double* U, double* L,
                double* stats, void* stream);
size_t abc_mvn_logpdf_workspace(int64_t M, int64_t N, int r, int prec);
/* K slots the X3 kernel executes per (candidate, population row) pair at
 * whitened rank r (the f16 MFMA work per pair is 2 K FLOP; K = 16 x the
 * v_mfma_f32_32x32x16_f16 instructions per 32x32 tile pair) and its 32-column
 * candidate tiles per wave (nullable outputs); returns the kernel (1 =
 * mvn_x3_kernel<K / 16, tiles> on 32x32x16).  A layout query for reporting
 * (bench.py names the instantiation its traffic file must match); no device
 * work. */
int abc_mvn_x3_layout(int r, int* kslots, int* tiles_per_wave);
int abc_mvn_logpdf(const double* x, int64_t M, int d, const void* packed,
                   const double* X, const double* w, int64_t N,
                   const double* mu, const double* U, int r, int prec,
                   double log_const, double log_w_shift, double* out,
                   const int64_t* hint_rows, void* ws, size_t ws_bytes,
                   void* stream);
/* Direct-difference fp64 VALU path: any r, and scipy's singular-covariance
 * support mask (pairs with |(x_i - X_j) V| >= support_tol get density 0;
 * V [d x nv] null-space basis, nv = d - r); d <= ABC_MAX_D (the
 * MultivariateNormalTransition density above d = 64). */
int abc_mvn_logpdf_direct(const double* x, int64_t M, const double* X,
                          const double* w, int64_t N, int d, const double* U,
                          int r, const double* V, int nv, double support_tol,
                          double log_const, double* out, void* stream);

/* ---- proposal: Transition.rvs + prior support (smc.py:610-662) ----------
 * Candidate g (global index idx0 .. idx0+B-1) draws, from Philox4x32-10 keyed
 * by (seed, generation, g, slot), an ancestor j ~ Cat(w) by inverse CDF over
 * `cdf` (inclusive prefix of w) and theta = X_j + L n, n ~ N(0, I_d)
 * (L: the lower-triangular square root of Sigma, L L^T = Sigma, [d x d]
 * row-major; entries above the diagonal are not read).  It re-draws while the
 * prior density is 0 (smc.py:654-656; at most max_attempts), and writes
 * theta [B x d], prior log-density [B], ancestor [B] and attempts used [B]
 * (attempts > max_attempts means "gave up").  With X == NULL it samples the
 * prior itself (t = 0, smc.py:631-634).
 * Prior: per dimension kind[k] (ABC_PRIOR_*) and params[4k .. 4k+4). */
/* Guide table for the ancestor draw: guide[k] = first index with
 * cdf > k * cdf[N-1] / N (k < N; int32 [N]).  Built once per fit; with it the
 * proposal's inverse-CDF search starts in a bracket of ~3 table bins. */
int abc_cdf_guide(const double* cdf, int64_t N, int32_t* guide, void* stream);
/* guide: nullable (binary search over the whole cdf). */
int abc_propose(const double* X, const double* cdf, const int32_t* guide,
                int64_t N, int d, const double* L, const int32_t* prior_kind,
                const double* prior_params, uint64_t seed, uint32_t generation,
                int64_t idx0, int64_t B, int max_attempts, double* theta,
                double* prior_logpdf, int64_t* ancestor, int32_t* attempts,
                void* stream);
/* Prior log-density of given parameters (Distribution.pdf,
 * pyabc/random_variables.py:425-452), product over dimensions. */
int abc_prior_logpdf(const double* theta, int64_t B, int d,
                     const int32_t* prior_kind, const double* prior_params,
                     double* out, void* stream);
/* u[b] in (0, 1): the uniform of candidate idx0 + b's prior stream for
 * dimension k in the attempt it accepted (attempts[b], from abc_propose; null:
 * the first attempt).  An ABC_PRIOR_HOST coordinate's t = 0 draw is the
 * host's ppf(u) (Distribution.rvs, random_variables.py:412-423, for a family
 * without a device sampler), keyed like every other draw. */
int abc_prior_uniforms(const int32_t* attempts, double* u, int64_t B, int k,
                       uint64_t seed, uint32_t generation, int64_t idx0,
                       void* stream);

/* ---- vectorised synthetic simulator (the Model.sample boundary,
 * pyabc/model.py:89-116): x[b,k] = a[k] * theta[b, src[k]] + sigma[k] * e,
 * e ~ N(0,1): normal k of candidate idx0+b's stream (Philox slot
 * 0x40000000 + k/4, four Box-Muller normals per slot). */
int abc_simulate_linear_gaussian(const double* theta, int64_t B, int d, int S,
                                 const int32_t* src, const double* a,
                                 const double* sigma, uint64_t seed,
                                 uint32_t generation, int64_t idx0, double* x,
                                 void* stream);

/* ---- PNormDistance.__call__ (pyabc/distance/distance.py:79-105) ----------
 * d[b] = (sum_k |wf[k] (x[b,k] - x0[k])|^p)^(1/p); p = +inf -> max.
 * wf = weights * factors, in x_0 key order. */
int abc_pnorm(const double* x, int64_t B, int S, const double* x0,
              const double* wf, double p, double* d, void* stream);

/* A proposal that exhausted max_attempts (attempts > max_attempts) is not a
 * valid candidate (the reference keeps drawing, smc.py:649-662): its
 * distance becomes `value` so that no acceptor takes it -- NaN for a
 * distance (NaN <= eps is false even at eps = +inf), the zero-probability
 * density (-inf on log scale, 0 on linear scale) for a StochasticAcceptor,
 * whose "distance" is a noise-model density (higher = more likely). */
int abc_mask_gave_up(double* dist, const int32_t* attempts, int64_t B,
                     int max_attempts, double value, void* stream);

/* ---- UniformAcceptor (acceptor.py:235-244) + order-preserving compaction -
 * accept[b] = d[b] <= eps.  Writes the positions of accepted rows in
 * increasing order to idx and their number to *count (device int64). */
size_t abc_compact_workspace(int64_t B);
int abc_accept_compact(const double* d, int64_t B, double eps, int64_t* idx,
                       int64_t* count, void* ws, size_t ws_bytes,
                       void* stream);
/* ---- fused candidate round: the whole per-candidate closure ---------------
 * Replaces one sampler round of pyabc/sampler/singlecore.py:20-38 /
 * multicore_evaluation_parallel.py:92-150 over the closure smc.py:588-724:
 * Transition.rvs + prior re-draw (smc.py:610-662; MultivariateNormalTransition
 * multivariatenormal.py:85-97 with L shared, LocalTransition
 * local_transition.py:141-145 with per-particle L, or the prior itself at
 * t = 0 when X == NULL), LinearGaussianModel (model.py:89-116), PNormDistance
 * (distance.py:79-105) and UniformAcceptor d <= eps (acceptor.py:235-244).
 * Candidate b of a round is global index idx0 + b, keyed exactly like
 * abc_propose / abc_simulate_linear_gaussian, so a round accepts precisely
 * the candidates the staged kernels (propose -> simulate -> pnorm ->
 * accept_compact) would.  A candidate whose proposal exhausted max_attempts
 * is rejected (the reference never accepts a zero-prior-density parameter).
 * The spec struct is HOST memory; the arrays it points to are device memory. */
typedef struct abc_candidate_spec {
  int d;                       /* parameters (sorted names)                */
  int S;                       /* summary statistics (x_0 key order)       */
  const double* X;             /* population [N x d]; NULL: prior draw     */
  const double* cdf;           /* inclusive scan of the weights [N]        */
  const int32_t* guide;        /* abc_cdf_guide table [N] (nullable)        */
  int64_t N;
  const double* L;             /* [d x d], or [N x d x d] per particle:
                                  lower-triangular factors (L L^T = cov;
                                  entries above the diagonal are not read) */
  int per_particle_L;
  const int32_t* prior_kind;   /* [d] ABC_PRIOR_*                          */
  const double* prior_params;  /* [4 d]                                    */
  int max_attempts;            /* prior re-draws per candidate             */
  const int32_t* src;          /* simulator: x_k = a_k theta[src_k]        */
  const double* a;             /*            + sigma_k e_k                 */
  const double* sigma;
  const double* x0;            /* PNorm: observed [S]                      */
  const double* wf;            /*        weights * factors [S]             */
  double p;                    /*        p >= 1, +inf = max norm           */
  uint64_t seed;
  uint32_t generation;
  const void* anc_table;       /* abc_ancestor_table of (X, cdf); required
                                  with X (the guide field is then unused) */
  const double* support_box;   /* [d x (lo, hi)] from abc_prior_support_box
                                  (nullable: each call computes it)        */
} abc_candidate_spec;
/* The prior's support box [d x (lo, hi)] the proposal's re-draw loop tests
 * (smc.py:654-656: a proposal with prior density 0 is re-drawn), computed
 * once per generation instead of once per round (device, 2 d doubles). */
int abc_prior_support_box(const int32_t* prior_kind, const double* prior_params, int d,
                          double* box, void* stream);
/* Ancestor table of a population for the fused rounds: the rows X_j with
 * their weight-scan value in 128-byte-aligned records, and a guide over
 * 4 N scan bins (abc_candidate.h).  Same ancestors as the cdf / guide
 * search (np.searchsorted(cdf, u * total, side="right"), smc.py:652 via
 * multivariatenormal.py:90-94), fewer cache lines per draw.  The header's
 * first double is max |X_jk| (the lazy early reject's support bound).
 * table: device buffer of abc_ancestor_table_bytes(N, d) bytes, 128-byte
 * aligned. */
int64_t abc_ancestor_table_bytes(int64_t N, int d);
int abc_ancestor_table(const double* X, const double* cdf, int64_t N, int d,
                       void* table, size_t table_bytes, void* stream);
/* One round of B candidates: writes the positions b (0 <= b < B, increasing)
 * of the first `cap` accepted candidates to idx and the number accepted in
 * the round (uncapped) to *count (device int64).  The threshold is eps, or,
 * when eps_dev (device, nullable) is given, *eps_dev * eps_scale read on the
 * device (QuantileEpsilon's quantile x its multiplier, so the round can be
 * queued before the host has the value).  rec_x (nullable) receives
 * the sum stats of every candidate [B x S] (record_rejected).  filter != 0
 * allows the exact early-rejection mode (first 4 statistics, p in {1,2,inf},
 * no rec_x; for the shared-L transition with every coordinate beyond the
 * 4th provably inside the support, only theta_0..3 of the first attempt):
 * the same accept set at lower cost when few candidates pass.
 * Workspace: abc_candidates_workspace(B) bytes whose first 256 bytes are
 * zero before the first call (e.g. hipMemset at allocation); every call
 * leaves them zero again (the round's tile ticket counter). */
size_t abc_candidates_workspace(int64_t B);
int abc_candidates_round(const abc_candidate_spec* spec, int64_t idx0,
                         int64_t B, double eps, const double* eps_dev,
                         double eps_scale, int filter, int64_t cap,
                         int64_t* idx, int64_t* count, double* rec_x,
                         void* ws, size_t ws_bytes, void* stream);
/* Rows of the kept candidates: for i < n, candidate idx0 + idx[i] ->
 * theta [n x d], prior log-density [n], ancestor [n] (nullable; -1 at t = 0),
 * sum stats x [n x S], distance [n]; bit-identical to the staged kernels.
 * n_dev (nullable, device int64): the rows are the first min(n, *n_dev) --
 * a launch sized on the device (abc_candidates_round's count), queued before
 * the host has read that count. */
/* Multi-rank round cutoff on the device: counts [nranks] (device int64, the
 * round's accept counts of every rank, all-gathered in rank order) ->
 * *keep (device int64) = how many of rank `rank`'s accepted candidates are
 * among the first `need` accepted in global order.  Lets a rank queue
 * abc_candidates_regen (n_dev = keep) before the host reads the counts;
 * the reference takes the first n by evaluation index
 * (pyabc/sampler/multicore_evaluation_parallel.py:133-135). */
int abc_round_keep(const int64_t* counts, int nranks, int rank, int64_t need, int64_t* keep,
                   void* stream);
int abc_candidates_regen(const abc_candidate_spec* spec, int64_t idx0,
                         const int64_t* idx, int64_t n, const int64_t* n_dev,
                         double* theta, double* prior_logpdf, int64_t* ancestor,
                         double* x, double* dist, void* stream);

/* Proposals only, candidates idx0 .. idx0 + B - 1: theta [B x d], prior
 * log-density [B] (-inf when the proposal gave up; may be null -- the
 * sampler computes it for the kept rows only, abc_prior_logpdf gives the
 * same bits), ancestor [B] (may be null), attempts [B] (may be null).  The fused round's proposal
 * (propose_one over the ancestor table, the prior support box computed once):
 * bit-identical to abc_propose / abc_local_propose and to the rows
 * abc_candidates_regen returns.  The spec's simulator / distance fields must
 * be valid but are not read.  Replaces, for the staged sampler path,
 * MultivariateNormalTransition.rvs / LocalTransition.rvs_single + the prior
 * re-draw loop (pyabc/smc.py:610-662, transition/multivariatenormal.py:85-97,
 * transition/local_transition.py:141-145).  Workspace:
 * abc_candidates_propose_workspace() bytes. */
size_t abc_candidates_propose_workspace(void);
int abc_candidates_propose(const abc_candidate_spec* spec, int64_t idx0, int64_t B,
                           double* theta, double* prior_logpdf, int64_t* ancestor,
                           int32_t* attempts, void* ws, size_t ws_bytes, void* stream);

/* Accept tail of a user simulator's round: PNormDistance of every row of
 * x [B x S] to x0 with weights*factors wf (pyabc/distance/distance.py:79-105,
 * the arithmetic of abc_pnorm per row) and the UniformAcceptor test d <= eps
 * (acceptor/acceptor.py:235-244) in one pass; rows whose attempts exceed
 * max_attempts (nullable) are rejected (abc_mask_gave_up).  Writes the
 * positions of the first `cap` accepted rows (increasing) to idx and the
 * number accepted (uncapped) to *count (device int64); no distance array.
 * Replaces, for VectorizedModels without a fused simulator, the staged
 * abc_pnorm + abc_mask_gave_up + abc_accept_compact of one round
 * (the per-candidate accept of pyabc/model.py:163-218 via smc.py:664-724).
 * Workspace: abc_candidates_workspace(B) bytes. */
int abc_pnorm_accept(const double* x, int64_t B, int S, const double* x0,
                     const double* wf, double p, double eps, const int32_t* attempts,
                     int max_attempts, int64_t cap, int64_t* idx, int64_t* count,
                     void* ws, size_t ws_bytes, void* stream);

/* Gather rows: out[i, :] = in[idx[i], :] (row width `cols` doubles). */
int abc_gather_rows(const double* in, const int64_t* idx, int64_t n, int cols,
                    double* out, void* stream);
/* The same for up to 8 arrays sharing one index list, in one launch:
 * outs[a][(out_row0[a] + i) * cols[a] + c] = ins[a][idx[i] * cols[a] + c].
 * ins/outs/cols/out_row0 are HOST arrays of n_arrays entries (the pointers
 * they hold are device memory); 8-byte elements (int64 columns travel as
 * their bit patterns). */
int abc_gather_rows_batch(int n_arrays, const double* const* ins,
                          const int* cols, double* const* outs,
                          const int64_t* out_row0, const int64_t* idx,
                          int64_t n, void* stream);

/* ---- importance weight (smc.py:768-811, single model) --------------------
 * w[i] = exp(prior_logpdf[i] - trans_logpdf[i]) * scale * acc_weights[i]
 * (t > 0; acc_weights = the StochasticAcceptor's acceptance weights, NULL
 * for the uniform acceptor). */
int abc_importance_weights(const double* prior_logpdf,
                           const double* trans_logpdf,
                           const double* acc_weights, int64_t A, double scale,
                           double* w, void* stream);

/* ---- QuantileEpsilon (epsilon.py:202-228 -> weighted_statistics.py:27-43)
 * abc_weighted_quantile: q = interp(alpha, (cumsum(w) - w/2) / sum(w),
 * points sorted ascending, ties by index), found by a weighted MSD select
 * (fixed-point bin weights, a few hundred points sorted around the knots;
 * abc_quantile.hip), written to *q (device double).  Weights >= 0.  When
 * the knots lie in more than 2048 points of one narrow slice of the key span
 * (2^-23 of it or less; ties by the thousand) it writes NaN: the caller then runs
 * abc_weighted_quantile_sorted (full stable radix sort, always decided).
 * abc_weighted_quantile's workspace is zero before its first call (e.g.
 * hipMemset at allocation) and every call leaves its control block zero.
 * abc_sort_pairs_f64: stable LSD radix sort of fp64 keys carrying fp64
 * values. */
size_t abc_sort_pairs_workspace(int64_t N);
int abc_sort_pairs_f64(const double* keys, const double* vals, int64_t N,
                       double* keys_out, double* vals_out, void* ws,
                       size_t ws_bytes, void* stream);
size_t abc_weighted_quantile_workspace(int64_t N);
int abc_weighted_quantile(const double* points, const double* w, int64_t N,
                          double alpha, double* q, void* ws, size_t ws_bytes,
                          void* stream);
size_t abc_weighted_quantile_sorted_workspace(int64_t N);
int abc_weighted_quantile_sorted(const double* points, const double* w, int64_t N,
                                 double alpha, double* q, void* ws, size_t ws_bytes,
                                 void* stream);

/* ---- AdaptivePNormDistance._update scales (distance.py:263-307,
 * scale.py:38-65) over recorded sum stats X [R x S] (row-major):
 * std: np.std (ddof 0); mad: median(|x - median(x)|), even R averaging the
 * two middle order statistics like np.median. */
size_t abc_column_stats_workspace(int64_t R, int S);
int abc_column_std(const double* X, int64_t R, int S, double* out, void* ws,
                   size_t ws_bytes, void* stream);
int abc_column_mad(const double* X, int64_t R, int S, double* out, void* ws,
                   size_t ws_bytes, void* stream);

/* ---- LocalTransition (pyabc/transition/local_transition.py:77-145) -------
 * fit: per particle n, the k nearest other particles (ties by index),
 * weighted covariance of their offsets (weights renormalised, unbiased
 * 1/(1 - sum a^2)), all-zero -> diag(|X[0]|), times scaling, then
 * "while det <= 0: cov += eps I".  Writes covs, inverse covs, dets,
 * Cholesky factors (for rvs) and log normalisation
 * log sqrt((2 pi)^d det) per particle.  d <= 64: d <= 16 on the templated
 * select / moments kernels, 16 < d <= 64 on runtime-d kernels (one
 * workgroup per particle, abc_local_wide.hip).  N < 2^31. */
size_t abc_local_fit_workspace(int64_t N, int d);
int abc_local_fit(const double* X, const double* w, int64_t N, int d,
                  int64_t k, double scaling, double eps, double* covs,
                  double* inv_covs, double* dets, double* chol,
                  double* log_norm, void* ws, size_t ws_bytes, void* stream);
/* pdf: out[i] = log( sum_j w_j exp(-d_ij^T inv_j d_ij / 2 - log_norm_j)
 * / sum_j w_j ), d_ij = X_j - x_i.  d <= 16: the quadratic form is a GEMM
 * over the candidates' quadratic features on fp64 MFMA (workspace: packed
 * population coefficients + per-chunk partial sums); 16 < d <= 64: a direct
 * fp64 quadratic form per pair (no workspace). */
size_t abc_local_logpdf_workspace(int64_t M, int64_t N, int d);
int abc_local_logpdf(const double* x, int64_t M, const double* X,
                     const double* w, int64_t N, int d, const double* inv_covs,
                     const double* log_norm, double* out, void* ws,
                     size_t ws_bytes, void* stream);
/* rvs: ancestor j ~ Cat(w) (cdf), theta = X_j + chol_j n; same Philox keying
 * and prior re-draw loop as abc_propose. */
int abc_local_propose(const double* X, const double* cdf,
                      const int32_t* guide, int64_t N, int d,
                      const double* chol, const int32_t* prior_kind,
                      const double* prior_params, uint64_t seed,
                      uint32_t generation, int64_t idx0, int64_t B,
                      int max_attempts, double* theta, double* prior_logpdf,
                      int64_t* ancestor, int32_t* attempts, void* stream);

/* ---- bootstrapped KDE variation (pyabc/cv/bootstrap.py:86-108) ----------
 * logdens [B x N] row-major: log densities of B bootstrapped transitions at
 * N test points.  variation[i] = std_b(exp) / mean_b(exp) (scipy.stats
 * .variation, ddof 0); *cv = sum_i variation[i] * scale * w[i] (device
 * double).  Replaces the numpy/scipy tail of calc_cv. */
size_t abc_bootstrap_cv_workspace(int64_t N);
int abc_bootstrap_cv(const double* logdens, int64_t B, int64_t N,
                     const double* w, double scale, double* variation,
                     double* cv, void* ws, size_t ws_bytes, void* stream);

/* ---- Stochastic acceptance (acceptor/acceptor.py:309-476,
 * distance/kernel.py:18-592, epsilon/temperature.py:276-742) ---------------
 * abc_kernel_logpdf: log pdf(x_0 | x) of a StochasticKernel per row of the
 *   sum-stat matrix x [B x S]; cols[K] = column of each kernel element (the
 *   kernel's sorted key order), x0k[K] the observed values.  kind:
 *   0 IndependentNormalKernel (par = var[K], c = sum log(2 pi var)),
 *   1 IndependentLaplaceKernel (par = scale[K], c = sum log(2 scale)),
 *   2 NormalKernel (U [K x r] with U U^T = pinv(cov), c = r log 2pi + log pdet),
 *   3 PoissonKernel, 4 BinomialKernel (par[0] = p), 5 NegativeBinomialKernel
 *   (par[0] = p).  ret_lin: write exp(log pdf) (SCALE_LIN).
 *   Replaces StochasticKernel.__call__ (kernel.py:207-226, 285-303, 361-378,
 *   426-445, 478-495, 533-552).
 * abc_stochastic_accept: StochasticAcceptor.__call__ (acceptor.py:434-476)
 *   for B candidates with global indices idx0.. : key[b] = u - acc (accepted
 *   iff key <= 0, feed to abc_accept_compact with eps 0), accw[b] = the
 *   acceptance weight.  u comes from the counter-based stream (seed,
 *   generation, index).
 * abc_temper_sums: one objective evaluation of AcceptanceRateScheme (mode 0,
 *   temperature.py:322-352) or EssScheme (mode 1, temperature.py:710-742) at
 *   beta, over R records with densities dens and log importance weights
 *   lr - lr_sub (log t_pd - log t_pd_prev; lr_sub may be NULL) shifted by
 *   `shift`; for mode 1, lr holds the linear population weights; mode 2
 *   writes max(lr - lr_sub); mode 3 = mode 0 with linear record weights in
 *   lr.  out[2] device doubles. */
int abc_kernel_logpdf(const double* x, int64_t B, int S, const int32_t* cols,
                      int K, const double* x0k, int kind, const double* par,
                      const double* U, int r, double c, int ret_lin,
                      double* out, void* stream);
int abc_stochastic_accept(const double* dens, int64_t B, double pdf_norm,
                          double temperature, int scale_log, int apply_iw,
                          uint64_t seed, uint32_t generation, int64_t idx0,
                          double* key, double* accw, void* stream);
size_t abc_temper_workspace(void);
int abc_temper_sums(const double* dens, const double* lr,
                    const double* lr_sub, int64_t R, double pdf_norm, int scale_log, int mode, double beta,
                    double shift, double* out, void* ws, size_t ws_bytes,
                    void* stream);

/* ---- multi-GPU collectives (RCCL over xGMI), SURVEY.md 8(b)/(e) -----------
 * The reference has no collective: MulticoreEvalParallelSampler
 * (multicore_evaluation_parallel.py:92-150) forks workers that share one
 * evaluation counter and queue their particles to the parent.  Here one
 * process drives one GPU and the ranks exchange, per generation, the accept
 * counts (all-gather), the accepted rows (one packed all-gather) and, when
 * the distance adapts, the recorded rows (pyabc_amd/sampler/distributed.py).
 * These entry points give a binding without torch.distributed the same
 * transport: RCCL is opened with dlopen on first use (librccl.so.1), so the
 * library itself does not depend on it.  The caller moves the 128-byte
 * unique id from rank 0 to the others by any channel (the Python binding
 * uses torch.distributed's broadcast), then every rank calls
 * abc_comm_init.  All calls are stream-ordered on `stream`. */
#define ABC_COMM_ID_BYTES 128
#define ABC_COMM_F64 0
#define ABC_COMM_I64 1
#define ABC_COMM_SUM 0
#define ABC_COMM_MAX 1
#define ABC_COMM_MIN 2
int abc_comm_unique_id(void* id);
int abc_comm_init(void** comm, int nranks, int rank, const void* id);
int abc_comm_destroy(void* comm);
/* recv[nranks * bytes] = the ranks' send[bytes] in rank order */
int abc_comm_allgather(void* comm, const void* send, void* recv, size_t bytes,
                       void* stream);
int abc_comm_allreduce(void* comm, const void* send, void* recv, size_t count,
                       int dtype, int op, void* stream);
int abc_comm_broadcast(void* comm, void* buf, size_t bytes, int root, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ABCGPU_H */
