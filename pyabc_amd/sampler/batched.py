"""BatchedGPUSampler: one ABC-SMC generation as a few large kernel launches.

Reference loop: pyabc/sampler/singlecore.py:20-38 and
multicore_evaluation_parallel.py:14-150 call the per-candidate closure
(smc.py:588-724) until n particles are accepted, keep the first n by
evaluation id and count every evaluation.  Here a round of B candidates per
rank runs as

  propose (abc_propose / abc_local_propose, prior re-draw loop inside)
  -> simulate (VectorizedModel, e.g. abc_simulate_linear_gaussian)
  -> distance (abc_pnorm) -> accept + order-preserving compaction
     (abc_accept_compact)

with one host read of the accept count per round.  Once n are accepted the
importance weights prior / transition (smc.py:768-811) are computed for the
accepted rows only -- the N_acc x N_pop transition density on MFMA
(abc_mvn_logpdf) -- and the accepted rows are gathered across ranks.

Semantics vs. the reference: the accepted set is the first n accepted in
global candidate-index order (deterministic for any rank count), and
``nr_evaluations_`` = global index of the n-th accepted + 1, i.e. no
overshoot is counted (the reference's MulticoreEval counts its overshoot,
multicore_evaluation_parallel.py:138).  Recorded sum stats (record_rejected)
are all candidates up to that cutoff, in index order (SingleCore semantics).
"""
import logging
import math

import numpy as np

from .. import gpu
from .._native import PRIOR_KINDS
from ..distance.distance import SumStatMatrix
from ..population import ColumnarParticles, Particle, Population
from ..parameters import Parameter
from ..random_variables import host_prior_draw, host_prior_logpdf
from . import distributed as dd
from .base import Sampler

logger = logging.getLogger("Sampler")


class ColumnarSample:
    """Sample of the batched sampler (device columns, see Sample)."""

    def __init__(self, columns, recorded, recorded_keys, record_rejected, ok,
                 accepted_flags=None, records=None):
        self._cols = columns
        self._records = records              # (theta, dens, key, anc) or None
        self._recorded = recorded            # [R, S] device or None
        self._recorded_keys = recorded_keys
        self._accepted_flags = accepted_flags
        self.record_rejected = record_rejected
        self.ok = ok

    @property
    def n_accepted(self):
        return 0 if self._cols is None else len(self._cols)

    def get_accepted_population(self):
        return Population.from_columns(self._cols)

    def first_m_sum_stats(self, m):
        rec = self._recorded
        if rec is None:
            return []
        if m is not None and np.isfinite(m) and m < rec.shape[0]:
            rec = rec[: int(m)].contiguous()
        return SumStatMatrix(rec, self._recorded_keys)

    def device_records(self, m=None):
        """(theta [R, d], density [R], acceptance key [R], ancestor [R] or
        None) of the first m recorded candidates (all evaluated candidates
        up to the cutoff, accepted and rejected, in index order); None if
        the generation did not record them (StochasticAcceptor runs with
        record_rejected only)."""
        if self._records is None:
            return None
        th, dn, key, anc = self._records
        if m is not None and np.isfinite(m) and m < th.shape[0]:
            m = int(m)
            th, dn, key = th[:m], dn[:m], key[:m]
            anc = None if anc is None else anc[:m]
        return th, dn, key, anc

    @property
    def all_sum_stats(self):
        return self.first_m_sum_stats(np.inf)

    def first_m_particles(self, m):
        c = self._cols
        th = c.theta.cpu().numpy()
        w = c.weights.cpu().numpy()
        d = c.distances.cpu().numpy()
        ss = c.sum_stats.cpu().numpy()
        parts = [Particle(m=c.m, parameter=Parameter(dict(zip(c.param_names, th[i]))),
                          weight=float(w[i]),
                          accepted_sum_stats=[dict(zip(c.sum_stat_keys, ss[i]))],
                          accepted_distances=[float(d[i])])
                 for i in range(len(c))]
        m = len(parts) if m is None or not np.isfinite(m) else int(m)
        return parts[:m]


class BatchedGPUSampler(Sampler):
    """Batched, device-resident sampler (single model, nr_samples_per_param 1).
    Closures outside that (a plain ``simulate_one``, a scalar model, ...) run
    the reference's per-candidate loop instead (_sample_per_candidate).

    Parameters
    ----------
    batch_size: candidates per rank and round (None: adapt to the measured
        acceptance rate).
    max_batch_size: cap on the adaptive batch of the staged path (default:
        what staged_round_bytes of candidate rows allow, at most 2^25).
    seed: base seed of the counter-based RNG (None: drawn from numpy's global
        RNG on rank 0 and broadcast).
    max_attempts: prior re-draws per candidate before giving up
        (the reference loops forever and warns at 1000, smc.py:658-662).
    check_max_eval: stop a generation once ``max_eval`` candidates are
        evaluated (sample not ok), like the reference samplers' flag of the
        same name (singlecore.py:14-26); off by default, as there.
    record_device_budget_bytes: optional cap on the HBM the recorded rows of
        one generation may take (default: none, as in the reference); when
        hit, the first rows that fit are kept and
        ``last_stats["records_truncated"]`` is set.
    """

    FUSED_MAX_STATS = 256     # abc_candidates_round: S <= SIM_SMAX
    FUSED_MAX_DIM = 64        # abc_candidates_round / _propose: d <= 64

    def __init__(self, batch_size=None, max_batch_size=None, seed=None,
                 max_attempts=10000, check_max_eval=False, fused=True,
                 max_fused_batch_size=1 << 31, filter_below=0.0,
                 filter_min_stats=5, record_budget_bytes=1 << 31,
                 record_device_budget_bytes=None, allow_per_candidate=True):
        super().__init__()
        # a generation without a batched form (plain closure, non-vectorised
        # model, discrete host prior, ...) runs the per-candidate loop with a
        # warning; False makes it a TypeError instead
        self.allow_per_candidate = allow_per_candidate
        self.check_max_eval = check_max_eval
        self.batch_size = batch_size
        self.max_batch_size = max_batch_size
        # device bytes one staged round may hold in candidate rows (theta,
        # sum stats, distance, ancestor, the user simulator's output): at
        # low acceptance rounds of 2^22 candidates meant hundreds of rounds
        # (one host read each) per generation
        self.staged_round_bytes = 1 << 34
        self.seed = seed
        self.max_attempts = max_attempts
        # fused candidate rounds (abc_candidates_round): one kernel per round,
        # one accept bit per candidate, accepted rows regenerated; used when
        # the model is a LinearGaussianModel, the distance a PNormDistance,
        # the acceptor uniform and the transition an MVN / LocalTransition
        self.fused = fused
        self.max_fused_batch_size = max_fused_batch_size
        # early-reject mode (the lazy head: theta_0..3 and 4 statistics
        # decide most rejections) below this acceptance rate, for rounds
        # where the lazy head applies (_lazy_capable) with at least
        # filter_min_stats statistics.  Off by default: the round is bound
        # by the ancestor table's random accesses (~2 Infinity-Cache misses
        # per candidate, the same with or without the head) as much as by
        # its arithmetic, and the head rejects few candidates when the 4
        # statistics are a small part of the distance: c3 bench 4.54e6 vs
        # 4.78e6 accepted/s; tools/bench_fused.py 1.4e10 vs 1.9e10
        # candidates/s at S = 32 (profiles/r02_lazy_filter_ab.log,
        # r02_lazy_filter_S.log)
        self.filter_below = filter_below
        self.filter_min_stats = filter_min_stats
        self.record_budget_bytes = record_budget_bytes  # rec rows per fused round
        # first m recorded candidates are all that is used
        # (ABCSMC.max_nr_recorded_particles, smc.py:998-1001)
        self.max_nr_recorded = np.inf
        # optional cap on the HBM held by the recorded rows of one
        # generation (all ranks' rows in global order count).  Off by
        # default: the reference keeps every recorded row (smc.py:987-990),
        # and a cap would make the adaptive scales depend on the GPU memory
        # setting.  When set and hit, the first rows that fit are kept, as if
        # max_nr_recorded_particles had been set: logged, and
        # last_stats["records_truncated"] is True
        self.record_device_budget_bytes = record_device_budget_bytes
        self._acc_rate = None
        self._acc_trend = 1.0
        self.last_stats = {}
        # set by ABCSMC.run: host reads of the previous generation (its ESS
        # line), run once this generation's transition density is queued --
        # the longest kernel, so the host work overlaps it
        self.on_density_queued = None

    def _base_seed(self, device):
        if self.seed is None:
            self.seed = dd.broadcast_int(np.random.randint(0, 2 ** 62), device)
        return self.seed

    def _round_size(self, needed, ws, d=1, S=1):
        if self.batch_size is not None:
            return int(self.batch_size)
        rate = self._acc_rate if self._acc_rate else 0.5
        # 30% margin: a second round costs more than the extra candidates
        b = int(math.ceil(needed / max(rate, 1e-9) * 1.3 / ws)) + 256
        cap = self.max_batch_size
        if cap is None:
            per = 8 * (2 * d + 2 * S) + 48     # theta, x (+ a user copy), dist, idx, lp, anc
            cap = max(1 << 16, min(1 << 25, self.staged_round_bytes // per))
        return int(min(max(b, 4096), cap))

    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False, show_progress=False):
        spec = simulate_one
        if not getattr(spec, "batched_capable", False):
            return self._sample_per_candidate(n, simulate_one, max_eval)
        dev = gpu.require_device()
        rank, ws = dd.world()
        seed = self._base_seed(dev)
        gen = spec.t & 0xFFFFFFFF
        record = self.sample_factory.record_rejected
        d = len(spec.param_names)
        fr = None if all_accepted else self._fused_round(spec, seed, gen, dev)
        if fr is not None:
            return self._sample_fused(n, fr, spec, max_eval, record, dev, rank, ws)

        acc_theta, acc_lp, acc_d, acc_x, acc_anc, acc_w = [], [], [], [], [], []
        rec_x = []
        stochastic = getattr(spec, "stochastic", None) is not None and not all_accepted
        # the accept tail (abc_pnorm_accept): a p-norm distance and the
        # uniform acceptor decided in one pass over the user simulator's
        # rows, no distance array; the kept rows' distances afterwards
        pnorm_tail = None
        if not (stochastic or all_accepted or spec.distance is None) and \
                hasattr(spec.distance, "fused_pnorm"):
            pnorm_tail = spec.distance.fused_pnorm(spec.t, spec.sum_stat_keys, dev)
        # StochasticAcceptor + record_rejected: keep every evaluated
        # candidate's (theta, density, key, ancestor) for the temperature
        rec_extra = [] if (stochastic and record) else None
        keeps = []          # per round: accepted rows kept by each rank
        rec_keeps = []      # per round: recorded rows of each rank
        rec_left = self._record_limit(len(spec.sum_stat_keys))
        cut = None          # ws > 1: the last round's cutoff, resolved in _assemble
        n_acc = 0
        base = 0
        n_eval = 0
        ok = True
        rounds = 0
        while n_acc < n:
            if self.check_max_eval and n_eval >= max_eval:
                ok = False
                break
            B = self._limit_to_max_eval(self._round_size(n - n_acc, ws, d,
                                                         len(spec.sum_stat_keys)), max_eval,
                                        n_eval, ws)
            lo, _ = dd.rank_range(base, B, rank)
            theta, lp, anc, att = self._propose(spec, B, seed, gen, lo, d)
            if spec.transition is None and getattr(spec, "host_prior", None):
                # t = 0: the host-scipy leg draws its coordinates as ppf of
                # the candidates' own prior-stream uniforms
                host_prior_draw(theta, att, spec.host_prior, seed, gen, lo)
            x = spec.model.simulate_batch(theta, seed, gen, lo)
            dist = None
            if pnorm_tail is not None:
                if x.dtype != gpu.F64 or not x.is_contiguous():
                    x = x.to(gpu.F64).contiguous()
                kk = min(n - n_acc, B)
                idx, cnt = gpu.pnorm_accept(x, spec.x0vec, *pnorm_tail, spec.eps,
                                            kk, att=att, max_attempts=self.max_attempts)
                if ws == 1:
                    both = gpu.torch.cat([cnt.view(1), idx[kk - 1:kk]]).cpu()
                    cnt_local = int(both[0])
                    pos_hint = int(both[1])
                else:
                    cnt_local = cnt
            elif all_accepted or spec.distance is None:
                dist = gpu.torch.full((B,), np.inf, dtype=gpu.F64, device=dev)
                idx = gpu.torch.arange(B, dtype=gpu.I64, device=dev)
                cnt_local = B
            else:
                dist = spec.distance.device_call(x, spec.x0vec, spec.t,
                                                 spec.sum_stat_keys)
                # a proposal that exhausted max_attempts never enters the
                # population (the reference loops until the prior density is
                # positive, smc.py:649-662): its distance becomes NaN (never
                # <= eps, even at eps = inf); under a StochasticAcceptor the
                # "distance" is a density, so it becomes the zero-probability
                # density instead (acceptance 0, weight 0, and a zero
                # acceptance base in the temperature records)
                if att is not None:
                    if stochastic:
                        gpu.mask_gave_up(dist, att, self.max_attempts,
                                         -np.inf if spec.stochastic[2] else 0.0)
                    else:
                        gpu.mask_gave_up(dist, att, self.max_attempts)
                if stochastic:
                    key, accw = gpu.stochastic_accept(dist, *spec.stochastic,
                                                      seed, gen, lo)
                    if att is not None:
                        # key +inf: never accepted, and marks the row for
                        # ABCSMC._device_records, which leaves it out
                        gpu.mask_gave_up(key, att, self.max_attempts, np.inf)
                    idx, cnt = gpu.accept_compact(key, 0.0)
                else:
                    idx, cnt = gpu.accept_compact(dist, spec.eps)
                if ws == 1:
                    # one read: the count and the index of the n-th accepted
                    # (meaningful only when this round completes the sample)
                    kk = min(n - n_acc, B)
                    tail = idx[kk - 1:kk] if idx.numel() >= kk else cnt.view(1)
                    both = gpu.torch.cat([cnt.view(1), tail]).cpu()
                    cnt_local = int(both[0])
                    pos_hint = int(both[1])
                else:
                    cnt_local = cnt        # gathered on the device, one host read
            counts = dd.allgather_counts(cnt_local, dev)
            keep = dd.cutoff(counts, n - n_acc)
            total_keep = int(keep.sum())
            k_mine = int(keep[rank])
            # evaluations up to the cutoff (global order); rec_all = recorded
            # rows of every rank this round (identical on all ranks)
            rec_all = np.full(ws, B, dtype=np.int64)
            if n_acc + total_keep >= n:
                c_rank = int(np.nonzero(keep)[0][-1])
                if ws > 1:
                    # the cutoff position travels in the generation's packed
                    # row gather (_assemble), not in a collective of its own
                    cut = self._pending_cut(idx, keep, c_rank, rank, B, dev)
                    evaluated = 0
                else:
                    pos = (pos_hint if not (all_accepted or spec.distance is None)
                           else self._local_cutoff_pos(idx, keep[c_rank]))
                    evaluated = c_rank * B + pos + 1
                    rec_all[c_rank] = pos + 1
                    rec_all[c_rank + 1:] = 0
            else:
                evaluated = ws * B
            rec_rows = int(rec_all[rank])
            if k_mine:
                sel = idx[:k_mine]
                lp_cols = [lp] if lp is not None else []
                if dist is None:
                    # the tail kept no distances: the kept rows' ones, the
                    # same per-row arithmetic (abc_pnorm)
                    cols = [theta] + lp_cols + [x] + ([anc] if anc is not None else [])
                    got = gpu.gather_rows_batch(cols, sel)
                    if lp is None:
                        got.insert(1, None)
                    got.insert(2, gpu.pnorm(got[2], spec.x0vec, *pnorm_tail))
                else:
                    cols = [theta] + lp_cols + [dist, x] + \
                        ([anc] if anc is not None else []) + ([accw] if stochastic else [])
                    got = gpu.gather_rows_batch(cols, sel)   # one launch
                    if lp is None:
                        got.insert(1, None)
                if got[1] is None:
                    # kept rows only: the bits the proposal kernel would have
                    # written (same device function)
                    got[1] = gpu.prior_logpdf(got[0], spec.prior_kind, spec.prior_params)
                    if (all_accepted or spec.distance is None) and att is not None:
                        # this branch keeps rows 0..k-1 unfiltered, including
                        # proposals that exhausted max_attempts: their last
                        # draw's density is not the proposal's, and the
                        # proposal kernel would have written -inf (weight 0)
                        gpu.mask_gave_up(got[1], att[:k_mine], self.max_attempts, -np.inf)
                acc_theta.append(got[0])
                acc_lp.append(got[1])
                acc_d.append(got[2])
                acc_x.append(got[3])
                if anc is not None:
                    acc_anc.append(got[4])
                if stochastic:
                    acc_w.append(got[-1])
            if record and cut is not None:
                # rows trimmed once the cutoff position is known (_finish_cut)
                rec_x.append(x)
                rec_keeps.append(None)
                if rec_extra is not None:
                    rec_extra.append((theta, dist, key, anc))
            elif record:
                rec_all, rec_left = self._cap_records(rec_all, rec_left)
                rec_rows = int(rec_all[rank])
                rec_x.append(x[:rec_rows].clone() if rec_rows < B // 2 else x[:rec_rows])
                rec_keeps.append(rec_all)
                if rec_extra is not None:
                    rec_extra.append((theta[:rec_rows], dist[:rec_rows],
                                      key[:rec_rows],
                                      None if anc is None else anc[:rec_rows]))
            keeps.append(keep)
            n_acc += total_keep
            n_eval += evaluated
            base += ws * B
            rounds += 1
            tot_cnt = int(counts.sum())
            self._acc_rate = max(tot_cnt / float(ws * B), 1e-6)
        if n_acc < n:
            ok = False
        cols = self._assemble(spec, acc_theta, acc_lp, acc_d, acc_x, dev, d,
                              all_accepted, keeps, acc_anc, acc_w, cut=cut)
        if cut is not None:
            n_eval, rec_left = self._finish_cut(cut, n_eval, rec_left, rec_keeps,
                                                rec_x if record else None,
                                                rec_extra, rank, ws)
        self.nr_evaluations_ = int(n_eval)
        self.last_stats = dict(rounds=rounds, evaluations=int(n_eval),
                               accepted=int(n_acc),
                               records_truncated=self._records_truncated)
        recorded = None
        records = None
        if record:
            recorded = self._gather_recorded(rec_x, rec_keeps, dev, ws)
            if rec_extra:
                parts = list(zip(*rec_extra))
                records = tuple(
                    None if any(a is None for a in col)
                    else self._gather_recorded(list(col), rec_keeps, dev, ws)
                    for col in parts)
        elif cols is not None:
            recorded = cols.sum_stats
        return ColumnarSample(cols, recorded, spec.sum_stat_keys,
                              record, ok and n_acc == n, records=records)

    def _sample_per_candidate(self, n, simulate_one, max_eval):
        """A closure the batched kernels cannot run -- a plain
        ``simulate_one``, or a GenerationSpec whose model is not vectorised,
        whose distance or acceptor has no device form, ... (``why_not``) --
        goes through the reference's per-candidate loop
        (sampler/base.py:172-214, singlecore.py:20-38): candidates one at a
        time until n are accepted, each candidate's transition, prior and
        distance still calling the device kernels where they have them (a
        batch of one).  With several ranks rank 0 runs the loop and the
        sample is broadcast, so every rank holds the same population."""
        why = getattr(simulate_one, "why_not", "")
        if not self.allow_per_candidate:
            raise TypeError("BatchedGPUSampler: this generation has no batched "
                            "form (" + (why or type(simulate_one).__name__)
                            + ") and allow_per_candidate=False")
        logger.warning("BatchedGPUSampler: per-candidate loop, orders of "
                       "magnitude slower than the batched path (%s)",
                       why or type(simulate_one).__name__)
        rank, ws = dd.world()
        res = None
        if rank == 0:
            sample = self._create_empty_sample()
            n_eval = 0
            while sample.n_accepted < n:
                if self.check_max_eval and n_eval >= max_eval:
                    break
                particle = simulate_one()
                n_eval += 1
                sample.append(particle)
            if sample.n_accepted < n:
                sample.ok = False
            res = (sample, n_eval)
        sample, n_eval = dd.broadcast_object(res)
        self.nr_evaluations_ = int(n_eval)
        self.last_stats = dict(rounds=0, evaluations=int(n_eval),
                               accepted=int(sample.n_accepted), per_candidate=True)
        return sample

    # ---- fused candidate rounds ------------------------------------------
    def _fused_round(self, spec, seed, gen, dev):
        """gpu.CandidateRound of this generation, or None when some piece has
        no fused form (custom simulator / distance, stochastic acceptor)."""
        if not self.fused or getattr(spec, "stochastic", None) is not None \
                or spec.distance is None or len(spec.param_names) > self.FUSED_MAX_DIM:
            return None
        if spec.transition is None and getattr(spec, "host_prior", None):
            return None     # t = 0 draws of host-leg coordinates: staged path
        sim = (spec.model.fused_simulator(dev)
               if hasattr(spec.model, "fused_simulator") else None)
        fp = (spec.distance.fused_pnorm(spec.t, spec.sum_stat_keys, dev)
              if hasattr(spec.distance, "fused_pnorm") else None)
        if sim is None or fp is None or len(spec.sum_stat_keys) > self.FUSED_MAX_STATS:
            return None
        prop = {}
        if spec.transition is not None:
            arrays = getattr(spec.transition, "proposal_arrays", None)
            if arrays is None:
                return None
            prop = arrays()
        src, a, sigma = sim
        wf, pval = fp
        fr = gpu.CandidateRound(len(spec.param_names), len(spec.sum_stat_keys),
                                spec.prior_kind, spec.prior_params, src, a,
                                sigma, spec.x0vec, wf, pval, seed, gen,
                                self.max_attempts, **prop)
        fr.src_host = getattr(spec.model, "src", None)   # host copy (_lazy_capable)
        return fr

    LAZY_KT = 4              # abc_candidate.h: the lazy head's coordinates

    def _lazy_capable(self, spec, fr):
        """Whether the fused round's early reject can take the lazy head
        (abc_candidate.h lazy_filter_ok): shared Cholesky factor, d and S
        beyond the head, p in {1, 2, inf}, the first 4 statistics reading
        theta_0..3, and unbounded priors (norm, laplace), whose support
        holds every proposal; the kernel re-checks the bound exactly."""
        s = fr.spec
        kinds = getattr(spec, "prior_kind_host", None)
        src = getattr(fr, "src_host", None)
        return (s.X is not None and not s.per_particle_L and s.d > self.LAZY_KT
                and s.S >= max(5, self.filter_min_stats) and s.p in (1.0, 2.0, math.inf)
                and kinds is not None
                and all(k in (PRIOR_KINDS["norm"], PRIOR_KINDS["laplace"])
                        for k in kinds)
                and src is not None and all(0 <= int(v) < self.LAZY_KT for v in src[:4]))

    # candidates per rank a first round may spend on spare: about what one
    # more round costs in fixed time (launch, scan, host read and the
    # loop's host work, ~0.2 ms) at ~2e10 candidates/s
    FIRST_ROUND_SPARE = 4_000_000

    def _fused_size(self, need, ws, rate, measured, S, record):
        """Candidates per rank for the next fused round: need / rate, with a
        6% margin once the rate was measured in this generation, capped by
        the launch and record budgets.  The generation's first round takes
        the previous generation's rate times its last drop (eps shrinks, so
        the rate keeps falling) plus a spare of up to 10%, bounded by what a
        second round would cost: small early generations then finish in one
        round, large ones add little.  Round sizes never change the result
        (candidates are keyed by their global index; the first `need`
        accepted in index order are kept)."""
        if self.batch_size is not None:
            return int(self.batch_size)
        r = rate if rate else 0.5
        if measured:
            mult = 1.06
        else:
            r *= self._acc_trend if rate else 1.0
            mult = 1.0 + min(0.1, self.FIRST_ROUND_SPARE * ws * max(r, 1e-12) / max(need, 1))
        b = need / max(r, 1e-12) * mult / ws + 4096
        cap = self.max_fused_batch_size
        if record:
            cap = min(cap, max(self.record_budget_bytes // (8 * S), 4096))
        return int(min(max(b, 4096), cap))

    def _limit_to_max_eval(self, B, max_eval, n_eval, ws):
        """With check_max_eval no round goes past max_eval evaluations
        (singlecore.py:25-31 checks before every simulation; with several
        ranks the overshoot is below one candidate per rank)."""
        if not self.check_max_eval or not np.isfinite(max_eval):
            return B
        left = int(math.ceil(max_eval)) - int(n_eval)
        return int(max(1, min(B, left // ws)))

    def _record_limit(self, S):
        self._records_truncated = False
        if self.record_device_budget_bytes is None:
            self._budget_capped = False
            return self.max_nr_recorded
        budget_rows = self.record_device_budget_bytes // (8 * max(S, 1))
        self._budget_capped = budget_rows < self.max_nr_recorded
        return min(self.max_nr_recorded, budget_rows)

    def _cap_records(self, rec_all, rec_left):
        """Keep only the first max_nr_recorded recorded candidates in global
        order (round-major, then rank); returns (rows per rank, rows left)."""
        if not np.isfinite(rec_left):
            return rec_all, rec_left
        out = np.zeros_like(rec_all)
        left = int(rec_left)
        for q in range(len(rec_all)):
            out[q] = min(int(rec_all[q]), left)
            left -= int(out[q])
        if left == 0 and out.sum() < rec_all.sum() and self._budget_capped:
            if not self._records_truncated:
                logger.warning("recorded sum stats exceed record_device_budget_bytes "
                               "(%d); keeping the first rows only",
                               self.record_device_budget_bytes)
            self._records_truncated = True
        return out, left

    def _sample_fused(self, n, fr, spec, max_eval, record, dev, rank, ws):
        """sample_until_n_accepted on fused rounds: per round one
        abc_candidates_round launch (accept bits -> indices of the first
        `need` accepted) and one host read; the kept rows are regenerated
        (abc_candidates_regen) bit-identical to the staged kernels."""
        torch = gpu.torch
        S = len(spec.sum_stat_keys)
        cols = {k: [] for k in ("theta", "lp", "dist", "x", "anc")}
        rec_x, rec_keeps, keeps = [], [], []
        arena, arena_off = None, 0
        # kept rows: pooled buffers filled through raw addresses (one set of
        # views per buffer, built after the loop)
        kept, kept_off, kept_segs = None, 0, []
        row_bytes = (8 * fr.d, 8, 8, 8 * S, 8)
        rec_left = self._record_limit(S)
        cut = None
        n_acc = n_eval = base = rounds = 0
        ok = True
        rate, measured = self._acc_rate, False
        tot_B = tot_cnt = 0
        filtered = reruns = 0
        while n_acc < n:
            if self.check_max_eval and n_eval >= max_eval:
                ok = False
                break
            need = n - n_acc
            B = self._limit_to_max_eval(self._fused_size(need, ws, rate, measured, S, record),
                                        max_eval, n_eval, ws)
            lo, _ = dd.rank_range(base, B, rank)
            rx = None
            if record and rec_left > 0:
                # recorded rows of consecutive rounds land back to back in one
                # arena (the next round starts after the rows this one keeps),
                # so the generation's matrix is a view, not a concatenation
                if arena is None or arena_off + B > arena.shape[0]:
                    arena = torch.empty((int(B * 1.25) + 4096, S), dtype=gpu.F64, device=dev)
                    arena_off = 0
                rx = arena[arena_off:arena_off + B]
            filt = (rate is not None and rate < self.filter_below and rx is None
                    and self._lazy_capable(spec, fr))
            filtered += int(filt)
            # the generation's first round takes the threshold on the device
            # (queued behind the quantile kernel, no host wait); later rounds
            # the host value, which has arrived by then
            thr = getattr(spec, "eps_device", None) if rounds == 0 else None
            if thr is not None:
                idx, cnt = fr.run(lo, B, 0.0, cap=need, filter=filt, rec_x=rx,
                                  eps_dev=thr[0], eps_scale=thr[1])
            else:
                idx, cnt = fr.run(lo, B, spec.eps, cap=need, filter=filt, rec_x=rx)
            pair = self._queue_pair(cnt, idx, min(need, B) - 1) if ws == 1 else None
            if ws == 1:
                n_keep = cnt
            else:
                # several ranks: the round's counts are all-gathered on the
                # device and this rank's share of the first `need` accepted
                # (global order) is computed there, so the regeneration is
                # queued before any host read, as on one rank
                gathered = dd.allgather_counts_device(cnt)
                n_keep = gpu.round_keep(gathered, need, rank)
                pair = self._queue_counts(gathered)
            # the kept rows' regeneration is queued before the count read,
            # sized on the device (the kept rows into the pooled buffer), so
            # the GPU is busy while the host reads the count
            if kept is None or kept_off + min(need, B) > kept[1]:
                if kept is not None and kept_off:
                    kept_segs.append((kept[0], kept_off))
                views = self._kept_buffers(min(need, B), fr.d, S, dev)
                kept = (views, views[0].shape[0], [v.data_ptr() for v in views])
                kept_off = 0
            fr.regen_into(lo, idx.data_ptr(), min(need, B),
                          [a + kept_off * b for a, b in zip(kept[2], row_bytes)],
                          n_dev=n_keep)
            if ws == 1:
                # one read: the count and the index of the need-th accepted
                cnt_local, pos_hint = self._wait_pair(pair)
                counts = dd.allgather_counts(cnt_local, dev)
            else:
                # the gathered counts, for the host's bookkeeping
                counts = self._wait_counts(pair)
            if thr is not None:
                spec.eps_device = None
                if np.isnan(thr[2].get()[0]):
                    # the select left the quantile undecided (knots in a tie
                    # run): the round ran at a NaN threshold and accepted
                    # nothing; run the same candidates again at the host
                    # value (the sort-based rerun, gpu.resolve_quantile).
                    # Every rank holds the same quantile, so all re-run
                    reruns += 1
                    spec.eps
                    continue
            keep = dd.cutoff(counts, need)
            total_keep = int(keep.sum())
            k_mine = int(keep[rank])
            rec_all = np.full(ws, B, dtype=np.int64)
            if n_acc + total_keep >= n:
                c_rank = int(np.nonzero(keep)[0][-1])
                if ws > 1:
                    cut = self._pending_cut(idx, keep, c_rank, rank, B, dev)
                    evaluated = 0
                else:
                    pos = pos_hint
                    evaluated = c_rank * B + pos + 1
                    rec_all[c_rank] = pos + 1
                    rec_all[c_rank + 1:] = 0
            else:
                evaluated = ws * B
            kept_off += k_mine              # regenerated before the count read
            if record and cut is not None and rx is not None:
                rec_x.append(rx)            # trimmed in _finish_cut
                rec_keeps.append(None)
            elif record:
                if rx is None:
                    rec_all = np.zeros(ws, dtype=np.int64)
                rec_all, rec_left = self._cap_records(rec_all, rec_left)
                rr = int(rec_all[rank])
                if rx is not None:
                    rec_x.append(rx[:rr])
                    arena_off += rr
                rec_keeps.append(rec_all)
            keeps.append(keep)
            n_acc += total_keep
            n_eval += evaluated
            base += ws * B
            rounds += 1
            tot_B += ws * B
            tot_cnt += int(counts.sum())
            rate, measured = max(int(counts.sum()) / float(ws * B), 1e-12), True
        if kept is not None and kept_off:
            kept_segs.append((kept[0], kept_off))
        for views, cnt in kept_segs:
            th, lp, anc, x, dist = (v[:cnt] for v in views)
            for k, v in zip(("theta", "lp", "dist", "x", "anc"), (th, lp, dist, x, anc)):
                cols[k].append(v)
        new_rate = max(tot_cnt / float(max(tot_B, 1)), 1e-12)
        if self._acc_rate:
            self._acc_trend = min(1.0, max(0.5, new_rate / self._acc_rate))
        self._acc_rate = new_rate
        if n_acc < n:
            ok = False
        out = self._assemble(spec, cols["theta"], cols["lp"], cols["dist"],
                             cols["x"], dev, fr.d, False, keeps,
                             cols["anc"] if spec.transition is not None else (),
                             cut=cut)
        if cut is not None:
            n_eval, rec_left = self._finish_cut(cut, n_eval, rec_left, rec_keeps,
                                                rec_x if record else None, None,
                                                rank, ws)
        self.nr_evaluations_ = int(n_eval)
        self.last_stats = dict(rounds=rounds, evaluations=int(n_eval),
                               accepted=int(n_acc), fused=True,
                               candidates=int(tot_B), filtered_rounds=filtered,
                               quantile_reruns=reruns,
                               records_truncated=self._records_truncated)
        recorded = None
        if record:
            recorded = self._gather_recorded(rec_x, rec_keeps, dev, ws)
            if recorded is None:
                recorded = torch.empty((0, S), dtype=gpu.F64, device=dev)
        elif out is not None:
            recorded = out.sum_stats
        return ColumnarSample(out, recorded, spec.sum_stat_keys, record,
                              ok and n_acc == n)

    def _queue_pair(self, cnt, idx, k):
        """Queue the round's (count, idx[k]) into a cached pinned pair (two
        async copies, no concatenation kernel, no allocation) and an event;
        _wait_pair reads it.  Work queued after the event (the kept rows'
        regeneration) runs while the host waits."""
        torch = gpu.torch
        if cnt.device.type != "cuda":              # host tensors (test doubles)
            return (int(cnt.reshape(-1)[0]), int(idx[k]))
        hp = getattr(self, "_pair_host", None)
        if hp is None:
            hp = self._pair_host = torch.empty(2, dtype=torch.int64, pin_memory=True)
            self._pair_ev = torch.cuda.Event()
        hp[0:1].copy_(cnt.reshape(1), non_blocking=True)
        hp[1:2].copy_(idx[k:k + 1], non_blocking=True)
        # the stream named by the tensor's device: record() with no stream
        # resolves the current device through torch.cuda.is_available (~40 us)
        self._pair_ev.record(torch.cuda.current_stream(cnt.device))
        return None

    def _wait_pair(self, queued):
        if queued is not None:
            return queued
        self._pair_ev.synchronize()
        return int(self._pair_host[0]), int(self._pair_host[1])

    def _queue_counts(self, gathered):
        """Queue the all-gathered round counts [ws] into a cached pinned
        buffer and an event (the multi-rank _queue_pair); _wait_counts
        reads them."""
        torch = gpu.torch
        if not gathered.is_cuda:
            return gathered.numpy().copy()
        ws = gathered.numel()
        hc = getattr(self, "_counts_host", None)
        if hc is None or hc.numel() != ws:
            hc = self._counts_host = torch.empty(ws, dtype=torch.int64, pin_memory=True)
            self._counts_ev = torch.cuda.Event()
        hc.copy_(gathered, non_blocking=True)
        self._counts_ev.record(torch.cuda.current_stream(gathered.device))
        return None

    def _wait_counts(self, queued):
        if queued is not None:
            return queued
        self._counts_ev.synchronize()
        return self._counts_host.numpy().copy()

    # population columns of the fused rounds are carved from pooled device
    # arenas: a generation's new population (kept by the History) would
    # otherwise need fresh allocations -- a hipMalloc and its host stall --
    # every generation
    _POOL_BYTES = 1 << 28

    def _kept_buffers(self, cap, d, S, dev):
        """theta [cap, d], lp, anc (int64), x [cap, S], dist as views of one
        pooled fp64 arena."""
        torch = gpu.torch
        pieces = (((cap, d), cap * d), ((cap,), cap), ((cap,), cap),
                  ((cap, S), cap * S), ((cap,), cap))
        need = sum(n_el + (-n_el) % 32 for _, n_el in pieces)   # 256-byte aligned
        pool, off = getattr(self, "_pool", (None, 0))
        if pool is None or pool.device != dev or off + need > pool.numel():
            pool = torch.empty(max(need, self._POOL_BYTES // 8), dtype=gpu.F64, device=dev)
            off = 0
        views = []
        for shape, n_el in pieces:
            views.append(pool[off:off + n_el].view(shape))
            off += n_el + (-n_el) % 32
        views[2] = views[2].view(torch.int64)
        self._pool = (pool, off)
        return tuple(views)

    def _gather_recorded(self, pieces, rec_keeps, dev, ws):
        """Concatenate this rank's recorded rows and, over several ranks,
        all-gather them back into global candidate-index order."""
        if not pieces:
            return None
        out = pieces[0] if len(pieces) == 1 else self._join_rows(pieces)
        if ws > 1:
            out = dd.allgather_rows_ordered([out.contiguous()], rec_keeps, dev)[0]
        return out.contiguous()

    @staticmethod
    def _join_rows(pieces):
        """Row blocks -> one [sum rows x S] tensor: a view when they lie back
        to back in one buffer (the fused rounds' record arena), else a copy."""
        torch = gpu.torch
        a = pieces[0]
        adjacent = all(
            p.dim() == 2 and p.is_contiguous() and p.shape[1] == a.shape[1]
            and p.untyped_storage().data_ptr() == a.untyped_storage().data_ptr()
            and p.data_ptr() == q.data_ptr() + q.numel() * q.element_size()
            for q, p in zip(pieces[:-1], pieces[1:]))
        if adjacent and a.is_contiguous():
            n = sum(p.shape[0] for p in pieces)
            return a.as_strided((n, a.shape[1]), a.stride())
        return torch.cat(pieces, 0)

    @staticmethod
    def _local_cutoff_pos(idx, k):
        return int(idx[int(k) - 1].item())

    @staticmethod
    def _pending_cut(idx, keep, c_rank, rank, B, dev):
        """The completing round of a multi-rank generation: the cut rank's
        local position of its last kept candidate stays on the device (no
        host read, no collective of its own) and rides in the packed row
        gather of _assemble; every other rank sends -1."""
        torch = gpu.torch
        if rank == c_rank:
            k = int(keep[c_rank])
            pos = idx[k - 1:k].to(gpu.F64)
        else:
            pos = torch.full((1,), -1.0, dtype=gpu.F64, device=dev)
        return dict(c_rank=c_rank, B=int(B), pos=pos)

    def _finish_cut(self, cut, n_eval, rec_left, rec_keeps, rec_x, rec_extra,
                    rank, ws):
        """Resolve the pending cutoff once _assemble has gathered the cut
        rank's position: evaluations up to the n-th accepted (global order),
        the last round's recorded rows per rank (capped like every round), and
        this rank's recorded pieces of that round trimmed to them."""
        c_rank, B = cut["c_rank"], cut["B"]
        pos = int(cut["gathered"][c_rank])
        n_eval += c_rank * B + pos + 1
        if rec_x is not None and rec_keeps and rec_keeps[-1] is None:
            rec_all = np.full(ws, B, dtype=np.int64)
            rec_all[c_rank] = pos + 1
            rec_all[c_rank + 1:] = 0
            rec_all, rec_left = self._cap_records(rec_all, rec_left)
            rr = int(rec_all[rank])
            rec_keeps[-1] = rec_all
            if rec_x and rec_x[-1].shape[0] != rr:
                rec_x[-1] = rec_x[-1][:rr]
            if rec_extra:
                rec_extra[-1] = tuple(None if a is None else a[:rr]
                                      for a in rec_extra[-1])
        return n_eval, rec_left

    def _proposal_round(self, spec, seed, gen, dev):
        """A proposal-only gpu.CandidateRound of this generation (dummy
        simulator / distance fields, never read), cached per generation:
        the staged path's proposals through the fused kernel's propose_one
        (ancestor table, support box computed once per launch; the same bits
        as gpu.propose).  None when the transition has no proposal arrays."""
        # keyed on the spec object itself (held here, so its id cannot be
        # reused by a later run's spec while the entry lives)
        if len(spec.param_names) > self.FUSED_MAX_DIM:
            return None     # d > 64: the transition's own (wide) proposal kernel
        key = (seed, gen)
        if getattr(self, "_prop_spec", None) is spec and self._prop_key == key:
            return self._prop_round
        arrays = None
        if spec.transition is not None:
            fn = getattr(spec.transition, "proposal_arrays", None)
            arrays = fn() if fn is not None else None
            if arrays is None:
                return None
        torch = gpu.torch
        z = torch.zeros(1, dtype=gpu.F64, device=dev)
        fr = gpu.CandidateRound(len(spec.param_names), 1, spec.prior_kind,
                                spec.prior_params, torch.zeros(1, dtype=torch.int32, device=dev),
                                z, z, z, z, 2.0, seed, gen, self.max_attempts,
                                **(arrays or {}))
        self._prop_spec, self._prop_key, self._prop_round = spec, key, fr
        return fr

    def _propose(self, spec, B, seed, gen, lo, d):
        fr = None
        if not (spec.transition is None and getattr(spec, "host_prior", None)):
            fr = self._proposal_round(spec, seed, gen, gpu.require_device())
        if fr is not None:
            # the prior log-density only for the rows kept (computed after
            # the kept-row gather in sample_until_n_accepted)
            th, lp, anc, att = fr.propose(lo, B, with_lp=False)
            return th, lp, (anc if spec.transition is not None else None), att
        if spec.transition is None:
            th, lp, _, att = gpu.propose(None, None, None, spec.prior_kind,
                                         spec.prior_params, seed, gen, lo, B,
                                         self.max_attempts, d)
            anc = None
        else:
            th, lp, anc, att = spec.transition.propose_device(
                B, spec.prior_kind, spec.prior_params, seed=seed,
                generation=gen, idx0=lo, max_attempts=self.max_attempts)
        return th, lp, anc, att

    @staticmethod
    def global_order(keeps):
        """Permutation from the rank-major all-gather (rank 0's rows of every
        round, then rank 1's, ...) to global candidate-index order (round
        major, then rank), from the per-round keep counts [rounds x ranks]."""
        k = np.asarray(keeps, dtype=np.int64).reshape(len(keeps), -1)
        if k.size == 0:
            return np.zeros(0, dtype=np.int64)
        rank_start = np.concatenate([[0], np.cumsum(k.sum(0))[:-1]])
        round_off = np.cumsum(k, axis=0) - k          # [rounds x ranks]
        starts = (rank_start[None, :] + round_off).ravel()   # round-major
        lens = k.ravel()
        tot = int(lens.sum())
        base = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]),
                         lens)
        return base + np.arange(tot, dtype=np.int64)

    @staticmethod
    def global_pieces(keeps):
        """The permutation of global_order as contiguous pieces (start, len)
        of the rank-major array, in global order (rounds x ranks pieces)."""
        k = np.asarray(keeps, dtype=np.int64).reshape(len(keeps), -1)
        if k.size == 0:
            return []
        rank_start = np.concatenate([[0], np.cumsum(k.sum(0))[:-1]])
        round_off = np.cumsum(k, axis=0) - k
        starts = (rank_start[None, :] + round_off).ravel()
        return [(int(a), int(n)) for a, n in zip(starts, k.ravel()) if n > 0]

    @staticmethod
    def reorder(t, pieces):
        """Rows of t in the order of the pieces (one concatenation)."""
        if len(pieces) <= 1:
            return t
        if all(a == b[0] + b[1] for b, (a, _) in zip(pieces[:-1], pieces[1:])) \
                and pieces[0][0] == 0:
            return t          # already in order
        return gpu.torch.cat([t[a:a + n] for a, n in pieces], 0)

    def _assemble(self, spec, acc_theta, acc_lp, acc_d, acc_x, dev, d,
                  all_accepted, keeps, acc_anc=(), acc_w=(), cut=None):
        rank, ws = dd.world()
        torch = gpu.torch
        def cat(lst):
            if len(lst) == 1:
                return lst[0]
            if lst[0].dim() == 2:
                return self._join_rows(lst)
            return self._join_rows([t.view(-1, 1) for t in lst]).view(-1)
        if acc_theta:
            theta, lp, dist, x = cat(acc_theta), cat(acc_lp), cat(acc_d), cat(acc_x)
        else:
            S = len(spec.sum_stat_keys)
            theta = torch.empty((0, d), dtype=gpu.F64, device=dev)
            lp = torch.empty(0, dtype=gpu.F64, device=dev)
            dist = torch.empty(0, dtype=gpu.F64, device=dev)
            x = torch.empty((0, S), dtype=gpu.F64, device=dev)
        # importance weights for this rank's accepted rows (smc.py:768-811);
        # a StochasticAcceptor's acceptance weights multiply in
        accw = cat(acc_w) if acc_w and len(acc_w) == len(acc_theta) else None
        if all_accepted:
            w = torch.ones(theta.shape[0], dtype=gpu.F64, device=dev)
        elif spec.transition is None:
            # t = 0: w = n_acc / n_per_param * prod(acceptance weights)
            w = (accw.contiguous() if accw is not None else
                 torch.ones(theta.shape[0], dtype=gpu.F64, device=dev))
        else:
            # ancestors of the accepted rows: population rows near them,
            # used by the x3 density kernel as exponent offsets
            anc = (cat(acc_anc) if acc_anc and
                   len(acc_anc) == len(acc_theta) else None)
            lt = spec.transition.logpdf_device(theta, hint=anc)
            hook, self.on_density_queued = self.on_density_queued, None
            if hook is not None:
                hook()
            hl = host_prior_logpdf(theta, getattr(spec, "host_prior", None))
            if hl is not None:
                lp = lp + hl      # the host-scipy leg's density factors
            w = gpu.importance_weights(lp, lt, spec.weight_scale,
                                       acc_w=None if accw is None else accw.contiguous())
        if ws > 1:
            # one packed all-gather; the rows come back in global
            # candidate-index order so the population (and every later draw
            # keyed on it) is the same for any number of ranks
            # (the cut rank's cutoff position rides in the same collective)
            parts = [theta, w, dist, x]
            extra = None if cut is None else cut["pos"]
            if len({a.dtype for a in parts}) == 1:
                got = dd.allgather_rows_ordered(parts, keeps, dev, extra=extra)
            else:
                got = [dd.allgather_rows_ordered([a], keeps, dev,
                                                 extra=extra if i == 0 else None)
                       for i, a in enumerate(parts)]
                if extra is not None:
                    got = ([got[0][0][0]] + [g[0] for g in got[1:]], got[0][1])
                else:
                    got = [g[0] for g in got]
            if extra is not None:
                got, cut["gathered"] = got
            theta, w, dist, x = got
        if theta.shape[0] == 0:
            return None
        return ColumnarParticles(theta.contiguous(), w.contiguous(),
                                 dist.contiguous(), x.contiguous(),
                                 spec.param_names, spec.sum_stat_keys, m=0)
