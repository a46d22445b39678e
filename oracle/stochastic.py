"""Stochastic acceptance restated in numpy / scipy (float64).

Test infrastructure only -- see ``oracle/__init__.py``.

  kernel values          pyabc/distance/kernel.py:207-226 (NormalKernel),
                         :285-303 (IndependentNormal), :361-378 (Laplace),
                         :426-445 (Binomial), :478-495 (Poisson),
                         :533-552 (NegativeBinomial)
  accept step            pyabc/acceptor/acceptor.py:434-476
  match_acceptance_rate  pyabc/epsilon/temperature.py:322-378
  EssScheme              pyabc/epsilon/temperature.py:686-742

The kernels evaluate scipy.stats exactly as the reference does, on a sum-stat
matrix (one row per simulation) instead of one dict.  The accept step replays
the device's uniform (Philox slot 0xFFFFFFF0, numpy's 53-bit double recipe)
in place of np.random.uniform.
"""
import numpy as np
import scipy.optimize
from scipy import stats

from .philox import philox4x32_10, uniform53

SLOT_ACCEPT = 0xFFFFFFF0


def kernel_values(kind, x, x0, par=None, cov=None, ret_log=True):
    """pdf(x_0 | x) for every row of x [B, K] (columns in kernel key order)
    against x0 [K]."""
    x = np.atleast_2d(np.asarray(x, dtype=float))
    x0 = np.asarray(x0, dtype=float)
    out = np.empty(x.shape[0])
    for b in range(x.shape[0]):
        if kind == "independent_normal":           # kernel.py:296-303
            var = np.asarray(par, dtype=float) * np.ones(x0.size)
            diff = x[b] - x0
            log_2_pi = np.sum(np.log(2) + np.log(np.pi) + np.log(var))
            squares = np.sum((diff ** 2) / var)
            v = -0.5 * (log_2_pi + squares)
        elif kind == "independent_laplace":        # kernel.py:371-378
            scale = np.asarray(par, dtype=float) * np.ones(x0.size)
            diff = x[b] - x0
            v = -(np.sum(np.log(2) + np.log(scale)) +
                  np.sum(np.abs(diff) / scale))
        elif kind == "normal":                     # kernel.py:221-226
            rv = stats.multivariate_normal(mean=np.zeros(x0.size), cov=cov)
            v = rv.logpdf(x[b] - x0)
        else:
            xi = np.asarray(x[b], dtype=int)
            ki = np.asarray(x0, dtype=int)
            if kind == "poisson":                  # kernel.py:490-495
                v = np.sum(stats.poisson.logpmf(k=ki, mu=xi))
            elif kind == "binomial":               # kernel.py:440-445
                v = np.sum(stats.binom.logpmf(k=ki, n=xi, p=par))
            elif kind == "negative_binomial":      # kernel.py:547-552
                v = np.sum(stats.nbinom.logpmf(k=ki, n=xi, p=par))
            else:
                raise ValueError(kind)
        out[b] = float(v)
    return out if ret_log else np.exp(out)


def accept_uniform(seed, generation, idx0, B):
    """The acceptance uniform of candidates idx0 .. idx0 + B - 1."""
    r = philox4x32_10(np.arange(idx0, idx0 + B, dtype=np.uint64),
                      SLOT_ACCEPT, generation, seed)
    return uniform53(r[:, 0], r[:, 1])


def stochastic_accept(dens, pdf_norm, temp, scale_log, apply_iw, u):
    """acceptor.py:453-474 vectorised: (accept mask, acceptance weight)."""
    dens = np.asarray(dens, dtype=float)
    with np.errstate(all="ignore"):
        if scale_log:
            acc = np.exp((dens - pdf_norm) * (1 / temp))
        else:
            acc = (dens / pdf_norm) ** (1 / temp)
        accept = acc >= u
        if apply_iw:
            w = acc / np.minimum(1, acc)
        else:
            w = np.ones_like(acc)
    w = np.where(acc == 0.0, 0.0, w)
    return accept, w


def match_acceptance_rate(weights, pds, pdf_norm, scale_log, target_rate):
    """temperature.py:343-378 (weights = t_pd / t_pd_prev, normalised
    here as in :333-334)."""
    weights = np.asarray(weights, dtype=float)
    weights = weights / np.sum(weights)
    pds = np.asarray(pds, dtype=float)

    def obj(b):
        beta = np.exp(b)
        if scale_log:
            acc_probs = np.exp((pds - pdf_norm) * beta)
        else:
            acc_probs = (pds / pdf_norm) ** beta
        acc_probs = np.minimum(acc_probs, 1.0)
        return np.sum(weights * acc_probs) - target_rate

    min_b = -100
    if obj(0) > 0:
        b_opt = 0
    elif obj(min_b) < 0:
        b_opt = min_b
    else:
        b_opt = scipy.optimize.bisect(obj, min_b, 0, maxiter=100000)
    return 1. / np.exp(b_opt)


def ess_temperature(pdfs, w, pdf_norm, scale_log, prev_temperature,
                    target_relative_ess=0.8):
    """temperature.py:710-742."""
    weights = np.array(w, dtype=float)
    pdfs = np.array(pdfs, dtype=float)
    values = np.exp(pdfs - pdf_norm) if scale_log else pdfs / pdf_norm
    weights /= np.sum(weights)
    target_ess = len(weights) * target_relative_ess
    beta_base = 0.0 if prev_temperature is None else 1. / prev_temperature

    def ess(beta):
        num = np.sum(weights * values ** beta) ** 2
        den = np.sum((weights * values ** beta) ** 2)
        return num / den

    def obj(beta):
        return (ess(beta) - target_ess) ** 2

    bounds = scipy.optimize.Bounds(lb=np.array([beta_base]),
                                   ub=np.array([1.]))
    ret = scipy.optimize.minimize(obj, x0=np.array([0.5 * (1 + beta_base)]),
                                  bounds=bounds)
    return float(1. / ret.x[0])
