"""Replay of the batched sampler's counter-based draws in numpy (float64).

Test infrastructure only -- see ``oracle/__init__.py``.  The semantics are
those of pyabc/smc.py:610-662 (_generate_valid_proposal: theta =
Transition.rvs(), re-draw while the prior density is 0) and
pyabc/transition/multivariatenormal.py:85-97 (ancestor ~ Cat(w) by inverse
CDF, theta = X_j + N(0, Sigma)); only the random stream differs from the
reference (numpy MT19937 there, Philox keyed by the global candidate index
here), so the device and this replay agree draw for draw.
"""
import numpy as np
from scipy import stats

from .philox import philox4x32_10, uniform01, uniform53, normal_pairs

SLOTS_PER_ATTEMPT = 65536
SLOT_PERTURB = 1
SLOT_PRIOR = 32
SLOT_SIM = 0x40000000

KIND = {"flat": -1, "norm": 0, "uniform": 1, "expon": 2, "laplace": 3,
        "lognorm": 4, "gamma": 5, "beta": 6}


def normals(index, slot0, n, generation, seed):
    """n normals per candidate: normal q from slot slot0 + q // 4."""
    index = np.asarray(index, dtype=np.uint64)
    out = np.empty((len(index), n))
    for q in range(0, n, 4):
        r = philox4x32_10(index, slot0 + q // 4, generation, seed)
        a0, a1 = normal_pairs(r[:, 0], r[:, 1])
        b0, b1 = normal_pairs(r[:, 2], r[:, 3])
        block = np.stack([a0, a1, b0, b1], axis=1)
        out[:, q:q + 4] = block[:, :min(4, n - q)]
    return out


def perturbation_normals(index, slot0, n, generation, seed, anc_words):
    """The n perturbation normals of one attempt (pyabc_amd/csrc/
    abc_candidate.h perturb_words): normals 0, 1 from the ancestor draw's
    unused words 2, 3 (anc_words [B, 4]); normals 2 q' + 2, 2 q' + 3 from half
    q' & 1 of slot slot0 + q' // 2."""
    index = np.asarray(index, dtype=np.uint64)
    out = np.empty((len(index), n))
    a0, a1 = normal_pairs(anc_words[:, 2], anc_words[:, 3])
    out[:, 0] = a0
    if n > 1:
        out[:, 1] = a1
    if n > 2:
        out[:, 2:] = normals(index, slot0, n - 2, generation, seed)
    return out


def prior_logpdf(theta, kinds, params):
    """Product prior in log space with scipy's closed-support pdfs."""
    theta = np.atleast_2d(theta)
    lp = np.zeros(len(theta))
    with np.errstate(divide="ignore"):
        for k, (kind, p) in enumerate(zip(kinds, params)):
            x = theta[:, k]
            if kind == "flat":
                continue
            if kind == "norm":
                lp += stats.norm.logpdf(x, p[0], p[1])
            elif kind == "uniform":
                lp += np.log(stats.uniform.pdf(x, p[0], p[1]))
            elif kind == "expon":
                lp += np.log(stats.expon.pdf(x, p[0], p[1]))
            elif kind == "laplace":
                lp += stats.laplace.logpdf(x, p[0], p[1])
            elif kind == "lognorm":
                lp += np.log(stats.lognorm.pdf(x, p[0], p[1], p[2]))
            elif kind == "gamma":
                lp += np.log(stats.gamma.pdf(x, p[0], p[1], p[2]))
            elif kind == "beta":
                lp += np.log(stats.beta.pdf(x, p[0], p[1], p[2], p[3]))
            else:
                raise ValueError(kind)
    return lp


def propose_local(X, w, chol, seed, generation, idx0, B, kinds=None, params=None,
                  max_attempts=1000):
    """Device abc_local_propose replayed (LocalTransition.rvs,
    pyabc/transition/local_transition.py:141-145: j ~ Cat(w), theta ~
    N(X_j, cov_j)): theta = X_j + chol_j n with the per-particle Cholesky
    factor chol [N, d, d]; same Philox streams and re-draw loop as
    propose_mvn."""
    return propose_mvn(X, w, chol, seed, generation, idx0, B, kinds, params,
                       max_attempts, per_particle=True)


def propose_mvn(X, w, L, seed, generation, idx0, B, kinds=None, params=None,
                max_attempts=1000, per_particle=False):
    """Device abc_propose replayed: returns theta, prior logpdf, ancestor,
    attempts."""
    X = np.asarray(X, dtype=np.float64)
    N, d = X.shape
    cdf = np.cumsum(np.asarray(w, dtype=np.float64))
    total = cdf[-1]
    kinds = kinds or ["flat"] * d
    params = params if params is not None else np.zeros((d, 4))
    idx = np.arange(idx0, idx0 + B, dtype=np.uint64)
    theta = np.empty((B, d))
    lp = np.full(B, -np.inf)
    anc = np.empty(B, dtype=np.int64)
    att = np.full(B, max_attempts + 1, dtype=np.int64)
    todo = np.ones(B, dtype=bool)
    for a in range(max_attempts):
        if not todo.any():
            break
        ii = idx[todo]
        s0 = a * SLOTS_PER_ATTEMPT
        r = philox4x32_10(ii, s0, generation, seed)
        u = uniform53(r[:, 0], r[:, 1])
        j = np.minimum(np.searchsorted(cdf, u * total, side="right"), N - 1)
        n = perturbation_normals(ii, s0 + SLOT_PERTURB, d, generation, seed, r)
        if per_particle:
            th = X[j] + np.einsum("bkq,bq->bk", np.asarray(L)[j], n)
        else:
            th = X[j] + n @ np.asarray(L).T
        l = prior_logpdf(th, kinds, params)
        pos = np.nonzero(todo)[0]
        theta[pos], lp[pos], anc[pos] = th, l, j
        ok = l > -np.inf
        att[pos[ok]] = a + 1
        todo[pos[ok]] = False
    return theta, lp, anc, att


def prior_uniforms(index, att, k, generation, seed):
    """The (0, 1) uniform of candidate `index`'s prior stream for dimension
    k in the attempt it accepted (device abc_prior_uniforms): words 0..1 of
    slot (att - 1) * 65536 + SLOT_PRIOR + 512 k, 53 bits plus a half.  An
    ABC_PRIOR_HOST coordinate's t = 0 draw is scipy's ppf of it."""
    index = np.asarray(index, dtype=np.uint64)
    att = np.maximum(np.asarray(att, dtype=np.int64) - 1, 0)
    out = np.empty(index.shape)
    for a in np.unique(att):
        sel = att == a
        r = philox4x32_10(index[sel], int(a) * SLOTS_PER_ATTEMPT + SLOT_PRIOR + 512 * k,
                          generation, seed)
        hi = (r[:, 0] >> np.uint32(5)).astype(np.float64)
        lo = (r[:, 1] >> np.uint32(6)).astype(np.float64)
        out[sel] = (hi * 67108864.0 + lo + 0.5) / 9007199254740992.0
    return out


def simulate_linear_gaussian(theta, src, a, sigma, seed, generation, idx0):
    """x[b, k] = a[k] theta[b, src[k]] + sigma[k] n_k (normal k of the
    candidate's simulation stream)."""
    theta = np.atleast_2d(theta)
    B = len(theta)
    S = len(src)
    idx = np.arange(idx0, idx0 + B, dtype=np.uint64)
    n = normals(idx, SLOT_SIM, S, generation, seed)
    return np.asarray(a)[None, :] * theta[:, np.asarray(src)] + \
        np.asarray(sigma)[None, :] * n
