"""Transition restatement (MultivariateNormalTransition, LocalTransition).

Test infrastructure only -- see ``oracle/__init__.py``.
"""
import numpy as np

LOG_2PI = np.log(2 * np.pi)


def smart_cov(X, w):
    """pyabc/transition/util.py:4-16 -- weighted sample covariance.

    One sample -> ``diag(|x_0|)``; otherwise ``np.cov(X, aweights=w,
    rowvar=False)`` which equals sum_i w_i (x_i - xbar)(x_i - xbar)^T /
    (1 - sum_i w_i^2) for normalised w.
    """
    X = np.asarray(X, dtype=np.float64)
    if X.shape[0] == 1:
        return np.diag(np.abs(X[0]))
    w = np.asarray(w, dtype=np.float64)
    wn = w / w.sum()
    mean = wn @ X
    D = X - mean
    cov = (D * wn[:, None]).T @ D / (1.0 - (wn ** 2).sum())
    return np.atleast_2d(cov)


def silverman_rule_of_thumb(n_samples, dimension):
    """pyabc/transition/multivariatenormal.py:27-37."""
    return (4 / n_samples / (dimension + 2)) ** (1 / (dimension + 4))


def psd_decompose(cov):
    """scipy.stats._multivariate._PSD (scipy 1.15.3) as used by
    ``st.multivariate_normal(cov, allow_singular=True)``
    (pyabc/transition/multivariatenormal.py:83).

    Returns U (d x r whitening: cov^+ = U U^T), log pseudo-determinant,
    rank r, null-space basis V (d x (d-r)) and the support tolerance.
    Eigenvalue cutoff: 1e6 * eps_f64 * max|s| (``_eigvalsh_to_eps``).
    """
    cov = np.atleast_2d(np.asarray(cov, dtype=np.float64))
    s, u = np.linalg.eigh(cov)
    eps = 1e6 * np.finfo(np.float64).eps * np.max(np.abs(s))
    keep = s > eps
    U = u[:, keep] / np.sqrt(s[keep])
    return dict(U=U, log_pdet=float(np.sum(np.log(s[keep]))),
                rank=int(keep.sum()), V=u[:, ~keep], support_tol=1e3 * eps)


def mvn_fit(X, w, scaling=1.0, bandwidth_selector=silverman_rule_of_thumb):
    """pyabc/transition/multivariatenormal.py:72-83 (+ transitionmeta.py:8-21).

    Returns the perturbation covariance Sigma = C * bw^2 * scaling and the
    normalised weights (the reference normalises ``w`` in place when
    ``not isclose(sum, 1)``).
    """
    X = np.asarray(X, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64).copy()
    if len(X) == 0:
        raise ValueError("NotEnoughParticles")
    if not np.isclose(w.sum(), 1):
        w /= w.sum()
    C = smart_cov(X, w)
    dim = C.shape[0]
    ess = 1 / (w ** 2).sum()
    bw = bandwidth_selector(ess, dim)
    return C * bw ** 2 * scaling, w


def mvn_logpdf(x, X, w, cov, block=256):
    """pyabc/transition/multivariatenormal.py:99-113, in log space.

    dens(x_i) = sum_j w_j N(x_i - X_j; 0, cov) with scipy's singular-cov
    semantics: pairs whose deviation leaves the support get density 0.
    Restated as log dens = -(r log 2pi + log pdet)/2 + LSE_j(log w_j
    - |(x_i - X_j) U|^2 / 2).
    """
    x = np.atleast_2d(np.asarray(x, dtype=np.float64))
    X = np.asarray(X, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64)
    p = psd_decompose(cov)
    U, r = p["U"], p["rank"]
    norm = -0.5 * (r * LOG_2PI + p["log_pdet"])
    Y = X @ U
    Z = x @ U
    with np.errstate(divide="ignore"):
        logw = np.log(w)
    out = np.empty(len(x))
    singular = r < X.shape[1]
    if singular:
        XV = X @ p["V"]
        xV = x @ p["V"]
    for b in range(0, len(x), block):
        zb = Z[b:b + block]
        q = logw[None, :] - 0.5 * ((zb[:, None, :] - Y[None, :, :]) ** 2).sum(2)
        if singular:
            res = np.linalg.norm(xV[b:b + block, None, :] - XV[None, :, :],
                                 axis=-1)
            q = np.where(res < p["support_tol"], q, -np.inf)
        m = q.max(1)
        with np.errstate(invalid="ignore"):
            s = np.exp(q - np.where(np.isfinite(m), m, 0)[:, None]).sum(1)
        out[b:b + block] = np.where(np.isfinite(m), m + np.log(s), -np.inf)
    return out + norm


def mvn_pdf(x, X, w, cov):
    return np.exp(mvn_logpdf(x, X, w, cov))


def local_k(n, dim, k=None, k_fraction=0.25):
    """pyabc/transition/local_transition.py:60-75 (``k`` property)."""
    if k_fraction is not None:
        k_ = int(k_fraction * n)
    else:
        k_ = k
    return max([k_, 10, dim])


def _local_cov(X, w, i, nq, d, scaling, EPS):
    """Covariance of particle i (local_transition.py:77-96, 125-139) from its
    nq - 1 nearest neighbours (ties by index), EPS loop of :112-123."""
    n = len(X)
    d2 = ((X - X[i]) ** 2).sum(1)
    order = np.lexsort((np.arange(n), d2))[:nq]
    if nq > 1:
        nb = order[1:]
        deltas = X[nb] - X[i]
        lw = w[nb]
    else:
        deltas = np.abs(X)
        lw = np.array([1.0])
    cov = smart_cov(deltas, lw / lw.sum())
    if np.abs(cov.sum()) == 0:
        for kd in range(d):
            cov[kd, kd] = np.abs(X[0, kd])
    cov = cov * scaling
    det = np.linalg.det(cov)
    while det <= 0:
        cov += np.identity(d) * EPS
        det = np.linalg.det(cov)
    return cov


def local_fit(X, w, k=None, k_fraction=0.25, scaling=1.0, EPS=1e-3, rows=None):
    """pyabc/transition/local_transition.py:77-96, 112-139.

    k+1 nearest neighbours per particle (column 0 = self is dropped), local
    weighted covariance of the neighbour offsets (weights renormalised over
    the neighbours), ``diag(|X[0]|)`` fallback for an all-zero covariance,
    scaled; then ``while det <= 0: cov += EPS * I``.  Neighbour order: by
    distance, ties by index (cKDTree's tie order is unspecified -- parity at
    exact ties is unpinned).  rows: only these particles (each costs one
    O(N log N) sort, so a random subset checks a large population).
    """
    X = np.asarray(X, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64).copy()
    if not np.isclose(w.sum(), 1):
        w /= w.sum()
    n, d = X.shape
    kk = local_k(n, d, k, k_fraction)
    nq = min(kk + 1, n)
    rows = np.arange(n) if rows is None else np.asarray(rows)
    covs = np.empty((len(rows), d, d))
    for o, i in enumerate(rows):
        covs[o] = _local_cov(X, w, int(i), nq, d, scaling, EPS)
    inv = np.linalg.inv(covs)
    dets = np.linalg.det(covs)
    normalization = np.sqrt((2 * np.pi) ** d * dets)
    return dict(covs=covs, inv_covs=inv, dets=dets, normalization=normalization,
                w=w, k=kk)


def local_pdf(x, X, fit):
    """pyabc/transition/local_transition.py:98-110: np.average over j of
    exp(-d_j^T inv_j d_j / 2) / normalization_j with weights w."""
    x = np.atleast_2d(np.asarray(x, dtype=np.float64))
    X = np.asarray(X, dtype=np.float64)
    out = np.empty(len(x))
    w = fit["w"]
    for i in range(len(x)):
        dist = X - x[i]
        md = np.einsum("ij,ijk,ik->i", dist, fit["inv_covs"], dist)
        out[i] = np.average(np.exp(-.5 * md) / fit["normalization"], weights=w)
    return out


def local_logpdf(x, X, fit):
    with np.errstate(divide="ignore"):
        return np.log(local_pdf(x, X, fit))
