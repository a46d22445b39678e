"""Bootstrapped KDE coefficient of variation (CPU restatement).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

pyabc/cv/bootstrap.py:6-41 (weights) and :44-110 (calc_cv); the population
size search of transition/predict_population_size.py:12-60 with the power law
of cv/powerlaw.py:1-17.
"""
import numpy as np

from .transition import mvn_fit, mvn_pdf


def bootstrap_variation(dens, w, scale=1.0):
    """bootstrap.py:86-108 for one model: dens [B, N] bootstrapped densities
    at the test points -> (variation [N] = std/mean over axis 0 with ddof 0,
    as scipy.stats.variation; cv = sum(variation * scale * w))."""
    dens = np.asarray(dens, dtype=np.float64)
    mean = dens.mean(axis=0)
    with np.errstate(divide="ignore", invalid="ignore"):
        var = dens.std(axis=0) / mean
    return var, float((var * scale * np.asarray(w)).sum())


def mvn_bootstrap_densities(samples, X_test):
    """bootstrap.py:36-40 with MultivariateNormalTransition: each bootstrap
    sample set [n, d] is fitted with uniform weights and its density taken
    at the test points."""
    out = []
    for S in samples:
        n = len(S)
        cov, w = mvn_fit(S, np.ones(n) / n)
        out.append(mvn_pdf(X_test, S, w, cov))
    return np.array(out)


def mvn_rvs(X, w, cov, n, rng):
    """multivariatenormal.py:85-91 (size=n): ancestors ~ Cat(w), plus
    N(0, cov) noise (numpy Generator here; the reference uses the legacy
    global RandomState, so draws agree in distribution only)."""
    idx = rng.choice(len(X), size=n, p=w)
    return X[idx] + rng.multivariate_normal(np.zeros(X.shape[1]), cov, size=n)


def mvn_calc_cv(n, X, w, n_bootstrap, rng):
    """bootstrap.py:44-110 for one MultivariateNormalTransition fitted to
    (X, w), test points = its own particles with their weights."""
    cov, w = mvn_fit(X, w)
    samples = [mvn_rvs(X, w, cov, n, rng) for _ in range(n_bootstrap)]
    return bootstrap_variation(mvn_bootstrap_densities(samples, X), w)[1]
