"""Distance restatement (PNormDistance, AdaptivePNormDistance).

Test infrastructure only -- see ``oracle/__init__.py``.
"""
import numpy as np


def pnorm(x, x0, w=None, f=None, p=2.0):
    """pyabc/distance/distance.py:79-105, vectorised over rows of ``x``.

    d = (sum_k |f_k w_k (x_k - x0_k)|^p)^(1/p); p = inf -> max_k.
    ``x`` is [M, S] in x_0 key order (distance.py:113-125).
    """
    x = np.atleast_2d(np.asarray(x, dtype=np.float64))
    x0 = np.asarray(x0, dtype=np.float64)
    S = x.shape[1]
    w = np.ones(S) if w is None else np.asarray(w, dtype=np.float64)
    f = np.ones(S) if f is None else np.asarray(f, dtype=np.float64)
    a = np.abs((f * w)[None, :] * (x - x0[None, :]))
    if p == np.inf:
        return a.max(1)
    return np.power(np.power(a, p).sum(1), 1.0 / p)


def standard_deviation(data):
    """pyabc/distance/scale.py:59-65 (np.std, ddof=0)."""
    return np.std(np.asarray(data, dtype=np.float64), axis=0)


def median_absolute_deviation(data):
    """pyabc/distance/scale.py:38-47: median(|x - median(x)|), numpy median
    (even n -> mean of the two middle values)."""
    data = np.asarray(data, dtype=np.float64)
    return np.median(np.abs(data - np.median(data, axis=0)), axis=0)


def adaptive_weights(X, scale_function="std", normalize_weights=True,
                     max_weight_ratio=None):
    """pyabc/distance/distance.py:263-348 (``_update``,
    ``_normalize_weights``, ``_bound_weights``) over all recorded sum stats
    X [R, S] (columns in x_0 key order).

    scale -> w = 0 if isclose(scale, 0) else 1/scale; w /= mean(w);
    optionally bound to ratio * min nonzero |w|.
    """
    X = np.asarray(X, dtype=np.float64)
    if scale_function in ("std", "standard_deviation"):
        scale = standard_deviation(X)
    elif scale_function in ("mad", "median_absolute_deviation"):
        scale = median_absolute_deviation(X)
    else:
        raise ValueError(scale_function)
    zero = np.isclose(scale, 0)
    w = np.where(zero, 0.0, 1.0 / np.where(zero, 1.0, scale))
    if normalize_weights:
        w = w / np.mean(w)
    if max_weight_ratio is not None:
        min_abs = np.min(np.abs(w[w != 0]))
        big = np.abs(w) / min_abs > max_weight_ratio
        w = np.where(big, np.sign(w) * max_weight_ratio * min_abs, w)
    return w
