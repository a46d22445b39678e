"""Epsilon restatement (weighted quantile / QuantileEpsilon).

Test infrastructure only -- see ``oracle/__init__.py``.
"""
import numpy as np


def weighted_quantile(points, weights=None, alpha=0.5, kind=None):
    """pyabc/weighted_statistics.py:27-43.

    Sort ascending; cs = cumsum(w); q = interp(alpha, cs - w/2, sorted).
    With tied keys the result depends on the order of the tied entries'
    weights: the reference uses numpy's default (unstable introsort) order,
    reproduced with ``kind=None``; the device radix sort is stable, i.e.
    ``kind="stable"``.  Parity at exact ties is therefore pinned to the
    stable order only.
    """
    points = np.asarray(points, dtype=np.float64)
    order = np.argsort(points, kind=kind)
    p = points[order]
    if weights is None:
        w = np.ones(len(p)) / len(p)
    else:
        w = np.asarray(weights, dtype=np.float64)[order]
    cs = np.cumsum(w)
    return float(np.interp(alpha, cs - 0.5 * w, p))


def quantile_epsilon(distances, weights, alpha=0.5, multiplier=1.0,
                     weighted=True, kind=None):
    """pyabc/epsilon/epsilon.py:202-228 (``QuantileEpsilon._update``)."""
    d = np.asarray(distances, dtype=np.float64)
    if weighted:
        w = np.asarray(weights, dtype=np.float64).astype(float)
        w = w / w.sum()
    else:
        w = np.ones(len(d)) / len(d)
    return weighted_quantile(d, w, alpha, kind) * multiplier
