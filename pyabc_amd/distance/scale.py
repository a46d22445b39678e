"""Scale functions for AdaptivePNormDistance (pyabc/distance/scale.py).

``standard_deviation`` and ``median_absolute_deviation`` are the two the
adaptive distance evaluates on the GPU over the recorded [R x S] sum-stat
matrix (abc_column_std / abc_column_mad).  Called on a plain list (the
reference signature ``f(data=list, x_0=float)``) they evaluate one column
through the same kernels.
"""
import numpy as np


def _column(data):
    from .. import gpu
    return gpu.as_dev(np.asarray(data, dtype=np.float64).reshape(-1, 1))


def median_absolute_deviation(data, **kwargs):
    """scale.py:38-47: median(|x - median(x)|)."""
    from .. import gpu
    return float(gpu.column_mad(_column(data)).cpu()[0])


median_absolute_deviation.device_kernel = "mad"


def standard_deviation(data, **kwargs):
    """scale.py:59-65: np.std."""
    from .. import gpu
    return float(gpu.column_std(_column(data)).cpu()[0])


standard_deviation.device_kernel = "std"


def mean_absolute_deviation(data, **kwargs):
    data = np.array(data)
    return np.mean(np.abs(data - np.mean(data)))


def bias(data, x_0, **kwargs):
    return np.abs(np.mean(data) - x_0)


def root_mean_square_deviation(data, x_0, **kwargs):
    return np.sqrt(bias(data, x_0) ** 2 + np.std(data) ** 2)


def median_absolute_deviation_to_observation(data, x_0, **kwargs):
    return np.median(np.abs(np.array(data) - x_0))


def mean_absolute_deviation_to_observation(data, x_0, **kwargs):
    return np.mean(np.abs(np.array(data) - x_0))


def combined_median_absolute_deviation(data, x_0, **kwargs):
    return (median_absolute_deviation(data)
            + median_absolute_deviation_to_observation(data, x_0))


def combined_mean_absolute_deviation(data, x_0, **kwargs):
    return (mean_absolute_deviation(data)
            + mean_absolute_deviation_to_observation(data, x_0))


def standard_deviation_to_observation(data, x_0, **kwargs):
    return np.std(np.abs(np.array(data) - x_0))


def span(data, **kwargs):
    return max(data) - min(data)


def mean(data, **kwargs):
    return np.mean(data)


def median(data, **kwargs):
    return np.median(data)
