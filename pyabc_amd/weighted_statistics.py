# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""Weighted statistics (pyabc/weighted_statistics.py:13-83), host versions
for the per-particle API; the generation engine uses the device kernels
(abc_weighted_quantile, pyabc_amd.gpu)."""
from functools import wraps

import numpy as np


def weight_checked(function):
    @wraps(function)
    def function_with_checking(points, weights=None, **kwargs):
        if weights is not None and not np.isclose(weights.sum(), 1):
            raise AssertionError(f"Weights not normalized: {weights.sum()}.")
        return function(points, weights, **kwargs)
    return function_with_checking


@weight_checked
def weighted_quantile(points, weights=None, alpha=0.5):
    sorted_indices = np.argsort(points)
    points = points[sorted_indices]
    if weights is None:
        weights = np.ones(len(points)) / len(points)
    else:
        weights = weights[sorted_indices]
    cs = np.cumsum(weights)
    return np.interp(alpha, cs - 0.5 * weights, points)


@weight_checked
def weighted_median(points, weights):
    return weighted_quantile(points, weights, alpha=0.5)


@weight_checked
def weighted_mean(points, weights):
    return (points * weights).sum()


@weight_checked
def weighted_std(points, weights):
    mean = weighted_mean(points, weights)
    return np.sqrt(((points - mean) ** 2 * weights).sum())


def effective_sample_size(weights):
    weights = np.array(weights)
    return np.sum(weights) ** 2 / np.sum(weights ** 2)
