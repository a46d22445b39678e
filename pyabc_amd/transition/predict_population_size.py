# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""Population size for a target KDE coefficient of variation.

Reference: pyabc/transition/predict_population_size.py:1-60.  Evaluates
calc_cv on range(n // 3, 2 n, n // 10) and inverts a fitted power law; each
calc_cv is a batch of device bootstraps (pyabc_amd/cv/bootstrap.py).
"""
import logging
from collections import namedtuple

from ..cv.powerlaw import fitpowerlaw

logger = logging.getLogger("CV Estimation")

CVEstimate = namedtuple("CVEstimate", "n_estimated n_samples_list cvs f popt")


def predict_population_size(current_pop_size: int, target_cv: float, calc_cv,
                            n_steps=10, first_step_factor=3) -> CVEstimate:
    if current_pop_size == 1:
        return CVEstimate(1, [], [], None, None)
    start = max(current_pop_size // first_step_factor, 1)
    stop = current_pop_size * 2
    step = max(current_pop_size // n_steps, 1)
    n_samples_list = list(range(start, stop, step))
    cvs = list(map(calc_cv, n_samples_list))
    try:
        popt, f, finv = fitpowerlaw(n_samples_list, cvs)
        return CVEstimate(finv(target_cv), n_samples_list, cvs, f, popt)
    except RuntimeError:
        logger.warning("Power law fit failed. Falling back to current nr "
                       "particles {}".format(current_pop_size))
        return CVEstimate(current_pop_size, n_samples_list, cvs, None, None)
