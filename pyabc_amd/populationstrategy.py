# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""Population size strategies (pyabc/populationstrategy.py:22-261).

AdaptivePopulationSize runs its bootstrapped CV
estimates on the device: every calc_cv call is N_BOOTSTR x (rvs + fit +
N_test x n transition densities) through the same kernels as a generation.
"""
import copy
import json
import logging
import warnings

import numpy as np

logger = logging.getLogger("Adaptation")


class PopulationStrategy:
    def __init__(self, nr_calibration_particles: int = None,
                 nr_samples_per_parameter: int = 1):
        self.nr_calibration_particles = nr_calibration_particles
        if nr_samples_per_parameter != 1:
            warnings.warn(
                "A nr_samples_per_parameter != 1 is deprecated since version "
                "0.9.23, the parameter will be removed in a future release.",
                DeprecationWarning)
        self.nr_samples_per_parameter = nr_samples_per_parameter

    def update(self, transitions, model_weights, t=None):
        pass

    def __call__(self, t: int = None) -> int:
        raise NotImplementedError

    def get_config(self):
        return {"name": self.__class__.__name__,
                "nr_calibration_particles": self.nr_calibration_particles,
                "nr_samples_per_parameter": self.nr_samples_per_parameter}

    def to_json(self):
        return json.dumps(self.get_config())


class ConstantPopulationSize(PopulationStrategy):
    def __init__(self, nr_particles: int, nr_calibration_particles: int = None,
                 nr_samples_per_parameter: int = 1):
        super().__init__(nr_calibration_particles=nr_calibration_particles,
                         nr_samples_per_parameter=nr_samples_per_parameter)
        self.nr_particles = nr_particles

    def __call__(self, t: int = None) -> int:
        if t == -1 and self.nr_calibration_particles is not None:
            return self.nr_calibration_particles
        return self.nr_particles

    def get_config(self):
        config = super().get_config()
        config["nr_particles"] = self.nr_particles
        return config


class AdaptivePopulationSize(PopulationStrategy):
    """populationstrategy.py:131-233: choose the population size whose
    bootstrapped KDE coefficient of variation matches ``mean_cv``
    (Klinger & Hasenauer 2017)."""

    def __init__(self, start_nr_particles, mean_cv: float = 0.05,
                 max_population_size: int = np.inf,
                 min_population_size: int = 10,
                 nr_samples_per_parameter: int = 1, n_bootstrap: int = 10,
                 nr_calibration_particles: int = None):
        super().__init__(nr_calibration_particles=nr_calibration_particles,
                         nr_samples_per_parameter=nr_samples_per_parameter)
        self.start_nr_particles = start_nr_particles
        self.max_population_size = max_population_size
        self.min_population_size = min_population_size
        self.mean_cv = mean_cv
        self.n_bootstrap = n_bootstrap
        self.nr_particles = start_nr_particles

    def get_config(self):
        config = super().get_config()
        config["start_nr_particles"] = self.start_nr_particles
        config["max_population_size"] = self.max_population_size
        config["min_population_size"] = self.min_population_size
        config["mean_cv"] = self.mean_cv
        config["n_bootstrap"] = self.n_bootstrap
        return config

    def update(self, transitions, model_weights, t=None):
        from .cv.bootstrap import calc_cv
        from .transition.predict_population_size import \
            predict_population_size
        test_X = [trans.X for trans in transitions]
        test_w = [trans.w for trans in transitions]
        reference_nr_part = self.nr_particles
        cv_estimate = predict_population_size(
            reference_nr_part, self.mean_cv,
            lambda nr_particles: calc_cv(nr_particles, model_weights,
                                         self.n_bootstrap, test_w,
                                         transitions, test_X)[0])
        if not np.isnan(cv_estimate.n_estimated):
            self.nr_particles = max(min(int(cv_estimate.n_estimated),
                                        self.max_population_size),
                                    self.min_population_size)
        # the bootstrap draws come from each process's own numpy RNG: with
        # several ranks, rank 0's size is the one every rank samples
        self.nr_particles = _agree_across_ranks(int(self.nr_particles))
        self.cv_estimate_ = cv_estimate
        logger.info("Change nr particles {} -> {}".format(
            reference_nr_part, self.nr_particles))

    def __call__(self, t: int = None) -> int:
        if t == -1 and self.nr_calibration_particles is not None:
            return self.nr_calibration_particles
        return self.nr_particles


def _agree_across_ranks(n):
    """Rank 0's value on every rank of the default process group (no-op
    without one)."""
    from .sampler import distributed as dd
    rank, ws = dd.world()
    if ws == 1:
        return n
    import torch
    dev = (torch.device("cuda", torch.cuda.current_device())
           if torch.cuda.is_available() and dd.dist.get_backend() == "nccl"
           else torch.device("cpu"))
    return dd.broadcast_int(n, dev)


class ListPopulationSize(PopulationStrategy):
    """populationstrategy.py:236-261: ``values[t]`` for generation t.
    (The reference's get_config reads a non-existent ``population_values``
    attribute; the values are reported here.)"""

    def __init__(self, values, nr_calibration_particles: int = None,
                 nr_samples_per_parameter: int = 1):
        super().__init__(nr_calibration_particles=nr_calibration_particles,
                         nr_samples_per_parameter=nr_samples_per_parameter)
        self.values = values

    def get_config(self):
        config = super().get_config()
        config["population_values"] = self.values
        return config

    def __call__(self, t: int = None) -> int:
        if t == -1 and self.nr_calibration_particles is not None:
            return self.nr_calibration_particles
        return self.values[t]
