"""Transition ABC (pyabc/transition/base.py:15-184), API-compatible.

Subclasses here keep their state on the GPU: ``fit`` uploads the population
once, ``pdf``/``rvs`` run HIP kernels, and ``fit_device``/``logpdf_device``/
``propose_device`` expose the device-resident entry points the batched
sampler drives without any host round trip.
"""
import copy
from abc import abstractmethod

import pandas as pd
from sklearn.base import BaseEstimator

from .exceptions import NotEnoughParticles
from .transitionmeta import TransitionMeta


class Transition(BaseEstimator, metaclass=TransitionMeta):
    NR_BOOTSTRAP = 5
    X = None
    w = None

    @abstractmethod
    def fit(self, X: pd.DataFrame, w) -> None:
        """Fit the perturbation kernel to the weighted population."""

    @abstractmethod
    def rvs_single(self) -> pd.Series:
        """One sample from the fitted kernel."""

    def rvs(self, size=None):
        if size is None:
            return self.rvs_single()
        return pd.DataFrame([self.rvs_single() for _ in range(size)])

    @abstractmethod
    def pdf(self, x):
        """Density of the fitted kernel at x (Series or DataFrame)."""

    def score(self, X, w):
        import numpy as np
        densities = self.pdf(X)
        return (np.log(densities) * w).sum()

    def no_meaningful_particles(self) -> bool:
        return len(self.X) == 0 or self.no_parameters

    # device tensors are immutable after fit(): share them on deepcopy
    # (ABCSMC deep-copies transitions every generation, smc.py:979).
    _SHARED = ()

    def __deepcopy__(self, memo):
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            if k in self._SHARED or k.startswith("_dev"):
                new.__dict__[k] = v
            else:
                new.__dict__[k] = copy.deepcopy(v, memo)
        return new


class DiscreteTransition(Transition):
    pass


__all__ = ["Transition", "DiscreteTransition", "NotEnoughParticles"]
