# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""Distance ABC (pyabc/distance/base.py:10-275), same interface."""
import json
from abc import ABC, abstractmethod


class Distance(ABC):
    def initialize(self, t, get_all_sum_stats, x_0=None):
        """Calibrate before the first generation (default: nothing)."""

    def configure_sampler(self, sampler):
        """Let the distance configure the sampler (default: nothing)."""

    def update(self, t, get_all_sum_stats) -> bool:
        return False

    @abstractmethod
    def __call__(self, x: dict, x_0: dict, t: int = None,
                 par: dict = None) -> float:
        ...

    def get_config(self) -> dict:
        return {"name": self.__class__.__name__}

    def to_json(self) -> str:
        return json.dumps(self.get_config())


class NoDistance(Distance):
    def __call__(self, x, x_0, t=None, par=None):
        raise Exception(
            f"{self.__class__.__name__} is not intended to be called.")


class IdentityFakeDistance(Distance):
    def __call__(self, x, x_0, t=None, par=None):
        return x


class AcceptAllDistance(Distance):
    def __call__(self, x, x_0, t=None, par=None):
        return -1


class SimpleFunctionDistance(Distance):
    def __init__(self, fun):
        super().__init__()
        self.fun = fun

    def __call__(self, x, x_0, t=None, par=None):
        return self.fun(x, x_0)

    def get_config(self):
        conf = super().get_config()
        try:
            conf["name"] = self.fun.__name__
        except AttributeError:
            try:
                conf["name"] = self.fun.__class__.__name__
            except AttributeError:
                pass
        return conf


def to_distance(maybe_distance):
    if maybe_distance is None:
        return NoDistance()
    if isinstance(maybe_distance, Distance):
        return maybe_distance
    return SimpleFunctionDistance(maybe_distance)
