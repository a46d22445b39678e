"""Epsilon ABC (pyabc/epsilon/base.py:10-167)."""
import json
from abc import ABC, abstractmethod

import numpy as np


class Epsilon(ABC):
    def __init__(self):
        pass

    def initialize(self, t, get_weighted_distances, get_all_records,
                   max_nr_populations, acceptor_config):
        pass

    def configure_sampler(self, sampler):
        pass

    def update(self, t, get_weighted_distances, get_all_records,
               acceptance_rate, acceptor_config):
        pass

    @abstractmethod
    def __call__(self, t: int) -> float:
        ...

    def get_config(self):
        return {"name": self.__class__.__name__}

    def to_json(self):
        return json.dumps(self.get_config())


class NoEpsilon(Epsilon):
    def __call__(self, t):
        return np.nan
