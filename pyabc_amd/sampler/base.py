# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""Sample / Sampler semantics (pyabc/sampler/base.py:8-233)."""
from abc import ABC, ABCMeta, abstractmethod
from typing import List

import numpy as np

from ..population import Particle, Population


class Sample:
    def __init__(self, record_rejected: bool = False, ok: bool = True):
        self._particles = []
        self.record_rejected = record_rejected
        self.ok = ok

    @property
    def all_sum_stats(self):
        return sum((p.accepted_sum_stats + p.rejected_sum_stats
                    for p in self._particles), [])

    def first_m_sum_stats(self, m):
        m = min(len(self._particles), m)
        return sum((p.accepted_sum_stats + p.rejected_sum_stats
                    for p in self._particles[:m]), [])

    def first_m_particles(self, m) -> List:
        m = min(len(self._particles), m)
        return self._particles[:m]

    @property
    def _accepted_particles(self) -> List[Particle]:
        return [p for p in self._particles if p.accepted]

    def append(self, particle: Particle):
        if particle.accepted or self.record_rejected:
            self._particles.append(particle)

    def __add__(self, other):
        sample = Sample(self.record_rejected)
        sample._particles = self._particles + other._particles
        return sample

    @property
    def n_accepted(self) -> int:
        return len(self._accepted_particles)

    def get_accepted_population(self) -> Population:
        return Population(self._accepted_particles)


class SampleFactory:
    def __init__(self, record_rejected: bool = False):
        self.record_rejected = record_rejected

    def __call__(self):
        return Sample(self.record_rejected)


def wrap_sample(f):
    """sampler/base.py:144-159: the accepted count must equal n when ok."""
    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False, show_progress=False):
        sample = f(self, n, simulate_one, max_eval, all_accepted,
                   show_progress)
        if sample.n_accepted != n and sample.ok:
            raise AssertionError(
                f"Expected {n} but got {sample.n_accepted} acceptances.")
        return sample
    return sample_until_n_accepted


class SamplerMeta(ABCMeta):
    def __init__(cls, name, bases, attrs):
        ABCMeta.__init__(cls, name, bases, attrs)
        cls.sample_until_n_accepted = wrap_sample(cls.sample_until_n_accepted)


class Sampler(ABC, metaclass=SamplerMeta):
    def __init__(self):
        self.nr_evaluations_ = 0
        self.sample_factory = SampleFactory(record_rejected=False)

    def _create_empty_sample(self) -> Sample:
        return self.sample_factory()

    @abstractmethod
    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False, show_progress=False):
        ...
