# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""SingleCoreSampler (pyabc/sampler/singlecore.py:6-38): the per-candidate
loop over ``simulate_one``; each candidate's plugins still run through the
GPU kernels (batch of one)."""
import numpy as np

from .base import Sampler


class SingleCoreSampler(Sampler):
    def __init__(self, check_max_eval: bool = False):
        super().__init__()
        self.check_max_eval = check_max_eval

    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False, show_progress=False):
        nr_simulations = 0
        sample = self._create_empty_sample()
        for _ in range(n):
            while True:
                if self.check_max_eval and nr_simulations >= max_eval:
                    break
                new_sim = simulate_one()
                sample.append(new_sim)
                nr_simulations += 1
                if new_sim.accepted:
                    break
        self.nr_evaluations_ = nr_simulations
        if sample.n_accepted < n:
            sample.ok = False
        return sample
