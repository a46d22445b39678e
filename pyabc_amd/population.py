"""Particles and populations (pyabc/population.py:19-289).

``Population`` keeps the reference's list-of-Particle interface, and adds a
columnar, device-resident form built by the batched sampler: theta [n, d],
weights [n], distances [n] and summary statistics [n, S] stay on the GPU;
``Particle`` objects are materialised only if a caller asks for them.
"""
import logging
from typing import Callable, List

import numpy as np
import pandas as pd

from .parameters import Parameter

logger = logging.getLogger("Population")


class Particle:
    def __init__(self, m: int, parameter: Parameter, weight: float,
                 accepted_sum_stats: List[dict], accepted_distances: List[float],
                 rejected_sum_stats: List[dict] = None,
                 rejected_distances: List[float] = None,
                 accepted: bool = True):
        self.m = m
        self.parameter = parameter
        self.weight = weight
        self.accepted_sum_stats = accepted_sum_stats
        self.accepted_distances = accepted_distances
        self.rejected_sum_stats = rejected_sum_stats or []
        self.rejected_distances = rejected_distances or []
        self.accepted = accepted


class ColumnarParticles:
    """Device columns of an accepted population (single model m)."""

    def __init__(self, theta, weights, distances, sum_stats, param_names,
                 sum_stat_keys, m=0):
        self.theta = theta              # [n, d] float64 device
        self.weights = weights          # [n] float64 device
        self.distances = distances      # [n] float64 device
        self.sum_stats = sum_stats      # [n, S] float64 device
        self.param_names = list(param_names)
        self.sum_stat_keys = list(sum_stat_keys)
        self.m = m

    def __len__(self):
        return int(self.theta.shape[0])


class WeightedDistances:
    """DataFrame-like (``.distance``, ``.w``) view that also carries the
    device tensors, so QuantileEpsilon stays on the GPU."""

    def __init__(self, distances, w):
        self.device_distance = distances
        self.device_w = w
        self._df = None

    def _frame(self):
        if self._df is None:
            self._df = pd.DataFrame({"distance": self.device_distance.cpu().numpy(),
                                     "w": self.device_w.cpu().numpy()})
        return self._df

    def __getattr__(self, item):
        return getattr(self._frame(), item)

    def __getitem__(self, item):
        return self._frame()[item]

    def __len__(self):
        return int(self.device_distance.numel())


class Population:
    def __init__(self, particles: List[Particle] = None, columns=None):
        if columns is not None:
            self._cols = columns
            self._list = None
            from . import gpu
            stats = gpu.normalize_weights(columns.weights)
            self._model_probabilities = {columns.m: 1.0}
            self._stats = stats
            return
        self._cols = None
        self._list = particles.copy()
        self._model_probabilities = None
        self._normalize_weights()

    @classmethod
    def from_columns(cls, columns: ColumnarParticles):
        return cls(columns=columns)

    @property
    def columns(self):
        return self._cols

    def __len__(self):
        return len(self._cols) if self._cols is not None else len(self._list)

    def _materialise(self):
        if self._list is None:
            c = self._cols
            th = c.theta.cpu().numpy()
            w = c.weights.cpu().numpy()
            dist = c.distances.cpu().numpy()
            ss = c.sum_stats.cpu().numpy() if c.sum_stats is not None else None
            self._list = [
                Particle(m=c.m,
                         parameter=Parameter(dict(zip(c.param_names, th[i]))),
                         weight=float(w[i]),
                         accepted_sum_stats=[dict(zip(c.sum_stat_keys, ss[i]))]
                         if ss is not None else [{}],
                         accepted_distances=[float(dist[i])])
                for i in range(len(c))]
        return self._list

    def get_list(self) -> List[Particle]:
        return self._materialise().copy()

    def _normalize_weights(self):
        store = self.to_dict()
        model_total_weights = {m: sum(particle.weight for particle in plist)
                               for m, plist in store.items()}
        population_total_weight = sum(model_total_weights.values())
        self._model_probabilities = {
            m: w / population_total_weight
            for m, w in model_total_weights.items()}
        for m in store:
            model_total_weight = model_total_weights[m]
            for particle in store[m]:
                particle.weight /= model_total_weight

    def update_distances(self, distance_to_ground_truth: Callable):
        for particle in self._materialise():
            for i in range(len(particle.accepted_distances)):
                particle.accepted_distances[i] = distance_to_ground_truth(
                    particle.accepted_sum_stats[i], particle.parameter)
        if self._cols is not None:
            from . import gpu
            d = np.array([p.accepted_distances[0] for p in self._list])
            self._cols.distances = gpu.as_dev(d, device=self._cols.theta.device)

    def update_distances_device(self, distance, x0vec, t):
        """Batched re-evaluation of the accepted distances (population.py:
        147-162) after the distance changed: one abc_pnorm launch."""
        c = self._cols
        c.distances = distance.device_call(c.sum_stats, x0vec, t,
                                           c.sum_stat_keys)
        self._list = None

    def get_model_probabilities(self) -> dict:
        return self._model_probabilities

    def get_weighted_distances(self):
        if self._cols is not None:
            # single model: model probability 1
            return WeightedDistances(self._cols.distances, self._cols.weights)
        rows = []
        for particle in self._list:
            model_probability = self._model_probabilities[particle.m]
            for distance in particle.accepted_distances:
                rows.append({'distance': distance,
                             'w': particle.weight * model_probability})
        return pd.DataFrame(rows)

    def get_weighted_sum_stats(self) -> tuple:
        weights, sum_stats = [], []
        for particle in self._materialise():
            mp = self._model_probabilities[particle.m]
            for sum_stat in particle.accepted_sum_stats:
                weights.append(particle.weight * mp)
                sum_stats.append(sum_stat)
        return weights, sum_stats

    def get_accepted_sum_stats(self):
        if self._cols is not None and self._cols.sum_stats is not None:
            from .distance.distance import SumStatMatrix
            return SumStatMatrix(self._cols.sum_stats, self._cols.sum_stat_keys)
        sum_stats = []
        for particle in self._list:
            sum_stats.extend(particle.accepted_sum_stats)
        return sum_stats

    def get_for_keys(self, keys):
        allowed_keys = ['weight', 'distance', 'parameter', 'sum_stat']
        for key in keys:
            if key not in allowed_keys:
                raise ValueError(f"Key {key} not in {allowed_keys}.")
        ret = {key: [] for key in keys}
        for particle in self._materialise():
            n_accepted = len(particle.accepted_distances)
            if 'weight' in keys:
                mp = self._model_probabilities[particle.m]
                ret['weight'].extend([particle.weight * mp] * n_accepted)
            if 'parameter' in keys:
                ret['parameter'].extend([particle.parameter] * n_accepted)
            if 'distance' in keys:
                ret['distance'].extend(particle.accepted_distances)
            if 'sum_stat' in keys:
                ret['sum_stat'].extend(particle.accepted_sum_stats)
        return ret

    def to_dict(self) -> dict:
        store = {}
        for particle in self._materialise():
            if particle is not None:
                store.setdefault(particle.m, []).append(particle)
            else:
                logger.warning("Empty particle.")
        return store
