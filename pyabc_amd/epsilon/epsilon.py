"""Epsilon schedules (pyabc/epsilon/epsilon.py:12-243).

QuantileEpsilon._update evaluates the weighted quantile on the GPU
(abc_weighted_quantile: weighted MSD select + np.interp semantics).
Weighted distances arrive either as the reference's DataFrame
(columns ``distance``, ``w``) or as a ``WeightedDistances`` object carrying
device tensors from the batched sampler (no host round trip).
"""
import logging

import numpy as np

from .. import gpu
from .base import Epsilon

logger = logging.getLogger("Epsilon")


class ConstantEpsilon(Epsilon):
    def __init__(self, constant_epsilon_value: float):
        super().__init__()
        self.constant_epsilon_value = constant_epsilon_value

    def get_config(self):
        config = super().get_config()
        config["constant_epsilon_value"] = self.constant_epsilon_value
        return config

    def __call__(self, t):
        return self.constant_epsilon_value


class ListEpsilon(Epsilon):
    def __init__(self, values):
        super().__init__()
        self.epsilon_values = list(values)

    def get_config(self):
        config = super().get_config()
        config["epsilon_values"] = self.epsilon_values
        return config

    def __call__(self, t):
        return self.epsilon_values[t]


def _device_distances(weighted_distances):
    """(distance tensor, weight tensor) on the device."""
    dd = getattr(weighted_distances, "device_distance", None)
    if dd is not None:
        return dd, weighted_distances.device_w
    d = np.asarray(weighted_distances.distance.values, dtype=np.float64)
    w = np.asarray(weighted_distances.w.values, dtype=np.float64)
    return gpu.as_dev(d), gpu.as_dev(w)


class QuantileEpsilon(Epsilon):
    def __init__(self, initial_epsilon='from_sample', alpha: float = 0.5,
                 quantile_multiplier: float = 1, weighted: bool = True):
        logger.debug(f"init quantile_epsilon initial_epsilon={initial_epsilon}"
                     f", quantile_multiplier={quantile_multiplier}")
        super().__init__()
        self._initial_epsilon = initial_epsilon
        self.alpha = alpha
        self.quantile_multiplier = quantile_multiplier
        self.weighted = weighted
        self._look_up = {}
        if self.alpha > 1 or self.alpha <= 0:
            raise ValueError("It must be 0 < alpha <= 1")

    def get_config(self):
        config = super().get_config()
        config.update({"initial_epsilon": self._initial_epsilon,
                       "alpha": self.alpha,
                       "quantile_multiplier": self.quantile_multiplier,
                       "weighted": self.weighted})
        return config

    def initialize(self, t, get_weighted_distances, get_all_records,
                   max_nr_populations, acceptor_config):
        if self._initial_epsilon != 'from_sample':
            return
        self._update(t, get_weighted_distances())
        logger.info(f"initial epsilon is {self(t)}")

    def __call__(self, t):
        if not self._look_up:
            self._set_initial_value(t)
        try:
            eps = self._look_up[t]
        except KeyError as e:
            raise KeyError(f"The epsilon value for time {t} does not exist: "
                           f"{repr(e)} ")
        if isinstance(eps, _PendingEps):  # device quantile still in flight
            eps = self._look_up[t] = eps.value()
        return eps

    def _set_initial_value(self, t):
        self._look_up = {t: self._initial_epsilon}

    def update(self, t, get_weighted_distances, get_all_records,
               acceptance_rate, acceptor_config):
        self._update(t, get_weighted_distances())

    def _update(self, t, weighted_distances):
        d, w = _device_distances(weighted_distances)
        if not self.weighted:
            w = gpu.torch.ones_like(d)
        # the kernel normalises w by its sum (epsilon.py:215-219)
        q = gpu.weighted_quantile(d, w, self.alpha)
        # read back lazily: __call__(t) is the first consumer
        self._look_up[t] = _PendingEps(gpu.HostFuture(q), self.quantile_multiplier,
                                       (d, w, self.alpha), q)

    def device_threshold(self, t):
        """(device quantile, multiplier) of generation t while its value is
        still on the way to the host -- the fused candidate round reads the
        threshold q * multiplier on the device, so it can be queued behind
        the quantile kernel -- else None."""
        eps = self._look_up.get(t) if self._look_up else None
        if isinstance(eps, _PendingEps) and eps.q_dev is not None:
            return eps.q_dev, eps._mult, eps._fut
        return None


class _PendingEps:
    """Quantile of the device kernel, resolved to a float on first use (an
    undecided select reruns on the sort-based kernel, gpu.resolve_quantile)."""

    def __init__(self, fut, multiplier, inputs=None, q_dev=None):
        self._fut = fut
        self._mult = multiplier
        self._inputs = inputs
        self.q_dev = q_dev

    def value(self):
        v = self._fut.get()[0]
        if self._inputs is not None:
            v = gpu.resolve_quantile(v, *self._inputs)
            self._inputs = None
        return float(v) * self._mult

    def __float__(self):
        return self.value()

    def __deepcopy__(self, memo):
        return self.value()

    def __reduce__(self):
        return (float, (self.value(),))


class MedianEpsilon(QuantileEpsilon):
    def __init__(self, initial_epsilon='from_sample', median_multiplier=1,
                 weighted=True):
        super().__init__(initial_epsilon=initial_epsilon, alpha=0.5,
                         quantile_multiplier=median_multiplier,
                         weighted=weighted)
