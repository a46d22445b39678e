# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""Acceptors (pyabc/acceptor/acceptor.py:32-476, pdf_norm.py:1-110).

UniformAcceptor ``d <= eps(t)``: the batched sampler applies the same test on
the device (abc_accept_compact).  StochasticAcceptor: accept with probability
(pdf / c)^(1/T); the batched sampler runs it as abc_stochastic_accept (the
uniform comes from each candidate's counter-based stream) followed by the
same order-preserving compaction.
"""
import json
import logging

import numpy as np

from .distance.kernel import SCALE_LIN, StochasticKernel
from .storage.json import save_dict_to_json

logger = logging.getLogger("Acceptor")


class AcceptorResult(dict):
    def __init__(self, distance: float, accept: bool, weight: float = 1.0):
        super().__init__()
        self.distance = distance
        self.accept = accept
        self.weight = weight

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError:
            raise AttributeError(key)

    __setattr__ = dict.__setitem__
    __delattr__ = dict.__delitem__


class Acceptor:
    def __init__(self):
        pass

    def initialize(self, t, get_weighted_distances, distance_function, x_0):
        pass

    def update(self, t, get_weighted_distances, prev_temp, acceptance_rate):
        pass

    def __call__(self, distance_function, eps, x, x_0, t, par):
        raise NotImplementedError()

    def get_epsilon_config(self, t):
        return None

    def get_config(self):
        return {"name": self.__class__.__name__}

    def to_json(self):
        return json.dumps(self.get_config())


class SimpleFunctionAcceptor(Acceptor):
    def __init__(self, fun):
        super().__init__()
        self.fun = fun

    def __call__(self, distance_function, eps, x, x_0, t, par):
        return self.fun(distance_function, eps, x, x_0, t, par)

    @staticmethod
    def assert_acceptor(maybe_acceptor):
        if isinstance(maybe_acceptor, Acceptor):
            return maybe_acceptor
        return SimpleFunctionAcceptor(maybe_acceptor)


def accept_use_current_time(distance_function, eps, x, x_0, t, par):
    """acceptor.py:235-244."""
    d = distance_function(x, x_0, t, par)
    accept = d <= eps(t)
    return AcceptorResult(distance=d, accept=accept)


def accept_use_complete_history(distance_function, eps, x, x_0, t, par):
    """acceptor.py:247-276."""
    d = distance_function(x, x_0, t, par)
    accept = d <= eps(t)
    if accept:
        for t_prev in range(0, t):
            try:
                d_prev = distance_function(x, x_0, t_prev, par)
                accept = d_prev <= eps(t_prev)
                if not accept:
                    break
            except Exception:
                accept = True
    return AcceptorResult(distance=d, accept=accept)


class UniformAcceptor(Acceptor):
    def __init__(self, use_complete_history: bool = False):
        super().__init__()
        self.use_complete_history = use_complete_history

    def __call__(self, distance_function, eps, x, x_0, t, par):
        if self.use_complete_history:
            return accept_use_complete_history(distance_function, eps, x,
                                               x_0, t, par)
        return accept_use_current_time(distance_function, eps, x, x_0, t, par)


# ---- pdf normalisations (acceptor/pdf_norm.py) ------------------------------

def pdf_norm_from_kernel(kernel_val: float, **kwargs):
    """pdf_norm.py:6-13: the kernel's own pdf_max."""
    return kernel_val


def _max_distance(weighted_distances):
    dd = getattr(weighted_distances, "device_distance", None)
    if dd is not None:
        from . import gpu
        if dd.numel() == 0:
            return -np.inf
        lr = dd.contiguous()
        return gpu.temper_sums(None, lr, 0.0, True, gpu.TEMPER_MAX)[0]
    pdfs = np.array(weighted_distances['distance'])
    return max(pdfs) if pdfs.size else -np.inf


def pdf_norm_max_found(prev_pdf_norm, get_weighted_distances, **kwargs):
    """pdf_norm.py:16-36: max over the previous normalisation and the
    current population's densities (one device max reduction for device
    populations)."""
    df = get_weighted_distances()
    if prev_pdf_norm is None:
        prev_pdf_norm = -np.inf
    return max(prev_pdf_norm, _max_distance(df))


class ScaledPDFNorm:
    """pdf_norm.py:39-110.  (The reference stores ``self.factor = 10``
    whatever factor is passed; kept for parity.)"""

    def __init__(self, factor: float = 10, alpha: float = 0.5,
                 min_acceptance_rate: bool = 0.1):
        self.factor = 10
        self.alpha = alpha
        self.min_acceptance_rate = min_acceptance_rate
        self._hit = False

    def __call__(self, prev_pdf_norm, get_weighted_distances, prev_temp,
                 acceptance_rate, **kwargs):
        pdf_norm = pdf_norm_max_found(
            prev_pdf_norm=prev_pdf_norm,
            get_weighted_distances=get_weighted_distances)
        offset = np.log(self.factor)
        if acceptance_rate >= self.min_acceptance_rate and not self._hit:
            return pdf_norm
        self._hit = True
        next_temp = 1 if prev_temp is None else self.alpha * prev_temp
        return pdf_norm - offset * next_temp


class StochasticAcceptor(Acceptor):
    """acceptor.py:309-476: accept iff pdf(x_0|x)/c)^(1/T) >= u, weight
    acc / min(1, acc) (rejection-control importance weighting)."""

    def __init__(self, pdf_norm_method=None,
                 apply_importance_weighting: bool = True,
                 log_file: str = None):
        super().__init__()
        if pdf_norm_method is None:
            pdf_norm_method = pdf_norm_max_found
        self.pdf_norm_method = pdf_norm_method
        self.apply_importance_weighting = apply_importance_weighting
        self.log_file = log_file
        self.pdf_norms = {}
        self.x_0 = None
        self.kernel_scale = None
        self.kernel_pdf_max = None

    def initialize(self, t, get_weighted_distances,
                   distance_function: StochasticKernel, x_0):
        self.x_0 = x_0
        self.kernel_scale = distance_function.ret_scale
        self.kernel_pdf_max = distance_function.pdf_max
        self._update(t, get_weighted_distances)

    def update(self, t, get_weighted_distances, prev_temp, acceptance_rate):
        self._update(t, get_weighted_distances, prev_temp, acceptance_rate)

    def _update(self, t, get_weighted_distances, prev_temp=None,
                acceptance_rate=1.0):
        pdf_norm = self.pdf_norm_method(
            kernel_val=self.kernel_pdf_max,
            get_weighted_distances=get_weighted_distances,
            prev_pdf_norm=None if not self.pdf_norms
            else max(self.pdf_norms.values()),
            acceptance_rate=acceptance_rate,
            prev_temp=prev_temp)
        self.pdf_norms[t] = pdf_norm
        self.log(t)

    def log(self, t):
        logger.debug(f"pdf_norm={self.pdf_norms[t]:.4e} for t={t}.")
        if self.log_file:
            save_dict_to_json(self.pdf_norms, self.log_file)

    def get_epsilon_config(self, t: int) -> dict:
        return dict(pdf_norm=self.pdf_norms[t],
                    kernel_scale=self.kernel_scale)

    def device_config(self, t, temperature):
        """(pdf_norm, temperature, log scale, importance weighting) of
        generation t for abc_stochastic_accept."""
        return (float(self.pdf_norms[t]), float(temperature),
                self.kernel_scale != SCALE_LIN,
                bool(self.apply_importance_weighting))

    def __call__(self, distance_function, eps, x, x_0, t, par):
        kernel = distance_function
        temp = eps(t)
        density = kernel(x, x_0, t, par)
        pdf_norm = self.pdf_norms[t]
        if kernel.ret_scale == SCALE_LIN:
            acc_prob = (density / pdf_norm) ** (1 / temp)
        else:
            acc_prob = np.exp((density - pdf_norm) * (1 / temp))
        threshold = np.random.uniform(low=0, high=1)
        accept = bool(acc_prob >= threshold)
        if acc_prob == 0.0:
            weight = 0.0
        elif self.apply_importance_weighting:
            weight = acc_prob / min(1, acc_prob)
        else:
            weight = 1.0
        if pdf_norm < density:
            logger.debug(
                f"Encountered density={density:.4e} > c={pdf_norm:.4e}, "
                f"thus weight={weight:.4e}.")
        return AcceptorResult(density, accept, weight)
