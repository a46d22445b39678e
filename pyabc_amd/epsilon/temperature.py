# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""Temperatures for the StochasticAcceptor (pyabc/epsilon/temperature.py).

  TemperatureBase / ListTemperature     :16-38
  Temperature (schemes, aggregation)    :41-244
  AcceptanceRateScheme / match_acceptance_rate :276-378
  ExpDecayFixedIterScheme   :381-423    ExpDecayFixedRatioScheme :426-493
  PolynomialDecayFixedIterScheme :496-546  DalyScheme :549-608
  FrielPettittScheme        :611-657    EssScheme :660-742

The two data-driven schemes evaluate their objectives as device reductions
(abc_temper_sums) over the records / population, while the scalar root find
(scipy bisect) and minimisation (scipy minimize) run exactly as in the
reference on the host around them.  Records come either as the reference's
list of dicts (per-particle samplers) or as ``DeviceRecords`` (batched
sampler: densities and log transition densities stay in HBM).
"""
import logging
import numbers
from typing import Callable, List, Union

import numpy as np
import scipy as sp
import scipy.optimize  # noqa: F401

from .. import gpu
from ..distance.kernel import SCALE_LIN
from ..storage.json import save_dict_to_json
from .base import Epsilon

logger = logging.getLogger("Epsilon")


class DeviceRecords:
    """All recorded candidates of a generation on the device: ``distance``
    (kernel densities) [R], ``log_pd_prev`` / ``log_pd`` (log transition
    densities under the previous and the new transition) [R], ``accepted``
    [R] the acceptance keys (accepted iff key <= 0, abc_stochastic_accept).  Behaves like the reference's list of record dicts when
    iterated (materialised lazily)."""

    def __init__(self, distance, log_pd_prev, log_pd, accepted):
        self.distance = distance
        self.log_pd_prev = log_pd_prev
        self.log_pd = log_pd
        self.accepted = accepted
        self._list = None

    def __len__(self):
        return int(self.distance.numel())

    def _materialise(self):
        if self._list is None:
            d = self.distance.cpu().numpy()
            tp = np.exp(self.log_pd_prev.cpu().numpy())
            tc = np.exp(self.log_pd.cpu().numpy())
            a = self.accepted.cpu().numpy()
            self._list = [dict(distance=d[i], transition_pd_prev=tp[i],
                               transition_pd=tc[i], accepted=bool(a[i] <= 0))
                          for i in range(d.size)]
        return self._list

    def __iter__(self):
        return iter(self._materialise())

    def __getitem__(self, i):
        return self._materialise()[i]


def _records_device(records):
    """(densities, weights, log t_pd_prev or None, log form) on the device.
    DeviceRecords carry log t_pd / log t_pd_prev (weight = exp of their
    difference); the reference's list of dicts carries linear densities
    (weight = t_pd / t_pd_prev as is, any sign)."""
    if isinstance(records, DeviceRecords):
        return (records.distance.contiguous(), records.log_pd.contiguous(),
                records.log_pd_prev.contiguous(), True)
    d = np.array([r['distance'] for r in records], dtype=float)
    tp = np.array([r['transition_pd_prev'] for r in records], dtype=float)
    tc = np.array([r['transition_pd'] for r in records], dtype=float)
    return gpu.as_dev(d), gpu.as_dev(tc / tp), None, False


class TemperatureBase(Epsilon):
    """temperature.py:16-23."""


class ListTemperature(TemperatureBase):
    """temperature.py:26-38."""

    def __init__(self, values: List[float]):
        super().__init__()
        self.values = values

    def __call__(self, t: int) -> float:
        return self.values[t]


class Temperature(TemperatureBase):
    """temperature.py:41-244."""

    def __init__(self, schemes: Union[Callable, List[Callable]] = None,
                 aggregate_fun: Callable[[List[float]], float] = None,
                 initial_temperature: float = None,
                 enforce_exact_final_temperature: bool = True,
                 log_file: str = None):
        super().__init__()
        self.schemes = schemes
        if aggregate_fun is None:
            aggregate_fun = min
        self.aggregate_fun = aggregate_fun
        if initial_temperature is None:
            initial_temperature = AcceptanceRateScheme()
        self.initial_temperature = initial_temperature
        self.enforce_exact_final_temperature = enforce_exact_final_temperature
        self.log_file = log_file
        self.max_nr_populations = None
        self.temperatures = {}
        self.temperature_proposals = {}

    def initialize(self, t, get_weighted_distances, get_all_records,
                   max_nr_populations, acceptor_config):
        self.max_nr_populations = max_nr_populations
        if self.schemes is None:
            acc_rate_scheme = AcceptanceRateScheme()
            decay_scheme = (
                ExpDecayFixedIterScheme() if np.isfinite(max_nr_populations)
                else ExpDecayFixedRatioScheme())
            self.schemes = [acc_rate_scheme, decay_scheme]
        self._update(t, get_weighted_distances, get_all_records, 1.0,
                     acceptor_config)

    def configure_sampler(self, sampler):
        if callable(self.initial_temperature):
            self.initial_temperature.configure_sampler(sampler)
        for scheme in self.schemes:
            scheme.configure_sampler(sampler)

    def update(self, t, get_weighted_distances, get_all_records,
               acceptance_rate, acceptor_config):
        self._update(t, get_weighted_distances, get_all_records,
                     acceptance_rate, acceptor_config)

    def _update(self, t, get_weighted_distances, get_all_records,
                acceptance_rate, acceptor_config):
        kwargs = dict(
            t=t,
            get_weighted_distances=get_weighted_distances,
            get_all_records=get_all_records,
            max_nr_populations=self.max_nr_populations,
            pdf_norm=acceptor_config['pdf_norm'],
            kernel_scale=acceptor_config['kernel_scale'],
            prev_temperature=self.temperatures.get(t - 1, None),
            acceptance_rate=acceptance_rate,
        )
        if t >= self.max_nr_populations - 1 \
                and self.enforce_exact_final_temperature:
            temps = [1.0]
        elif not self.temperatures:
            if callable(self.initial_temperature):
                temps = [self.initial_temperature(**kwargs)]
            elif isinstance(self.initial_temperature, numbers.Number):
                temps = [self.initial_temperature]
            else:
                raise ValueError(
                    "Initial temperature must be a float or a callable")
        else:
            temps = [scheme(**kwargs) for scheme in self.schemes]
        fallback = self.temperatures[t - 1] \
            if t - 1 in self.temperatures else np.inf
        temperature = self.aggregate_fun(temps)
        temperature = max(min(temperature, fallback), 1.0)
        if not np.isfinite(temperature):
            raise ValueError("Temperature must be finite.")
        self.temperatures[t] = temperature
        logger.debug(f"Proposed temperatures for {t}: {temps}.")
        self.temperature_proposals[t] = temps
        if self.log_file:
            save_dict_to_json(self.temperature_proposals, self.log_file)

    def __call__(self, t: int) -> float:
        return self.temperatures[t]


class TemperatureScheme:
    """temperature.py:247-273."""

    def __init__(self):
        pass

    def configure_sampler(self, sampler):
        pass

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        pass


class AcceptanceRateScheme(TemperatureScheme):
    """temperature.py:276-340: the temperature whose predicted acceptance
    rate over the importance-reweighted records is ``target_rate``."""

    def __init__(self, target_rate: float = 0.3, min_rate: float = None):
        self.target_rate = target_rate
        self.min_rate = min_rate

    def configure_sampler(self, sampler):
        sampler.sample_factory.record_rejected = True

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if self.min_rate is not None and acceptance_rate < self.min_rate:
            return np.inf
        records = get_all_records()
        dens, lr, lr_prev, log_form = _records_device(records)
        return match_acceptance_rate(dens, lr, pdf_norm, kernel_scale,
                                     self.target_rate, lr_prev, log_form)


def match_acceptance_rate(dens, lr, pdf_norm, kernel_scale, target_rate,
                          lr_prev=None, log_form=True):
    """temperature.py:343-378 with the objective
    sum_i w_i min(acc_i(beta), 1) - target evaluated on the device, w the
    normalised importance weights t_pd / t_pd_prev (exp(lr - lr_prev) in log
    form, lr itself otherwise); same bisection bracket, tolerances and corner
    cases as the reference."""
    scale_log = kernel_scale != SCALE_LIN
    if log_form:
        shift = gpu.temper_sums(None, lr, 0.0, scale_log, gpu.TEMPER_MAX,
                                lr_sub=lr_prev)[0]
        mode = gpu.TEMPER_ACCEPTANCE
    else:
        shift, mode = 0.0, gpu.TEMPER_ACCEPTANCE_LIN

    def obj(b):
        a, tot = gpu.temper_sums(dens, lr, pdf_norm, scale_log, mode,
                                 np.exp(b), shift, lr_sub=lr_prev)
        return a / tot - target_rate

    return _bisect_temperature(obj)


def _bisect_temperature(obj):
    min_b = -100
    if obj(0) > 0:
        b_opt = 0
    elif obj(min_b) < 0:
        logger.info("AcceptanceRateScheme: Numerics limit temperature.")
        b_opt = min_b
    else:
        b_opt = sp.optimize.bisect(obj, min_b, 0, maxiter=100000)
    beta_opt = np.exp(b_opt)
    return 1. / beta_opt


class ExpDecayFixedIterScheme(TemperatureScheme):
    """temperature.py:381-423."""

    def __init__(self):
        pass

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if max_nr_populations == np.inf:
            raise ValueError(
                "The ExpDecayFixedIterScheme requires a finite "
                "`max_nr_populations`.")
        if prev_temperature is None:
            return np.inf
        t_to_go = max_nr_populations - t
        return prev_temperature ** ((t_to_go - 1) / t_to_go)


class ExpDecayFixedRatioScheme(TemperatureScheme):
    """temperature.py:426-493."""

    def __init__(self, alpha: float = 0.5, min_rate: float = 1e-4,
                 max_rate: float = 0.5):
        self.alpha = alpha
        self.min_rate = min_rate
        self.max_rate = max_rate
        self.alphas = {}

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if prev_temperature is None:
            return np.inf
        alpha = self.alphas.get(t - 1, self.alpha)
        if acceptance_rate > self.max_rate and t > 1:
            logger.debug("ExpDecayFixedRatioScheme: "
                         "Reacting to high acceptance rate.")
            alpha = max(alpha / 2, alpha - (1 - alpha) * 2)
        if acceptance_rate < self.min_rate:
            logger.debug("ExpDecayFixedRatioScheme: "
                         "Reacting to low acceptance rate.")
            alpha = alpha + (1 - alpha) / 2
        self.alphas[t] = alpha
        return self.alphas[t] * prev_temperature


class PolynomialDecayFixedIterScheme(TemperatureScheme):
    """temperature.py:496-546."""

    def __init__(self, exponent: float = 3):
        self.exponent = exponent

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if prev_temperature is None:
            return np.inf
        if max_nr_populations == np.inf:
            raise ValueError("Can only perform PolynomialDecayScheme step "
                             "with a finite max_nr_populations.")
        t_to_go = max_nr_populations - t
        temps = np.linspace(1, prev_temperature ** (1 / self.exponent),
                            t_to_go + 1) ** self.exponent
        logger.debug(f"Temperatures proposed by polynomial decay method: "
                     f"{temps}.")
        return temps[-2]


class DalyScheme(TemperatureScheme):
    """temperature.py:549-608."""

    def __init__(self, alpha: float = 0.5, min_rate: float = 1e-4):
        self.alpha = alpha
        self.min_rate = min_rate
        self.k = {}

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if prev_temperature is None:
            return np.inf
        eps_base = np.sqrt(prev_temperature)
        if not self.k:
            self.k[t - 1] = eps_base
        k_base = self.k[t - 1]
        if acceptance_rate < self.min_rate:
            logger.debug("DalyScheme: Reacting to low acceptance rate.")
            k_base = self.alpha * k_base
        self.k[t] = min(k_base, self.alpha * eps_base)
        eps = eps_base - self.k[t]
        return eps ** 2


class FrielPettittScheme(TemperatureScheme):
    """temperature.py:611-657."""

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if prev_temperature is None:
            return np.inf
        if max_nr_populations == np.inf:
            raise ValueError("Can only perform FrielPettittScheme step with a "
                             "finite max_nr_populations.")
        beta_base = 1. / prev_temperature
        t_to_go = max_nr_populations - t
        beta = beta_base + ((1. - beta_base) * 1 / t_to_go) ** 2
        return 1. / beta


class EssScheme(TemperatureScheme):
    """temperature.py:660-742: the temperature at which the reweighted
    population keeps ``target_relative_ess`` of its size; the ESS objective
    is a device reduction, scipy's bounded minimiser drives it."""

    def __init__(self, target_relative_ess: float = 0.8):
        self.target_relative_ess = target_relative_ess

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        df = get_weighted_distances()
        dd = getattr(df, "device_distance", None)
        if dd is not None:
            dens, w = dd.contiguous(), df.device_w.contiguous()
        else:
            dens = gpu.as_dev(np.array(df['distance'], dtype=float))
            w = gpu.as_dev(np.array(df['w'], dtype=float))
        n = int(w.numel())
        target_ess = n * self.target_relative_ess
        beta_base = 0.0 if prev_temperature is None else 1. / prev_temperature
        scale_log = kernel_scale != SCALE_LIN

        def obj(beta):
            # ESS = (sum w v^b)^2 / sum (w v^b)^2 is invariant to the
            # reference's normalisation of w
            b = float(np.asarray(beta).ravel()[0])
            s1, s2 = gpu.temper_sums(dens, w, pdf_norm, scale_log,
                                     gpu.TEMPER_ESS, b)
            return (s1 * s1 / s2 - target_ess) ** 2

        bounds = sp.optimize.Bounds(lb=np.array([beta_base]),
                                    ub=np.array([1.]))
        ret = sp.optimize.minimize(obj, x0=np.array([0.5 * (1 + beta_base)]),
                                   bounds=bounds)
        return 1. / ret.x
