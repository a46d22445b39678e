"""ABCSMC orchestration (pyabc/smc.py:45-1079), same public API.

The generation loop, calibration, stopping rules and between-generation
updates follow the reference line for line in behaviour (citations inline).
What changes is the per-candidate closure: ``_create_simulate_function``
returns a ``GenerationSpec`` that is still callable per candidate (so the
reference's sampler contract holds for ``SingleCoreSampler``) but also
exposes the device pieces -- prior spec, transition, vectorised model,
distance, epsilon -- that ``BatchedGPUSampler`` runs as batched HIP kernels.
Populations produced by the batched sampler stay on the GPU; the next fit,
the adaptive distance update and the epsilon quantile read them in place.
"""
import copy
import datetime
import logging
from typing import Callable, List, Union

import numpy as np
import pandas as pd

from . import gpu
from .acceptor import (Acceptor, SimpleFunctionAcceptor, StochasticAcceptor,
                       UniformAcceptor)
from .distance import Distance, PNormDistance, StochasticKernel, to_distance
from .epsilon import DeviceRecords, Epsilon, MedianEpsilon, TemperatureBase
from .model import Model, SimpleModel, VectorizedModel
from .parameters import Parameter
from .population import Particle, Population
from .populationstrategy import ConstantPopulationSize, PopulationStrategy
from .random_variables import RV, Distribution, host_prior_logpdf
from .sampler import BatchedGPUSampler, Sampler, SingleCoreSampler
from .storage import History
from .transition import MultivariateNormalTransition, Transition
from .weighted_statistics import effective_sample_size

logger = logging.getLogger("ABC")


def identity(x):
    return x


class GenerationSpec:
    """Everything one generation needs, per candidate or batched.

    ``__call__`` is the reference closure ``simulate_one`` (smc.py:588-606);
    the attributes describe the same computation to BatchedGPUSampler.
    """

    def __init__(self, abc, t, all_accepted=False):
        self.t = t
        self.all_accepted = all_accepted
        self._abc = abc
        self.param_names = abc.parameter_priors[0].get_parameter_names()
        self.model = abc.models[0]
        self.nr_samples_per_parameter = \
            abc.population_size.nr_samples_per_parameter
        self.weight_scale = 1.0 / self.nr_samples_per_parameter
        self.transition = None if (t <= 0 or all_accepted) else abc.transitions[0]
        self.distance = None if all_accepted else abc.distance_function
        # the threshold on the host is read on first use (the fused rounds
        # take it on the device, eps_device, and need the host value only
        # after their first round)
        self._eps = None
        dev_thr = getattr(abc.eps, "device_threshold", None)
        self.eps_device = None if (all_accepted or dev_thr is None) else dev_thr(t)
        self.sum_stat_keys = list(abc.x_0.keys())
        # StochasticAcceptor: (pdf_norm, temperature, log scale, importance
        # weighting) of this generation for abc_stochastic_accept
        self.stochastic = None
        if isinstance(abc.acceptor, StochasticAcceptor) and not all_accepted:
            self.stochastic = abc.acceptor.device_config(t, self.eps)
        self._closure = None
        self._init_device(abc)

    @property
    def eps(self):
        if self.all_accepted:
            return None
        if self._eps is None:
            self._eps = self._abc.eps(self.t)
        return self._eps

    def _init_device(self, abc):
        why = []
        if len(abc.models) != 1:
            why.append("more than one model")
        if not isinstance(self.model, VectorizedModel):
            why.append("model is not a VectorizedModel")
        elif list(self.model.sum_stat_keys) != self.sum_stat_keys:
            why.append("model sum_stat_keys differ from x_0 key order")
        if abc.summary_statistics is not identity:
            why.append("custom summary_statistics function")
        if self.nr_samples_per_parameter != 1:
            why.append("nr_samples_per_parameter != 1")
        if isinstance(abc.acceptor, StochasticAcceptor):
            if not getattr(abc.distance_function, "batched_capable", False):
                why.append("StochasticAcceptor without a batched noise-model "
                           "kernel")
        elif not isinstance(abc.acceptor, UniformAcceptor) or \
                abc.acceptor.use_complete_history:
            why.append("acceptor is not UniformAcceptor(current time) or "
                       "StochasticAcceptor")
        if self.distance is not None and (
                not hasattr(self.distance, "device_call")
                or not getattr(self.distance, "batched_capable", True)):
            why.append("distance has no device kernel")
        if self.transition is not None and not hasattr(self.transition,
                                                       "propose_device"):
            why.append("transition has no device kernel")
        prior = abc.parameter_priors[0]
        # the prior's device form and host components, computed once per
        # run() (ABCSMC.run resets the cache; the prior does not change
        # during a run)
        cached = abc.__dict__.get("_prior_spec_cache")
        if cached is not None and cached[0] is prior:
            spec, host = cached[1], cached[2]
        else:
            spec = prior.device_spec() if hasattr(prior, "device_spec") else None
            host = prior.host_components() if spec is not None else []
            abc.__dict__["_prior_spec_cache"] = (prior, spec, host)
        if spec is None:
            why.append("prior component without a batched form (not a scipy "
                       "RV, or a discrete / non-frozen scipy distribution "
                       "outside the device families)")
        # components without a device sampler: host-scipy density / draws
        self.host_prior = host
        self.why_not = "; ".join(why)
        self.batched_capable = not why
        if self.batched_capable:
            # prior and x_0 device constants: uploaded once per run, reused
            # by every generation (they change only if the prior or x_0 do)
            x0 = np.array([abc.x_0[k] for k in self.sum_stat_keys], dtype=np.float64)
            key = (np.asarray(spec[0]).tobytes(), np.asarray(spec[1]).tobytes(),
                   x0.tobytes())
            cache = abc.__dict__.setdefault("_device_consts", {})
            if key not in cache:
                dev = gpu.require_device()
                cache.clear()
                cache[key] = (gpu.as_dev(spec[0], dtype=gpu.torch.int32, device=dev),
                              gpu.as_dev(spec[1], device=dev),
                              gpu.as_dev(x0, device=dev))
            self.prior_kind, self.prior_params, self.x0vec = cache[key]
            self.prior_kind_host = tuple(int(k) for k in np.asarray(spec[0]).ravel())

    def __call__(self):
        if self._closure is None:
            if self.all_accepted:
                self._closure = self._abc._create_simulate_from_prior_function(self.t)
            else:
                self._closure = self._abc._create_simulate_function_closure(self.t)
        return self._closure()


class ModelPerturbationKernel:
    """Model jump of multi-model runs (the role of
    random_variables.py:455-538 at smc.py:641-649): from model m stay with
    probability p_stay, else move to one of the other models uniformly.
    Not on the batched path (single-model generations only)."""

    def __init__(self, nr_of_models: int, probability_to_stay=None):
        self.nr_of_models = int(nr_of_models)
        if self.nr_of_models == 1:
            p = 1.0
        elif probability_to_stay is None:
            p = 1.0 / self.nr_of_models
        else:
            p = float(np.clip(probability_to_stay, 0.0, 1.0))
        self.probability_to_stay = p

    def _row(self, m):
        n = self.nr_of_models
        if not 0 <= m < n:
            raise Exception("m has to be between 0 and nr_of_models - 1")
        if n == 1:
            return np.ones(1)
        row = np.full(n, (1.0 - self.probability_to_stay) / (n - 1))
        row[m] = self.probability_to_stay
        return row

    def rvs(self, m: int) -> int:
        row = self._row(int(m))
        return 0 if row.size == 1 else int(np.random.choice(row.size, p=row))

    def pmf(self, n: int, m: int) -> float:
        # the reference accepts n == nr_of_models (mass 0) and raises beyond
        # (random_variables.py:527-531)
        if not 0 <= n <= self.nr_of_models:
            raise Exception("n and m have to be between 0 and nr_of_models - 1")
        row = self._row(int(m))
        return float(row[n]) if n < row.size else 0.0


class ABCSMC:
    """Approximate Bayesian Computation - Sequential Monte Carlo
    (pyabc/smc.py:45-236 for the parameters).  Default sampler here is
    BatchedGPUSampler when the model is vectorised, else SingleCoreSampler."""

    def __init__(self, models, parameter_priors, distance_function=None,
                 population_size=100, summary_statistics=identity,
                 model_prior: RV = None, model_perturbation_kernel=None,
                 transitions=None, eps: Epsilon = None, sampler: Sampler = None,
                 acceptor: Acceptor = None,
                 stop_if_only_single_model_alive: bool = False,
                 max_nr_recorded_particles: int = np.inf,
                 show_progress: bool = False):
        if not isinstance(models, list):
            models = [models]
        self.models = list(map(SimpleModel.assert_model, models))
        if not isinstance(parameter_priors, list):
            parameter_priors = [parameter_priors]
        self.parameter_priors = parameter_priors
        if len(self.models) != len(self.parameter_priors):
            raise AssertionError(
                "Number models and number parameter priors have to agree.")
        if distance_function is None:
            distance_function = PNormDistance()
        self.distance_function = to_distance(distance_function)
        self.summary_statistics = summary_statistics
        if model_prior is None:
            model_prior = RV("randint", 0, len(self.models))
        self.model_prior = model_prior
        if model_perturbation_kernel is None:
            model_perturbation_kernel = ModelPerturbationKernel(
                len(self.models), probability_to_stay=.7)
        self.model_perturbation_kernel = model_perturbation_kernel
        if transitions is None:
            transitions = [MultivariateNormalTransition() for _ in self.models]
        if not isinstance(transitions, list):
            transitions = [transitions]
        self.transitions = transitions
        if eps is None:
            eps = MedianEpsilon(median_multiplier=1)
        self.eps = eps
        if isinstance(population_size, int):
            population_size = ConstantPopulationSize(population_size)
        self.population_size = population_size
        if sampler is None:
            sampler = (BatchedGPUSampler()
                       if all(isinstance(m, VectorizedModel) for m in self.models)
                       else SingleCoreSampler())
        self.sampler = sampler
        if acceptor is None:
            acceptor = UniformAcceptor()
        self.acceptor = SimpleFunctionAcceptor.assert_acceptor(acceptor)
        self.stop_if_only_single_model_alive = stop_if_only_single_model_alive
        self.max_nr_recorded_particles = max_nr_recorded_particles
        self.show_progress = show_progress
        self.x_0 = None
        self.history = None
        self._initial_population = None
        self.minimum_epsilon = None
        self.max_nr_populations = None
        self.min_acceptance_rate = None
        self.generation_log = []
        # optional callable(t) run after each completed generation (timing
        # hooks; not part of the reference API)
        self.generation_callback = None
        self._sanity_check()

    def _sanity_check(self):
        """smc.py:238-248: the stochastic components go together."""
        stochastics = [isinstance(self.acceptor, StochasticAcceptor),
                       isinstance(self.eps, TemperatureBase),
                       isinstance(self.distance_function, StochasticKernel)]
        if not all(stochastics) and any(stochastics):
            raise ValueError(
                "Please only use acceptor.StochasticAcceptor, "
                "epsilon.TemperatureBase and distance.StochasticKernel "
                "together.")

    def __getstate__(self):
        state = self.__dict__.copy()
        del state['sampler']
        state.pop("_device_consts", None)   # device tensors stay per process
        return state

    # -- history ------------------------------------------------------------
    def new(self, db: str, observed_sum_stat: dict = None, *, gt_model=None,
            gt_par=None, meta_info=None) -> History:
        """smc.py:255-353."""
        if observed_sum_stat is None:
            observed_sum_stat = {}
        self.x_0 = observed_sum_stat
        self.history = History(db)
        if gt_par is None:
            gt_par = {}
        model_names = [model.name for model in self.models]
        self.history.store_initial_data(
            gt_model, meta_info, observed_sum_stat, gt_par, model_names,
            self.distance_function.to_json(), self.eps.to_json(),
            self.population_size.to_json())
        return self.history

    def load(self, db: str, abc_id: int = 1, observed_sum_stat: dict = None):
        """smc.py:355-389: resume from an in-process History object or a
        ``sqlite:///path`` file (written by this engine or by pyABC)."""
        if isinstance(db, History):
            self.history = db
            self.history.id = abc_id
        else:
            self.history = History(db)
            self.history.load_run(abc_id)
        if observed_sum_stat is None:
            observed_sum_stat = self.history.observed_sum_stat()
        self.x_0 = observed_sum_stat
        return self.history

    # -- calibration (smc.py:391-542) -------------------------------------
    def _initialize_dist_eps_acc(self, t: int):
        def get_initial_sum_stats():
            return self._get_initial_population(t).get_accepted_sum_stats()

        def _get_initial_population_with_distances():
            population = self._get_initial_population(t)
            self._update_population_distances(population, t)
            return population

        def get_initial_weighted_distances():
            return _get_initial_population_with_distances().get_weighted_distances()

        self.distance_function.initialize(t, get_initial_sum_stats, self.x_0)
        self.acceptor.initialize(t, get_initial_weighted_distances,
                                 self.distance_function, self.x_0)

        def get_initial_records():
            population = _get_initial_population_with_distances()
            if population.columns is not None:
                # calibration sample on the device: transition densities 1
                d = population.columns.distances
                one = gpu.torch.zeros_like(d)
                return DeviceRecords(d, one, one, gpu.torch.full_like(d, -1.0))
            records = []
            for particle in population.get_list():
                for d in particle.accepted_distances:
                    records.append({'distance': d, 'transition_pd_prev': 1.0,
                                    'transition_pd': 1.0, 'accepted': True})
            return records

        self.eps.initialize(t, get_initial_weighted_distances,
                            get_initial_records, self.max_nr_populations,
                            self.acceptor.get_epsilon_config(t))

    def _update_population_distances(self, population, t):
        """population.update_distances (population.py:147-162), batched on
        the device for columnar populations."""
        if population.columns is not None and hasattr(self.distance_function,
                                                      "device_call"):
            x0vec = gpu.as_dev(np.array([self.x_0[k] for k in population.columns.sum_stat_keys],
                                        dtype=np.float64))
            population.update_distances_device(self.distance_function, x0vec, t)
        else:
            def distance_to_ground_truth(x, par):
                return self.distance_function(x, self.x_0, t, par)
            population.update_distances(distance_to_ground_truth)

    def _get_initial_population(self, t: int):
        if self._initial_population is None:
            if self.history.n_populations > 0:
                population = self.history.get_population()
            else:
                population = self._sample_from_prior(t)
                self.history.update_nr_samples(History.PRE_TIME,
                                               self.sampler.nr_evaluations_)
            self._initial_population = population
        return self._initial_population

    def _create_simulate_from_prior_function(self, t: int):
        model_prior = self.model_prior
        parameter_priors = self.parameter_priors
        models = self.models
        summary_statistics = self.summary_statistics

        def simulate_one():
            m = int(model_prior.rvs())
            theta = parameter_priors[m].rvs()
            model_result = models[m].summary_statistics(t, theta,
                                                        summary_statistics)
            return Particle(m=m, parameter=theta, weight=1.0,
                            accepted_sum_stats=[model_result.sum_stats],
                            accepted_distances=[np.inf],
                            rejected_sum_stats=[], rejected_distances=[],
                            accepted=True)
        return simulate_one

    def _sample_from_prior(self, t: int):
        logger.info(f"Calibration sample before t={t}.")
        spec = GenerationSpec(self, -1, all_accepted=True)
        sample = self.sampler.sample_until_n_accepted(
            self.population_size(-1), spec, max_eval=np.inf,
            all_accepted=True, show_progress=self.show_progress)
        return sample.get_accepted_population()

    # -- per-candidate closure (smc.py:544-811) ---------------------------
    def _create_simulate_function(self, t: int):
        return GenerationSpec(self, t)

    def _create_simulate_function_closure(self, t: int):
        model_probabilities = self.history.get_model_probabilities(t - 1)
        m = np.array(model_probabilities.index)
        p = np.array(model_probabilities.p)
        model_prior = self.model_prior
        parameter_priors = self.parameter_priors
        model_perturbation_kernel = self.model_perturbation_kernel
        transitions = self.transitions
        nr_samples_per_parameter = self.population_size.nr_samples_per_parameter
        models = self.models
        summary_statistics = self.summary_statistics
        distance_function = self.distance_function
        eps = self.eps
        acceptor = self.acceptor
        x_0 = self.x_0
        weight_function = self._create_weight_function(t)

        def simulate_one():
            parameter = ABCSMC._generate_valid_proposal(
                t, m, p, model_prior, parameter_priors,
                model_perturbation_kernel, transitions)
            return ABCSMC._evaluate_proposal(
                *parameter, t, nr_samples_per_parameter, models,
                summary_statistics, distance_function, eps, acceptor, x_0,
                weight_function)
        return simulate_one

    @staticmethod
    def _generate_valid_proposal(t, m, p, model_prior, parameter_priors,
                                 model_perturbation_kernel, transitions):
        """smc.py:610-662.  t = 0: (model, theta) from the priors.  Later:
        a source model from the previous generation's probabilities p over
        the alive models m, moved by the model perturbation kernel (a move to
        a dead model is simply drawn again), theta from the target model's
        transition; repeated until the pair has positive prior density."""
        if t == 0:
            model = int(model_prior.rvs())
            return model, parameter_priors[model].rvs()
        alive = {int(v) for v in m}
        zero_density = 0
        while True:
            model = int(m[0])
            if len(m) > 1:
                source = int(m[np.random.choice(len(p), p=p)])
                model = int(model_perturbation_kernel.rvs(source))
                if model not in alive:
                    continue
            theta = Parameter(**transitions[model].rvs().to_dict())
            if model_prior.pmf(model) * parameter_priors[model].pdf(theta) > 0:
                return model, theta
            zero_density += 1
            if zero_density == 1000:
                logger.warning("1000 proposals in a row fell outside the prior "
                               "support; check the transition's scaling.")

    @staticmethod
    def _evaluate_proposal(m_ss, theta_ss, t, nr_samples_per_parameter, models,
                           summary_statistics, distance_function, eps,
                           acceptor, x_0, weight_function):
        accepted_sum_stats, accepted_distances = [], []
        rejected_sum_stats, rejected_distances = [], []
        accepted_weights = []
        for _ in range(nr_samples_per_parameter):
            model_result = models[m_ss].accept(t, theta_ss, summary_statistics,
                                               distance_function, eps,
                                               acceptor, x_0)
            if model_result.accepted:
                accepted_sum_stats.append(model_result.sum_stats)
                accepted_distances.append(model_result.distance)
                accepted_weights.append(model_result.weight)
            else:
                rejected_sum_stats.append(model_result.sum_stats)
                rejected_distances.append(model_result.distance)
        accepted = len(accepted_sum_stats) > 0
        weight = (weight_function(accepted_distances, m_ss, theta_ss,
                                  accepted_weights) if accepted else 0)
        return Particle(m=m_ss, parameter=theta_ss, weight=weight,
                        accepted_sum_stats=accepted_sum_stats,
                        accepted_distances=accepted_distances,
                        rejected_sum_stats=rejected_sum_stats,
                        rejected_distances=rejected_distances,
                        accepted=accepted)

    def _create_transition_pdf(self, t: int, transitions=None):
        if t == 0:
            return self._create_prior_pdf()
        model_probabilities = self.history.get_model_probabilities(t - 1)
        model_perturbation_kernel = self.model_perturbation_kernel
        if transitions is None:
            transitions = self.transitions

        def transition_pdf(m_ss, theta_ss):
            model_factor = sum(
                row.p * model_perturbation_kernel.pmf(m_ss, m)
                for m, row in model_probabilities.iterrows())
            particle_factor = transitions[m_ss].pdf(pd.Series(dict(theta_ss)))
            transition_pd = model_factor * particle_factor
            if transition_pd == 0:
                logger.debug("Transition density is zero!")
            return transition_pd
        return transition_pdf

    def _create_prior_pdf(self):
        model_prior = self.model_prior
        parameter_priors = self.parameter_priors

        def prior_pdf(m_ss, theta_ss):
            return model_prior.pmf(m_ss) * parameter_priors[m_ss].pdf(theta_ss)
        return prior_pdf

    def _create_weight_function(self, t: int):
        nr_samples_per_parameter = self.population_size.nr_samples_per_parameter
        if t == 0:
            def prior_weight_function(distance_list, m_ss, theta_ss,
                                      acceptance_weights):
                weight = len(distance_list) / nr_samples_per_parameter
                weight *= np.prod(acceptance_weights)
                return weight
            return prior_weight_function
        transition_pdf = self._create_transition_pdf(t)
        prior_pdf = self._create_prior_pdf()

        def weight_function(distance_list, m_ss, theta_ss, acceptance_weights):
            prior_pd = prior_pdf(m_ss, theta_ss)
            transition_pd = transition_pdf(m_ss, theta_ss)
            acceptance_weight = np.prod(acceptance_weights)
            fraction = len(distance_list) / nr_samples_per_parameter
            return prior_pd * acceptance_weight * fraction / transition_pd
        return weight_function

    # -- run (smc.py:813-958) ----------------------------------------------
    def run(self, minimum_epsilon: float = None,
            max_nr_populations: int = np.inf,
            min_acceptance_rate: float = 0.) -> History:
        if minimum_epsilon is None:
            # smc.py:860-864: a temperature schedule ends at T = 1
            minimum_epsilon = 1.0 if isinstance(self.eps, TemperatureBase) \
                else 0.0
        self.minimum_epsilon = minimum_epsilon
        self.max_nr_populations = max_nr_populations
        self.min_acceptance_rate = min_acceptance_rate
        t0 = self.history.max_t + 1
        self.history.start_time = datetime.datetime.now()
        self.__dict__.pop("_prior_spec_cache", None)
        self._fit_transitions(t0)
        self._adapt_population_size(t0)
        self._initialize_dist_eps_acc(t0)
        self.distance_function.configure_sampler(self.sampler)
        self.eps.configure_sampler(self.sampler)
        if hasattr(self.sampler, "max_nr_recorded"):
            # the batched sampler keeps only the recorded rows that are used
            self.sampler.max_nr_recorded = self.max_nr_recorded_particles
        t_max = t0 + max_nr_populations - 1
        t = t0
        # host reads deferred into the next generation (the ESS line of
        # generation t): a sampler with an on_density_queued hook runs them
        # once that generation's transition density is queued, so the host
        # never waits for a density while the GPU runs dry behind it
        pending = []

        def flush():
            while pending:
                pending.pop(0)()
        while t <= t_max:
            # the threshold is read after the sample: the fused rounds take
            # it on the device (GenerationSpec.eps_device), so the first round
            # is queued behind the quantile kernel instead of waiting for it
            t_start = datetime.datetime.now()
            simulate_one = self._create_simulate_function(t)
            pop_size = self.population_size(t)
            max_eval = (np.inf if min_acceptance_rate == 0.
                        else pop_size / min_acceptance_rate)
            if pending and hasattr(self.sampler, "on_density_queued"):
                self.sampler.on_density_queued = flush
            try:
                sample = self.sampler.sample_until_n_accepted(
                    pop_size, simulate_one, max_eval,
                    show_progress=self.show_progress)
            finally:
                if hasattr(self.sampler, "on_density_queued"):
                    self.sampler.on_density_queued = None
                flush()
            current_eps = self.eps(t)
            logger.info(f"t: {t}, eps: {current_eps}.")
            if not sample.ok:
                logger.info("Stopping: sample not ok.")
                break
            population = sample.get_accepted_population()
            n_sim = self.sampler.nr_evaluations_
            model_names = [model.name for model in self.models]
            self.history.append_population(t, current_eps, population, n_sim,
                                           model_names)
            pop_size = len(population)
            acceptance_rate = pop_size / n_sim
            # the ESS is read after the next fit is queued (no host sync
            # while the transition-density kernel is still running)
            ess_read = self._ess_async(population)
            self._prepare_next_iteration(t + 1, sample, population,
                                         acceptance_rate)
            entry = dict(t=t, eps=float(current_eps), n_sim=int(n_sim), ess=None,
                         seconds=(datetime.datetime.now() - t_start).total_seconds())
            self.generation_log.append(entry)

            def log_ess(entry=entry, ess_read=ess_read, pop_size=pop_size,
                        n_sim=n_sim, rate=acceptance_rate):
                entry["ess"] = ess = float(ess_read())
                logger.info(f"Acceptance rate: {pop_size} / {n_sim} = "
                            f"{rate:.4e}, ESS={ess:.4e}.")
            pending.append(log_ess)
            # a generation callback sees this generation's log complete (its
            # ESS read here, not deferred behind the next density)
            if not hasattr(self.sampler, "on_density_queued") or \
                    self.generation_callback is not None:
                flush()
            if self.generation_callback is not None:
                self.generation_callback(t)
            if current_eps <= minimum_epsilon:
                logger.info("Stopping: minimum epsilon.")
                break
            elif self.stop_if_only_single_model_alive \
                    and self.history.nr_of_models_alive() <= 1:
                logger.info("Stopping: single model alive.")
                break
            elif acceptance_rate < min_acceptance_rate:
                logger.info("Stopping: minimum acceptance rate.")
                break
            t += 1
        flush()
        self.history.done()
        return self.history

    @staticmethod
    def _ess_async(population):
        if population.columns is not None:
            fut = gpu.HostFuture(population._stats[1:2])
            return lambda: float(fut.get()[0])
        ess = ABCSMC._ess(population)
        return lambda: ess

    @staticmethod
    def _ess(population):
        """effective_sample_size of the normalised weights (smc.py:930)."""
        if population.columns is not None:
            return float(population._stats[1].item())
        return effective_sample_size(population.get_weighted_distances()['w'])

    def _prepare_next_iteration(self, t, sample, population, acceptance_rate):
        """smc.py:960-1040."""
        prev_transitions = copy.deepcopy(self.transitions)
        self._fit_transitions(t)
        self._adapt_population_size(t)

        def get_recorded_sum_stats():
            return sample.first_m_sum_stats(self.max_nr_recorded_particles)

        df_updated = self.distance_function.update(t, get_recorded_sum_stats)

        def get_weighted_distances():
            if df_updated:
                self._update_population_distances(population, t)
            return population.get_weighted_distances()

        self.acceptor.update(t, get_weighted_distances, self.eps(t - 1),
                             acceptance_rate)

        def get_all_records():
            dev = self._device_records(t, sample, prev_transitions)
            if dev is not None:
                return dev
            recorded_particles = sample.first_m_particles(
                self.max_nr_recorded_particles)
            records = []
            transition_pdf_prev = self._create_transition_pdf(t - 1,
                                                              prev_transitions)
            transition_pdf = self._create_transition_pdf(t)
            for particle in recorded_particles:
                all_distances = (particle.accepted_distances
                                 + particle.rejected_distances)
                tp_prev = transition_pdf_prev(particle.m, particle.parameter)
                tp = transition_pdf(particle.m, particle.parameter)
                for d in all_distances:
                    records.append({'distance': d, 'transition_pd_prev': tp_prev,
                                    'transition_pd': tp,
                                    'accepted': particle.accepted})
            return records

        self.eps.update(t, get_weighted_distances, get_all_records,
                        acceptance_rate, self.acceptor.get_epsilon_config(t))

    def _device_records(self, t, sample, prev_transitions):
        """Records of the batched sampler (smc.py:1008-1035) with the two
        transition densities evaluated for all of them on the device: log
        t_pd_prev under the transition that proposed them (the prior for
        t - 1 == 0), log t_pd under the freshly fitted one."""
        recs = getattr(sample, "device_records", None)
        if recs is None or len(self.models) != 1:
            return None
        rec = recs(self.max_nr_recorded_particles)
        if rec is None:
            return None
        theta, dist, key, anc = rec
        # a proposal that exhausted the prior re-draws (key +inf, see
        # BatchedGPUSampler) is not a candidate the reference could have
        # recorded (it loops until the prior density is positive,
        # smc.py:649-662): left out of the records
        gave_up = key == np.inf
        if bool(gave_up.any()):
            keep = ~gave_up
            theta, dist, key = theta[keep], dist[keep], key[keep]
            anc = None if anc is None else anc[keep]
        if t - 1 == 0:
            spec = self.parameter_priors[0].device_spec()
            kinds = gpu.as_dev(spec[0], dtype=gpu.torch.int32, device=theta.device)
            lp_prev = gpu.prior_logpdf(theta, kinds,
                                       gpu.as_dev(spec[1], device=theta.device))
            hl = host_prior_logpdf(theta, self.parameter_priors[0].host_components())
            if hl is not None:
                lp_prev = lp_prev + hl
        else:
            tr_prev = prev_transitions[0]
            if not hasattr(tr_prev, "logpdf_device"):
                return None
            lp_prev = tr_prev.logpdf_device(theta, hint=anc)
        tr = self.transitions[0]
        if not hasattr(tr, "logpdf_device"):
            return None
        lp = tr.logpdf_device(theta)
        return DeviceRecords(dist, lp_prev, lp, key)

    def _adapt_population_size(self, t):
        if t == 0:
            return
        if type(self.population_size).update is PopulationStrategy.update:
            # the strategy ignores the transitions (ConstantPopulationSize):
            # no copies of them, no model-probability table
            return
        w = np.array(list(self.history.model_probabilities_dict(
            self.history.max_t).values()))
        # smc.py:1042-1063: the strategy works on copies (device tensors are
        # shared by Transition.__deepcopy__, not duplicated)
        self.population_size.update(copy.deepcopy(self.transitions), w, t)

    def _fit_transitions(self, t):
        """smc.py:1065-1079; device-resident populations are fitted in
        place (no DataFrame round trip)."""
        if t == 0:
            return
        for m in self.history.alive_models(t - 1):
            cols = self.history.get_population_device(t - 1)
            tr = self.transitions[m]
            if cols is not None and hasattr(tr, "fit_device"):
                tr.fit_device(cols.theta, cols.weights, cols.param_names)
            else:
                particles, w = self.history.get_distribution(m, t - 1)
                tr.fit(particles, w)
