"""Models (pyabc/model.py:15-270) plus the vectorised model the batched GPU
sampler drives.

The reference evaluates one parameter at a time (Model.accept,
model.py:163-218).  ``VectorizedModel`` is the batched boundary: a callable
mapping a device tensor theta [B, d] (columns = sorted parameter names) to a
device tensor of summary statistics [B, S] (columns = ``sum_stat_keys``,
matching x_0's key order).  ``LinearGaussianModel`` is the built-in HIP
simulator used by the benchmark configurations.
"""
import numpy as np

from .parameters import Parameter


class ModelResult:
    def __init__(self, sum_stats=None, distance=None, accepted=None,
                 weight=1.0):
        self.sum_stats = sum_stats if sum_stats is not None else {}
        self.distance = distance
        self.accepted = accepted
        self.weight = weight


class Model:
    def __init__(self, name: str = "model"):
        self.name = name

    def __repr__(self):
        return "<{} {}>".format(self.__class__.__name__, self.name)

    def sample(self, pars):
        raise NotImplementedError()

    def summary_statistics(self, t, pars, sum_stats_calculator) -> ModelResult:
        raw_data = self.sample(pars)
        sum_stats = sum_stats_calculator(raw_data)
        return ModelResult(sum_stats=sum_stats)

    def distance(self, t, pars, sum_stats_calculator, distance_calculator,
                 x_0) -> ModelResult:
        res = self.summary_statistics(t, pars, sum_stats_calculator)
        res.distance = distance_calculator(res.sum_stats, x_0, t, pars)
        return res

    def accept(self, t, pars, sum_stats_calculator, distance_calculator,
               eps_calculator, acceptor, x_0):
        result = self.summary_statistics(t, pars, sum_stats_calculator)
        acc_res = acceptor(distance_function=distance_calculator,
                           eps=eps_calculator, x=result.sum_stats, x_0=x_0,
                           t=t, par=pars)
        result.distance = acc_res.distance
        result.accepted = acc_res.accept
        result.weight = acc_res.weight
        return result


class IntegratedModel(Model):
    """A model that simulates and decides acceptance in one call, so it can
    stop a simulation early once eps is out of reach (the role of
    pyabc/model.py:273-328).  Subclasses implement ``integrated_simulate``
    and return ``ModelResult(accepted=False)`` for a rejection, or
    ``ModelResult(accepted=True, distance=..., sum_stats=...)``.  Runs on the
    per-candidate path (it is not a ``VectorizedModel``)."""

    def integrated_simulate(self, pars, eps: float) -> ModelResult:
        raise NotImplementedError()

    def accept(self, t, pars, sum_stats_calculator, distance_calculator,
               eps_calculator, acceptor, x_0):
        return self.integrated_simulate(pars, eps_calculator(t))


class SimpleModel(Model):
    def __init__(self, sample_function, name=None):
        if name is None:
            name = sample_function.__name__
        super().__init__(name)
        self.sample_function = sample_function

    def sample(self, pars):
        return self.sample_function(pars)

    @staticmethod
    def assert_model(model_or_function):
        if isinstance(model_or_function, Model):
            return model_or_function
        return SimpleModel(model_or_function)


class VectorizedModel(Model):
    """Batched simulator: ``simulate_batch(theta, seed, generation, idx0)``
    returns device sum stats [B, S] in ``sum_stat_keys`` order.  ``seed``,
    ``generation`` and ``idx0`` (the global index of row 0) let a simulator
    key its noise like the rest of the engine, so results are independent of
    batching and rank count."""

    def __init__(self, simulate_batch, sum_stat_keys, name="model"):
        super().__init__(name)
        self._simulate_batch = simulate_batch
        self.sum_stat_keys = list(sum_stat_keys)
        self._counter = 0
        self._seed = None

    def simulate_batch(self, theta, seed, generation, idx0):
        return self._simulate_batch(theta, seed, generation, idx0)

    def sample(self, pars):
        """Per-particle path (reference interface): a batch of one."""
        from . import gpu
        names = sorted(pars.keys())
        theta = gpu.as_dev(np.array([[pars[k] for k in names]], dtype=np.float64))
        if self._seed is None:
            self._seed = int(np.random.randint(0, 2 ** 62))
        x = self.simulate_batch(theta, self._seed, 0xFFFFFFFF, self._counter)
        self._counter += 1
        return dict(zip(self.sum_stat_keys, x.cpu().numpy()[0]))


class LinearGaussianModel(VectorizedModel):
    """x_k = a_k * theta[src_k] + sigma_k * eps_k (abc_simulate_linear_gaussian).

    Covers the benchmark configurations: the conjugate Gaussian models
    (src_k = k, a = 1, sigma = 0.5) and the 256-statistic heterogeneous-scale
    model of config 4 (src_k = k mod 4, a_k, sigma_k fixed by a seed)."""

    def __init__(self, parameter_names, sum_stat_keys, src, a=None,
                 sigma=None, name="linear_gaussian"):
        super().__init__(self._run, sum_stat_keys, name)
        self.parameter_names = sorted(parameter_names)
        S = len(self.sum_stat_keys)
        self.src = np.asarray(src, dtype=np.int32)
        self.a = np.ones(S) if a is None else np.asarray(a, dtype=np.float64)
        self.sigma = (np.ones(S) if sigma is None
                      else np.asarray(sigma, dtype=np.float64))
        if not (len(self.src) == len(self.a) == len(self.sigma) == S):
            raise ValueError("src, a, sigma need one entry per sum stat")
        if S and (self.src.min() < 0 or self.src.max() >= len(self.parameter_names)):
            raise ValueError("src entries must index the parameters")
        self._dev = None

    def _device_arrays(self, device):
        if self._dev is None or self._dev[0].device != device:
            from . import gpu
            self._dev = (gpu.as_dev(self.src, dtype=gpu.torch.int32, device=device),
                         gpu.as_dev(self.a, device=device),
                         gpu.as_dev(self.sigma, device=device))
        return self._dev

    def fused_simulator(self, device):
        """(src int32, a, sigma) device arrays for the fused candidate kernel
        (abc_candidate_spec); None when a subclass replaced the simulator."""
        if type(self)._run is not LinearGaussianModel._run or \
                type(self).simulate_batch is not VectorizedModel.simulate_batch:
            return None
        return self._device_arrays(device)

    def _run(self, theta, seed, generation, idx0):
        from . import gpu
        src, a, sigma = self._device_arrays(theta.device)
        return gpu.simulate_linear_gaussian(theta, src, a, sigma, seed,
                                            generation, idx0)

    def __getstate__(self):
        s = self.__dict__.copy()
        s["_dev"] = None
        return s

