"""Stochastic kernels (noise models) on the GPU.

Reference: pyabc/distance/kernel.py
  StochasticKernel          :18-97   (ret_scale, keys = sorted(x_0), pdf_max)
  SimpleFunctionKernel      :100-150
  NormalKernel              :153-226 (scipy multivariate_normal(0, cov))
  IndependentNormalKernel   :229-303
  IndependentLaplaceKernel  :306-378
  BinomialKernel            :381-445, binomial_pdf_max :555-566
  PoissonKernel             :448-495
  NegativeBinomialKernel    :498-552
  _diff_arr / _arr          :569-592

A kernel's value is the log (SCALE_LOG) or linear (SCALE_LIN) density of the
observed data x_0 given a simulation x.  ``device_call`` evaluates it for a
whole candidate batch (device sum-stat matrix [B, S], columns in x_0 key
order) with one abc_kernel_logpdf launch; ``__call__`` is the reference's
per-particle interface (dicts, array-valued keys allowed) and runs the same
kernel on one row.  Parameters given as callables of the particle parameters
(``var(par)``, ``scale(par)``, ``p(par)``) are evaluated on the host per call
and are not batched (``device_spec`` returns None for them).
"""
from typing import Callable, List, Union

import numpy as np

from .. import gpu
from ..transition.multivariatenormal import psd_whitening
from .base import Distance

SCALE_LIN = "SCALE_LIN"
SCALE_LOG = "SCALE_LOG"
SCALES = [SCALE_LIN, SCALE_LOG]

_LOG_2PI = float(np.log(2) + np.log(np.pi))


def _arr(x, keys):
    """Flatten the values of keys (scalars or arrays) into one vector
    (kernel.py:581-592)."""
    arr = []
    for key in keys:
        val = x[key]
        try:
            arr.extend(val)
        except Exception:
            arr.append(val)
    return np.asarray(arr)


def _diff_arr(x, x_0, keys):
    """kernel.py:569-578."""
    diff = []
    for key in keys:
        d = x[key] - x_0[key]
        try:
            diff.extend(d)
        except Exception:
            diff.append(d)
    return np.asarray(diff)


class StochasticKernel(Distance):
    """Base class (kernel.py:18-97)."""

    #: abc_kernel_logpdf kind of the subclass (None: no device kernel)
    KIND = None

    def __init__(self, ret_scale: str = SCALE_LIN, keys: List[str] = None,
                 pdf_max: float = None):
        StochasticKernel.check_ret_scale(ret_scale)
        self.ret_scale = ret_scale
        self.keys = keys
        self.pdf_max = pdf_max
        self._dev_cache = {}

    def initialize(self, t: int, get_all_sum_stats: Callable[[], List[dict]],
                   x_0: dict = None):
        if self.keys is None:
            self.initialize_keys(x_0)

    @staticmethod
    def check_ret_scale(ret_scale):
        if ret_scale not in SCALES:
            raise ValueError(
                f"The ret_scale {ret_scale} must be one of {SCALES}.")

    def initialize_keys(self, x):
        self.keys = sorted(x)

    def get_config(self):
        return {"name": self.__class__.__name__, "ret_scale": self.ret_scale,
                "keys": self.keys, "pdf_max": self.pdf_max}

    # -- device path -------------------------------------------------------
    def device_spec(self, dim):
        """(par [K], c, U or None) for abc_kernel_logpdf, or None when a
        parameter is a callable of the particle parameters."""
        return None

    def _values(self, xmat, cols, x0k, spec, out=None):
        par, c, U = spec
        dev = xmat.device
        return gpu.kernel_logpdf(
            xmat, cols, x0k, self.KIND, gpu.as_dev(par, device=dev), c,
            U=None if U is None else gpu.as_dev(U, device=dev),
            ret_lin=self.ret_scale == SCALE_LIN, out=out)

    @property
    def batched_capable(self):
        return self.KIND is not None and self.device_spec(1) is not None

    def device_call(self, xmat, x0vec, t, keys, out=None):
        """Kernel values of B simulations (device [B, S], columns in ``keys``
        order = x_0 key order) against x_0 (device [S])."""
        keys = list(keys)
        if self.keys is None:
            self.keys = sorted(keys)
        ck = (tuple(keys), tuple(self.keys), str(xmat.device))
        if ck not in self._dev_cache:
            missing = [k for k in self.keys if k not in keys]
            if missing:
                raise KeyError(f"kernel keys {missing} not in the sum stats")
            idx = [keys.index(k) for k in self.keys]
            cols = gpu.as_dev(np.asarray(idx, dtype=np.int32),
                              dtype=gpu.torch.int32, device=xmat.device)
            x0k = x0vec[cols.long()].contiguous()
            if self.KIND in ("poisson", "binomial", "negative_binomial"):
                x0k = x0k.trunc()
            spec = self.device_spec(len(idx))
            if spec is None:
                raise TypeError(f"{type(self).__name__} with callable "
                                "parameters has no batched device kernel")
            self._dev_cache.clear()
            self._dev_cache[ck] = (cols, x0k, spec)
        cols, x0k, spec = self._dev_cache[ck]
        return self._values(xmat, cols, x0k, spec, out=out)

    def _row_call(self, xv, x0v, spec):
        """One particle through the device kernel: xv, x0v flat host
        vectors in kernel key order."""
        dev = gpu.require_device()
        K = xv.size
        xm = gpu.as_dev(np.asarray(xv, dtype=np.float64).reshape(1, K), device=dev)
        cols = gpu.as_dev(np.arange(K, dtype=np.int32), dtype=gpu.torch.int32,
                          device=dev)
        x0k = gpu.as_dev(np.asarray(x0v, dtype=np.float64), device=dev)
        return float(self._values(xm, cols, x0k, spec).cpu()[0])

    def __deepcopy__(self, memo):
        import copy
        new = self.__class__.__new__(self.__class__)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            setattr(new, k, {} if k == "_dev_cache" else copy.deepcopy(v, memo))
        return new


class SimpleFunctionKernel(StochasticKernel):
    """kernel.py:100-150 (user function; per-particle only)."""

    def __init__(self, fun: Callable, ret_scale: str = SCALE_LIN,
                 keys: List[str] = None, pdf_max: float = None):
        super().__init__(ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)
        self.fun = fun

    def __call__(self, x: dict, x_0: dict, t: int = None,
                 par: dict = None) -> float:
        return self.fun(x=x, x_0=x_0, t=t, par=par)


class NormalKernel(StochasticKernel):
    """kernel.py:153-226: log N(x - x_0; 0, cov) (scipy semantics,
    allow_singular=False)."""
    KIND = "normal"

    def __init__(self, cov: np.ndarray = None, ret_scale: str = SCALE_LOG,
                 keys: List[str] = None, pdf_max: float = None):
        super().__init__(ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)
        self.cov = cov
        self._psd = None

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t=t, get_all_sum_stats=get_all_sum_stats, x_0=x_0)
        self._init_distr(x_0)
        if self.pdf_max is None:
            self.pdf_max = self(x_0, x_0)

    def _init_distr(self, x_0):
        if self.cov is None:
            dim = sum(np.size(x_0[key]) for key in self.keys)
            self.cov = np.eye(dim)
        self.cov = np.atleast_2d(np.asarray(self.cov, dtype=np.float64))
        psd = psd_whitening(self.cov)
        if psd["rank"] < self.cov.shape[0]:
            raise np.linalg.LinAlgError("singular matrix")
        self._psd = psd
        self._dev_cache = {}

    def device_spec(self, dim):
        if self._psd is None:
            return None
        psd = self._psd
        return (np.zeros(1), psd["rank"] * _LOG_2PI + psd["log_pdet"],
                np.ascontiguousarray(psd["U"]))

    def __call__(self, x: dict, x_0: dict, t: int = None,
                 par: dict = None) -> float:
        if self.keys is None:
            self.initialize_keys(x_0)
        if self._psd is None:
            self._init_distr(x_0)
        xv, x0v = _arr(x, self.keys), _arr(x_0, self.keys)
        return self._row_call(xv.astype(np.float64), x0v.astype(np.float64),
                              self.device_spec(xv.size))


class _IndependentKernel(StochasticKernel):
    """Shared parameter handling of the independent normal / Laplace
    kernels (kernel.py:271-283, 347-359)."""
    _PARAM = None

    def __init__(self, param, keys=None, pdf_max=None):
        super().__init__(ret_scale=SCALE_LOG, keys=keys, pdf_max=pdf_max)
        setattr(self, self._PARAM, param)

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t=t, get_all_sum_stats=get_all_sum_stats, x_0=x_0)
        dim = sum(np.size(x_0[key]) for key in self.keys)
        val = getattr(self, self._PARAM)
        if val is None:
            val = np.ones(dim)
        if not callable(val):
            val = np.asarray(val) * np.ones(dim)
        setattr(self, self._PARAM, val)
        self._dev_cache = {}
        if self.pdf_max is None and not callable(val):
            self.pdf_max = self(x_0, x_0)

    def _const(self, v):
        raise NotImplementedError

    def _param_vector(self, par, n):
        val = getattr(self, self._PARAM)
        v = np.asarray(val(par) if callable(val) else val, dtype=np.float64)
        if v.size == 1:
            v = v * np.ones(n)
        return v.ravel()

    def device_spec(self, dim):
        val = getattr(self, self._PARAM)
        if val is None or callable(val):
            return None
        v = self._param_vector(None, dim)
        return v, self._const(v), None

    def __call__(self, x: dict, x_0: dict, t: int = None, par: dict = None):
        if self.keys is None:
            self.initialize_keys(x_0)
        xv = _arr(x, self.keys).astype(np.float64)
        x0v = _arr(x_0, self.keys).astype(np.float64)
        v = self._param_vector(par, xv.size)
        return self._row_call(xv, x0v, (v, self._const(v), None))


class IndependentNormalKernel(_IndependentKernel):
    """kernel.py:229-303: -0.5 (sum log(2 pi var) + sum diff^2 / var)."""
    KIND = "independent_normal"
    _PARAM = "var"

    def __init__(self, var: Union[Callable, List[float], float] = None,
                 keys: List[str] = None, pdf_max: float = None):
        super().__init__(var, keys=keys, pdf_max=pdf_max)

    def _const(self, v):
        return float(np.sum(np.log(2) + np.log(np.pi) + np.log(v)))


class IndependentLaplaceKernel(_IndependentKernel):
    """kernel.py:306-378: -(sum log(2 b) + sum |diff| / b)."""
    KIND = "independent_laplace"
    _PARAM = "scale"

    def __init__(self, scale: Union[Callable, List[float], float] = None,
                 keys: List[str] = None, pdf_max: float = None):
        super().__init__(scale, keys=keys, pdf_max=pdf_max)
        self.dim = None

    def _const(self, v):
        return float(np.sum(np.log(2) + np.log(v)))


class _CountKernel(StochasticKernel):
    """Poisson / binomial / negative binomial observation models: x and
    x_0 are cast to int (kernel.py:432-433, 484-485, 539-540)."""

    def __init__(self, p=None, ret_scale=SCALE_LOG, keys=None, pdf_max=None):
        super().__init__(ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)
        if p is not None and not callable(p) and (p > 1 or p < 0):
            raise ValueError(
                f"The success probability p={p} must be in the interval"
                f"[0, 1].")
        self.p = p

    def device_spec(self, dim):
        if callable(self.p):
            return None
        return (np.array([0.0 if self.p is None else float(self.p)]), 0.0,
                None)

    def __call__(self, x: dict, x_0: dict, t: int = None,
                 par: dict = None) -> float:
        if self.keys is None:
            self.initialize_keys(x_0)
        xv = np.asarray(_arr(x, self.keys), dtype=int).astype(np.float64)
        x0v = np.asarray(_arr(x_0, self.keys), dtype=int).astype(np.float64)
        if callable(self.p):
            p = np.asarray(self.p(par), dtype=np.float64).ravel()
            if p.size > 1:
                # per-element p: one single-element launch per entry
                vals = [self._row_call(xv[j:j + 1], x0v[j:j + 1],
                                       (np.array([p[j]]), 0.0, None))
                        for j in range(xv.size)]
                if self.ret_scale == SCALE_LIN:
                    return float(np.prod(vals))
                return float(np.sum(vals))
            spec = (p[:1], 0.0, None)
        else:
            spec = self.device_spec(xv.size)
        return self._row_call(xv, x0v, spec)


class BinomialKernel(_CountKernel):
    """kernel.py:381-445: sum binom.logpmf(k=x_0, n=x, p)."""
    KIND = "binomial"

    def __init__(self, p: Union[float, Callable], ret_scale: str = SCALE_LOG,
                 keys: List[str] = None, pdf_max: float = None):
        super().__init__(p, ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t=t, get_all_sum_stats=get_all_sum_stats, x_0=x_0)
        if self.pdf_max is None and not callable(self.p):
            self.pdf_max = binomial_pdf_max(x_0, self.keys, self.p,
                                            self.ret_scale)


class PoissonKernel(_CountKernel):
    """kernel.py:448-495: sum poisson.logpmf(k=x_0, mu=x)."""
    KIND = "poisson"

    def __init__(self, ret_scale: str = SCALE_LOG, keys: List[str] = None,
                 pdf_max: float = None):
        super().__init__(None, ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t=t, get_all_sum_stats=get_all_sum_stats, x_0=x_0)
        if self.pdf_max is None:
            self.pdf_max = self(x_0, x_0)


class NegativeBinomialKernel(_CountKernel):
    """kernel.py:498-552: sum nbinom.logpmf(k=x_0, n=x, p)."""
    KIND = "negative_binomial"

    def __init__(self, p: float, ret_scale: str = SCALE_LOG,
                 keys: List[str] = None, pdf_max: float = None):
        super().__init__(p, ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)


def binomial_pdf_max(x_0, keys, p, ret_scale):
    """kernel.py:555-566: the binomial log pmf is maximal in n at
    n = max(ceil((k - p) / p), 0); evaluated by the device kernel."""
    ks = np.asarray(_arr(x_0, keys), dtype=int).astype(np.float64)
    ns = np.maximum(np.ceil((ks - p) / p), 0)
    k = BinomialKernel(p, ret_scale=SCALE_LOG, keys=list(range(ks.size)))
    log_pdf_max = k._row_call(ns, ks, k.device_spec(ks.size))
    if ret_scale == SCALE_LIN:
        return np.exp(log_pdf_max)
    return log_pdf_max
