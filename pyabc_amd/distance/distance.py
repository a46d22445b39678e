"""PNormDistance / AdaptivePNormDistance on the GPU.

Reference: pyabc/distance/distance.py
  PNormDistance.__call__           :79-105  (Python loop over keys)
  format_dict / get_for_t_or_latest :113-136
  AdaptivePNormDistance            :139-363 (configure_sampler :210-224,
                                    initialize :226-245, update :247-261,
                                    _update :263-307, _normalize_weights
                                    :309-323, _bound_weights :325-348)
Distances are evaluated by abc_pnorm over a device sum-stat matrix whose
columns follow x_0's key order; the adaptive scales by abc_column_std /
abc_column_mad over all recorded sum stats (accepted and rejected).
"""
import logging

import numpy as np

from .. import gpu
from .base import Distance
from .scale import standard_deviation

logger = logging.getLogger("Distance")


class SumStatMatrix:
    """Device-resident recorded sum stats: ``data`` [R, S] float64 tensor with
    columns in ``keys`` order.  Behaves like the reference's list of dicts
    when iterated (materialised lazily)."""

    def __init__(self, data, keys):
        self.data = data
        self.keys = list(keys)
        self._list = None

    def _materialise(self):
        if self._list is None:
            arr = self.data.cpu().numpy()
            self._list = [dict(zip(self.keys, row)) for row in arr]
        return self._list

    def __len__(self):
        return int(self.data.shape[0])

    def __iter__(self):
        return iter(self._materialise())

    def __getitem__(self, i):
        return self._materialise()[i]


class PNormDistance(Distance):
    def __init__(self, p: float = 2, weights: dict = None, factors: dict = None):
        super().__init__()
        if p < 1:
            raise ValueError("It must be p >= 1")
        self.p = p
        self.weights = weights
        self.factors = factors
        self._dev_wf_cache = {}

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t, get_all_sum_stats, x_0)
        self.format_weights_and_factors(t, x_0.keys())

    def format_weights_and_factors(self, t, sum_stat_keys):
        self.weights = PNormDistance.format_dict(self.weights, t, sum_stat_keys)
        self.factors = PNormDistance.format_dict(self.factors, t, sum_stat_keys)

    # -- device path -------------------------------------------------------
    def weight_vector(self, t, keys):
        """w * f per key (x_0 order) for generation t; a key absent from the
        weight dict contributes 0 (distance.py:96-104)."""
        self.format_weights_and_factors(t, keys)
        w = PNormDistance.get_for_t_or_latest(self.weights, t)
        f = PNormDistance.get_for_t_or_latest(self.factors, t)
        return np.array([(f[k] * w[k]) if (k in w and k in f) else 0.0
                         for k in keys], dtype=np.float64)

    def device_call(self, xmat, x0vec, t, keys, out=None):
        """Distances of B simulations (device [B, S], columns in ``keys``
        order) to x_0 (device [S])."""
        return gpu.pnorm(xmat, x0vec, self._device_weights(t, keys, xmat.device),
                         float(self.p), out=out)

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_dev_wf_cache"] = {}     # device tensors stay per process
        return state

    def _device_weights(self, t, keys, device):
        """weight_vector(t, keys) on the device, uploaded only when it changed
        (a pageable host-to-device copy synchronises the stream: once per
        round of the staged sampler otherwise)."""
        wv = np.ascontiguousarray(self.weight_vector(t, keys), dtype=np.float64)
        key = (wv.tobytes(), str(device))
        cache = self.__dict__.setdefault("_dev_wf_cache", {})
        if key not in cache:
            cache.clear()
            cache[key] = gpu.as_dev(wv, device=device)
        return cache[key]

    def fused_pnorm(self, t, keys, device):
        """(wf device [S], p) for the fused candidate kernel, or None when a
        subclass replaced the distance itself."""
        cls = type(self)
        if cls.device_call is not PNormDistance.device_call or \
                cls.__call__ is not PNormDistance.__call__ or \
                cls.weight_vector is not PNormDistance.weight_vector:
            return None
        return self._device_weights(t, keys, device), float(self.p)

    # -- reference per-particle interface ----------------------------------
    def __call__(self, x: dict, x_0: dict, t: int = None, par: dict = None):
        self.format_weights_and_factors(t, x_0.keys())
        w = PNormDistance.get_for_t_or_latest(self.weights, t)
        f = PNormDistance.get_for_t_or_latest(self.factors, t)
        keys = list(w)
        # keys missing in x or x_0 contribute 0: zero weight, dummy values
        wf = np.array([f[k] * w[k] if (k in x and k in x_0) else 0.0
                       for k in keys], dtype=np.float64)
        xv = np.array([[float(x[k]) if k in x and k in x_0 else 0.0
                        for k in keys]], dtype=np.float64)
        x0v = np.array([float(x_0[k]) if k in x and k in x_0 else 0.0
                        for k in keys], dtype=np.float64)
        d = gpu.pnorm(gpu.as_dev(xv), gpu.as_dev(x0v), gpu.as_dev(wf),
                      float(self.p))
        return float(d.cpu()[0])

    def get_config(self) -> dict:
        return {"name": self.__class__.__name__, "p": self.p,
                "weights": self.weights, "factors": self.factors}

    @staticmethod
    def format_dict(w, t, sum_stat_keys, default_val=1.):
        if w is None:
            w = {t: {k: default_val for k in sum_stat_keys}}
        elif not isinstance(next(iter(w.values())), dict):
            w = {t: w}
        return w

    @staticmethod
    def get_for_t_or_latest(w, t):
        if t not in w:
            t = max(w)
        return w[t]


class AdaptivePNormDistance(PNormDistance):
    def __init__(self, p: float = 2, initial_weights: dict = None,
                 factors: dict = None, adaptive: bool = True,
                 scale_function=None, normalize_weights: bool = True,
                 max_weight_ratio: float = None, log_file: str = None):
        super().__init__(p=p, weights=None, factors=factors)
        self.initial_weights = initial_weights
        self.factors = factors
        self.adaptive = adaptive
        if scale_function is None:
            scale_function = standard_deviation
        self.scale_function = scale_function
        self.normalize_weights = normalize_weights
        self.max_weight_ratio = max_weight_ratio
        self.log_file = log_file
        self.x_0 = None

    def configure_sampler(self, sampler):
        if self.adaptive:
            sampler.sample_factory.record_rejected = True

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t, get_all_sum_stats, x_0)
        self.x_0 = x_0
        if self.initial_weights is not None:
            self.weights[t] = self.initial_weights
            return
        self._update(t, get_all_sum_stats())

    def update(self, t, get_all_sum_stats):
        if not self.adaptive:
            return False
        self._update(t, get_all_sum_stats())
        return True

    def _scales(self, all_sum_stats, keys):
        kern = getattr(self.scale_function, "device_kernel", None)
        if isinstance(all_sum_stats, SumStatMatrix) and all_sum_stats.keys == keys:
            mat = all_sum_stats.data
        elif kern is not None:
            if any(not all(k in s for k in keys) for s in all_sum_stats):
                mat = None     # ragged: per-key path below (distance.py:278-283)
            else:
                rows = [[float(s[k]) for k in keys] for s in all_sum_stats]
                mat = gpu.as_dev(np.asarray(rows, dtype=np.float64).reshape(-1, len(keys)))
        else:
            mat = None
        if kern is not None and mat is not None:
            col = gpu.column_std(mat) if kern == "std" else gpu.column_mad(mat)
            return col.cpu().numpy()
        scales = []
        for key in keys:
            current = [s[key] for s in all_sum_stats if key in s]
            scales.append(self.scale_function(data=current, x_0=self.x_0[key]))
        return np.asarray(scales, dtype=np.float64)

    def _update(self, t, all_sum_stats):
        # distance.py:263-348 with the per-key loops as array operations (the
        # same IEEE operations per key: 1 / scale, / mean, the ratio bound;
        # ~1 ms of host time per generation at S = 256 otherwise)
        keys = list(self.x_0.keys())
        scales = np.asarray(self._scales(all_sum_stats, keys), dtype=np.float64)
        zero = np.isclose(scales, 0)
        with np.errstate(divide="ignore"):
            w = np.where(zero, 0.0, 1.0 / np.where(zero, 1.0, scales))
        w = self._normalize_weights(w)
        w = self._bound_weights(w)
        self.weights[t] = dict(zip(keys, w.tolist()))
        self.log(t)

    def _normalize_weights(self, w):
        if not self.normalize_weights:
            return w
        return w / np.mean(w)

    def _bound_weights(self, w):
        if self.max_weight_ratio is None:
            return w
        min_abs_weight = np.min(np.abs(w[w != 0]))
        over = np.abs(w) / min_abs_weight > self.max_weight_ratio
        return np.where(over, np.sign(w) * self.max_weight_ratio * min_abs_weight, w)

    def get_config(self) -> dict:
        return {"name": self.__class__.__name__, "p": self.p,
                "factors": self.factors, "adaptive": self.adaptive,
                "scale_function": self.scale_function.__name__,
                "normalize_weights": self.normalize_weights,
                "max_weight_ratio": self.max_weight_ratio}

    def log(self, t):
        # formatted only when emitted: the S-key dict's repr is ~0.2 ms at S = 256
        logger.debug("updated weights[%s] = %s", t, self.weights[t])
        if self.log_file:
            import json
            with open(self.log_file, "w") as f:
                json.dump({str(k): {kk: float(vv) for kk, vv in v.items()}
                           for k, v in self.weights.items()}, f)
