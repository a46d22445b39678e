"""Random variables and priors (pyabc/random_variables.py:16-538).

``RV`` / ``Distribution`` keep the reference's scipy-backed per-particle API.
``Distribution.device_spec()`` describes the prior to the GPU kernels
(kinds ABC_PRIOR_* of include/abcgpu.h) when every component is a supported
scipy family; the batched sampler refuses priors it cannot evaluate on the
device rather than falling back to the CPU.
"""
import logging
from abc import ABC, abstractmethod
from functools import reduce

import numpy as np

from .parameters import Parameter, ParameterStructure

rv_logger = logging.getLogger("RV")


class RVBase(ABC):
    @abstractmethod
    def copy(self):
        ...

    @abstractmethod
    def rvs(self, *args, **kwargs):
        ...

    @abstractmethod
    def pmf(self, x, *args, **kwargs):
        ...

    @abstractmethod
    def pdf(self, x, *args, **kwargs):
        ...

    @abstractmethod
    def cdf(self, x, *args, **kwargs):
        ...


class RV(RVBase):
    """Pickleable wrapper of ``scipy.stats.<name>(*args, **kwargs)``."""

    @classmethod
    def from_dictionary(cls, dictionary: dict):
        return cls(dictionary['type'], *dictionary.get('args', []),
                   **dictionary.get('kwargs', {}))

    def __init__(self, name: str, *args, **kwargs):
        self.name = name
        self.args = args
        self.kwargs = kwargs
        self.distribution = None
        self.__setstate__(self.__getstate__())

    def __getattr__(self, item):
        if item in ("distribution", "__setstate__", "__getstate__"):
            raise AttributeError(item)
        return getattr(self.distribution, item)

    def __getstate__(self):
        return self.name, self.args, self.kwargs

    def __setstate__(self, state):
        self.name, self.args, self.kwargs = state
        import scipy.stats as st
        self.distribution = getattr(st, self.name)(*self.args, **self.kwargs)

    def copy(self):
        return self.__class__(self.name, *self.args, **self.kwargs)

    def rvs(self, *args, **kwargs):
        return self.distribution.rvs(*args, **kwargs)

    def pmf(self, x, *args, **kwargs):
        return self.distribution.pmf(x, *args, **kwargs)

    def pdf(self, x, *args, **kwargs):
        return self.distribution.pdf(x, *args, **kwargs)

    def cdf(self, x, *args, **kwargs):
        return self.distribution.cdf(x, *args, **kwargs)

    def __repr__(self):
        return (f"<RV(name={self.name}, args={self.args} "
                f"kwargs={self.kwargs})>")

    # -- device description ------------------------------------------------
    _SHAPES = {"norm": 0, "uniform": 0, "expon": 0, "laplace": 0,
               "lognorm": 1, "gamma": 1, "beta": 2}

    def device_spec(self):
        """(kind, [4 params]) for the GPU kernels, or None if unsupported."""
        from ._native import PRIOR_KINDS
        if self.name not in self._SHAPES:
            return None
        nshape = self._SHAPES[self.name]
        dist = self.distribution
        shapes = list(dist.args[:nshape])
        rest = list(dist.args[nshape:])
        kw = dict(dist.kwds)
        shape_names = {"lognorm": ["s"], "gamma": ["a"], "beta": ["a", "b"]}
        for nm in shape_names.get(self.name, [])[len(shapes):]:
            if nm not in kw:
                return None
            shapes.append(kw.pop(nm))
        loc = rest[0] if len(rest) > 0 else kw.pop("loc", 0.0)
        scale = rest[1] if len(rest) > 1 else kw.pop("scale", 1.0)
        if kw:
            return None
        p = [float(v) for v in shapes] + [float(loc), float(scale)]
        p += [0.0] * (4 - len(p))
        return PRIOR_KINDS[self.name], p


class RVDecorator(RVBase):
    def __init__(self, component: RVBase):
        self.component = component

    def rvs(self, *args, **kwargs):
        return self.component.rvs(*args, **kwargs)

    def pmf(self, x, *args, **kwargs):
        return self.component.pmf(x, *args, **kwargs)

    def pdf(self, x, *args, **kwargs):
        return self.component.pdf(x, *args, **kwargs)

    def cdf(self, x, *args, **kwargs):
        return self.component.cdf(x, *args, **kwargs)

    def copy(self):
        return self.__class__(self.component.copy())

    def decorator_repr(self):
        return "Decorator"

    def __repr__(self):
        return f"[{self.decorator_repr()}]" + self.component.__repr__()

    def device_spec(self):
        return None


class LowerBoundDecorator(RVDecorator):
    """pyabc/random_variables.py:263-325 (host only)."""
    MAX_TRIES = 10000

    def __init__(self, component: RV, lower_bound: float):
        if component.cdf(lower_bound) == 1:
            raise Exception(
                "LowerBoundDecorator: Conditioning on a set of measure zero.")
        self.lower_bound = lower_bound
        super().__init__(component)

    def copy(self):
        return self.__class__(self.component.copy(), self.lower_bound)

    def decorator_repr(self):
        return "Lower: X > {lower:2f}".format(lower=self.lower_bound)

    def rvs(self, *args, **kwargs):
        for _ in range(LowerBoundDecorator.MAX_TRIES):
            sample = self.component.rvs()
            if not (sample <= self.lower_bound):
                return sample
        return None

    def pdf(self, x, *args, **kwargs):
        if x <= self.lower_bound:
            return 0.
        return (self.component.pdf(x)
                / (1 - self.component.cdf(self.lower_bound)))

    def pmf(self, x, *args, **kwargs):
        if x <= self.lower_bound:
            return 0.
        return (self.component.pmf(x)
                / (1 - self.component.cdf(self.lower_bound)))

    def cdf(self, x, *args, **kwargs):
        if x <= self.lower_bound:
            return 0.
        lower_mass = self.component.cdf(self.lower_bound)
        return (self.component.cdf(x) - lower_mass) / (1 - lower_mass)


class Distribution(ParameterStructure):
    """Independent product of RVs: the prior of a model."""

    def __repr__(self):
        return "<Distribution {keys}>".format(
            keys=str(list(self.get_parameter_names()))[1:-1])

    @classmethod
    def from_dictionary_of_dictionaries(cls, dict_of_dicts: dict):
        return cls({key: RV.from_dictionary(value)
                    for key, value in dict_of_dicts.items()})

    def copy(self):
        return self.__class__(**{key: value.copy()
                                 for key, value in self.items()})

    def update_random_variables(self, **random_variables):
        self.update(random_variables)

    def get_parameter_names(self) -> list:
        return sorted(self.keys())

    def rvs(self) -> Parameter:
        return Parameter(**{key: val.rvs() for key, val in self.items()})

    def pdf(self, x):
        if sorted(x.keys()) != sorted(self.keys()):
            raise Exception("Random variable parameter mismatch. Expected: " +
                            str(sorted(self.keys())) +
                            " got " + str(sorted(x.keys())))
        if len(self) > 0:
            res = []
            for key, val in x.items():
                try:
                    res.append(self[key].pdf(val))
                except AttributeError:
                    res.append(self[key].pmf(val))
            return reduce(lambda s, t: s * t, res)
        return 1

    def device_spec(self):
        """(kinds [d] int32, params [d*4] float64) in sorted-name order, or
        None when a component has no device implementation."""
        kinds, params = [], []
        for name in self.get_parameter_names():
            rv = self[name]
            spec = rv.device_spec() if hasattr(rv, "device_spec") else None
            if spec is None:
                return None
            kinds.append(spec[0])
            params.extend(spec[1])
        return np.asarray(kinds, dtype=np.int32), np.asarray(params, np.float64)


class ModelPerturbationKernel:
    """pyabc/random_variables.py:455-538."""

    def __init__(self, nr_of_models: int, probability_to_stay=None):
        self.nr_of_models = nr_of_models
        if nr_of_models == 1:
            self.probability_to_stay = 1
        else:
            if probability_to_stay is None:
                self.probability_to_stay = 1 / nr_of_models
            else:
                self.probability_to_stay = min(max(probability_to_stay, 0), 1)

    def _get_discrete_rv(self, m):
        p_stay = self.probability_to_stay
        p_move = (1 - p_stay) / (self.nr_of_models - 1)
        probabilities = [p_stay if n == m else p_move
                         for n in range(self.nr_of_models)]
        return RV('rv_discrete',
                  values=(range(len(probabilities)), probabilities))

    def rvs(self, m: int) -> int:
        if not 0 <= m <= self.nr_of_models - 1:
            raise Exception('m has to be between 0 and nr_of_models - 1')
        if self.nr_of_models == 1:
            return 0
        return self._get_discrete_rv(m).rvs()

    def pmf(self, n: int, m: int) -> float:
        if not (0 <= n <= self.nr_of_models
                and 0 <= m <= self.nr_of_models - 1):
            raise Exception(
                'n and m have to be between 0 and nr_of_models - 1')
        if self.nr_of_models == 1:
            return 1 if n == m else 0
        return self._get_discrete_rv(m).pmf(n)
