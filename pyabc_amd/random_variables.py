"""Priors: pyABC's ``RV`` / ``Distribution`` interface
(pyabc/random_variables.py:111-196 and :328-452) over ``scipy.stats``, plus
the description the batched sampler needs to evaluate them.

Per-candidate use (the reference's closure, SingleCoreSampler) goes straight
to scipy.  For the batched GPU path every component becomes one of the
device prior kinds of include/abcgpu.h:

* the seven families the kernels implement (norm, uniform, expon, laplace,
  lognorm, gamma, beta) -> their own kind and parameters;
* any other scipy distribution -> ``ABC_PRIOR_HOST``: the device only knows
  its support interval [lo, hi] (``dist.support()``) for the proposal's
  re-draw test (smc.py:654-656) and a point inside it; the density and the
  t = 0 draws of that coordinate are a vectorised host-scipy leg
  (``host_logpdf`` on the accepted rows, ``host_ppf`` of the device's own
  per-candidate uniforms), so the rest of the generation stays on the device
  and the draws stay keyed by the global candidate index.

The HOST kind assumes the density is positive inside the support interval
(true of scipy's continuous families).  Discrete distributions outside the
device families and non-frozen scipy objects have no batched form
(``device_spec`` is None): such priors run the per-candidate loop, which
re-draws until the prior density is positive as the reference does.
"""
import logging
from abc import ABC, abstractmethod

import numpy as np

from .parameters import Parameter, ParameterStructure

rv_logger = logging.getLogger("RV")

# scipy family -> (number of shape parameters, their keyword names)
_DEVICE_FAMILIES = {"norm": (), "uniform": (), "expon": (), "laplace": (),
                    "lognorm": ("s",), "gamma": ("a",), "beta": ("a", "b")}


class RVBase(ABC):
    """The interface a prior component offers (random_variables.py:16-108)."""

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


def _frozen(name, args, kwargs):
    import scipy.stats
    return getattr(scipy.stats, name)(*args, **kwargs)


def _rebuild_rv(name, args, kwargs):
    return RV(name, *args, **kwargs)


class RV(RVBase):
    """``scipy.stats.<name>(*args, **kwargs)`` that pickles by its recipe.

    ``name``, ``args``, ``kwargs`` and the frozen ``distribution`` are
    public as in the reference; unknown attributes (``mean``, ``ppf``, ...)
    are looked up on the frozen distribution."""

    def __init__(self, name: str, *args, **kwargs):
        self.name = name
        self.args = args
        self.kwargs = kwargs
        self.distribution = _frozen(name, args, kwargs)

    @classmethod
    def from_dictionary(cls, dictionary: dict):
        """{"type": name, "args": [...], "kwargs": {...}}."""
        return cls(dictionary["type"], *dictionary.get("args", []),
                   **dictionary.get("kwargs", {}))

    def __reduce__(self):
        return _rebuild_rv, (self.name, self.args, self.kwargs)

    def __getattr__(self, item):
        # only reached for names not set in __init__; "distribution" itself
        # missing means a half-built object (unpickling): no recursion
        if item == "distribution":
            raise AttributeError(item)
        return getattr(self.distribution, item)

    def copy(self):
        return RV(self.name, *self.args, **self.kwargs)

    def rvs(self, *args, **kwargs):
        return self.distribution.rvs(*args, **kwargs)

    def pdf(self, x, *args, **kwargs):
        return self.distribution.pdf(x, *args, **kwargs)

    def pmf(self, x, *args, **kwargs):
        return self.distribution.pmf(x, *args, **kwargs)

    def cdf(self, x, *args, **kwargs):
        return self.distribution.cdf(x, *args, **kwargs)

    def __repr__(self):
        return f"<RV(name={self.name}, args={self.args} kwargs={self.kwargs})>"

    # -- batched-sampler description -----------------------------------------
    @property
    def is_discrete(self):
        import scipy.stats
        dist = getattr(self.distribution, "dist", self.distribution)
        return (isinstance(dist, scipy.stats.rv_discrete)
                or not hasattr(dist, "pdf"))

    def device_spec(self):
        """(kind, [4 params]) for the device kernels: a device family, or
        ABC_PRIOR_HOST with (lo, hi, centre) of the support interval; None
        when the component has no batched form.  That is the case for a
        discrete distribution outside the device families (its pmf vanishes
        between the support's points, where the reference re-draws,
        smc.py:649-662, and the support box cannot) and for anything that is
        not a frozen continuous scipy distribution (e.g. ``rv_discrete(values=
        ...)``, a bare distribution object)."""
        import scipy.stats
        from ._native import PRIOR_KINDS
        fam = self._device_family_params()
        if fam is not None:
            return PRIOR_KINDS[self.name], fam
        if (not isinstance(self.distribution, scipy.stats._distn_infrastructure.rv_frozen)
                or self.is_discrete):
            return None
        lo, hi = (float(v) for v in self.distribution.support())
        if np.isfinite(lo) and np.isfinite(hi):
            c = 0.5 * (lo + hi)
        elif np.isfinite(lo):
            c = lo + 1.0
        elif np.isfinite(hi):
            c = hi - 1.0
        else:
            c = 0.0
        return PRIOR_KINDS["host"], [lo, hi, c, 0.0]

    def _device_family_params(self):
        """[shape..., loc, scale] padded to 4, or None if the kernels have no
        implementation of this distribution (or its parametrisation)."""
        if self.name not in _DEVICE_FAMILIES:
            return None
        shape_names = _DEVICE_FAMILIES[self.name]
        frozen = self.distribution
        pos = list(frozen.args)
        kw = dict(frozen.kwds)
        shapes = pos[:len(shape_names)]
        for nm in shape_names[len(shapes):]:
            if nm not in kw:
                return None
            shapes.append(kw.pop(nm))
        rest = pos[len(shape_names):]
        loc = rest[0] if rest else kw.pop("loc", 0.0)
        scale = rest[1] if len(rest) > 1 else kw.pop("scale", 1.0)
        if kw:
            return None
        vals = [float(v) for v in (*shapes, loc, scale)]
        return vals + [0.0] * (4 - len(vals))

    def host_logpdf(self, x):
        """Vectorised log density (log pmf for discrete families)."""
        x = np.asarray(x, dtype=np.float64)
        if self.is_discrete:
            return self.distribution.logpmf(x)
        return self.distribution.logpdf(x)

    def host_ppf(self, u):
        return np.asarray(self.distribution.ppf(np.asarray(u, np.float64)),
                          dtype=np.float64)


class RVDecorator(RVBase):
    """Wraps a prior component (``self.component``) and forwards to it;
    subclasses override what they change (pyabc random_variables.py:199-260).
    ``repr`` is ``[<decorator_repr()>]<component repr>``.  Decorated
    components have no batched form: priors that use them run the
    per-candidate loop."""

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
        return type(self)(self.component.copy())

    def decorator_repr(self) -> str:
        return "Decorator"

    def __repr__(self):
        return f"[{self.decorator_repr()}]{self.component!r}"


class LowerBoundDecorator(RVDecorator):
    """The component conditioned on X > lower_bound (pyabc
    random_variables.py:263-325): rejection draws (at most MAX_TRIES, then
    None), densities and cdf renormalised by the mass above the bound."""

    MAX_TRIES = 10000

    def __init__(self, component: RVBase, lower_bound: float):
        if component.cdf(lower_bound) == 1:
            raise Exception("LowerBoundDecorator: Conditioning on a set of "
                            "measure zero.")
        super().__init__(component)
        self.lower_bound = lower_bound

    def copy(self):
        return type(self)(self.component.copy(), self.lower_bound)

    def decorator_repr(self):
        return f"Lower: X > {self.lower_bound:2f}"

    def _mass_above(self):
        return 1 - self.component.cdf(self.lower_bound)

    def rvs(self, *args, **kwargs):
        tries = 0
        while tries < self.MAX_TRIES:
            tries += 1
            x = self.component.rvs()
            if not x <= self.lower_bound:     # NaN passes, as in the reference
                return x
        return None

    def pdf(self, x, *args, **kwargs):
        return 0. if x <= self.lower_bound else \
            self.component.pdf(x) / self._mass_above()

    def pmf(self, x, *args, **kwargs):
        return 0. if x <= self.lower_bound else \
            self.component.pmf(x) / self._mass_above()

    def cdf(self, x, *args, **kwargs):
        if x <= self.lower_bound:
            return 0.
        below = self.component.cdf(self.lower_bound)
        return (self.component.cdf(x) - below) / (1 - below)


class Distribution(ParameterStructure):
    """Independent product of RVs over named parameters: a model's prior
    (random_variables.py:328-452)."""

    def __repr__(self):
        return "<Distribution {}>".format(str(list(self.get_parameter_names()))[1:-1])

    @classmethod
    def from_dictionary_of_dictionaries(cls, dict_of_dicts: dict):
        return cls({key: RV.from_dictionary(spec) for key, spec in dict_of_dicts.items()})

    def copy(self):
        return self.__class__(**{key: rv.copy() for key, rv in self.items()})

    def update_random_variables(self, **random_variables):
        self.update(random_variables)

    def get_parameter_names(self) -> list:
        return sorted(self.keys())

    def rvs(self) -> Parameter:
        return Parameter(**{key: rv.rvs() for key, rv in self.items()})

    def pdf(self, x):
        """Product of the component densities (pmf where a component has no
        pdf); the keys of x must be the prior's."""
        if sorted(x.keys()) != sorted(self.keys()):
            raise Exception("Random variable parameter mismatch. Expected: "
                            + str(sorted(self.keys())) + " got " + str(sorted(x.keys())))
        dens = None
        for key, value in x.items():
            rv = self[key]
            try:
                term = rv.pdf(value)
            except AttributeError:
                term = rv.pmf(value)
            dens = term if dens is None else dens * term
        return 1 if dens is None else dens

    # -- batched-sampler description -----------------------------------------
    def device_spec(self):
        """(kinds [d] int32, params [d*4] float64) in sorted-name order, or
        None when a component is not a scipy-backed RV."""
        kinds, params = [], []
        for name in self.get_parameter_names():
            rv = self[name]
            spec = rv.device_spec() if hasattr(rv, "device_spec") else None
            if spec is None:
                return None
            kind, par = spec
            kinds.append(kind)
            params.extend(par)
        return np.asarray(kinds, dtype=np.int32), np.asarray(params, np.float64)

    def host_components(self):
        """[(column, RV)] of the components on the host-scipy leg
        (ABC_PRIOR_HOST), columns in sorted-name order."""
        from ._native import PRIOR_KINDS
        out = []
        for col, name in enumerate(self.get_parameter_names()):
            rv = self[name]
            spec = rv.device_spec() if hasattr(rv, "device_spec") else None
            if spec is not None and spec[0] == PRIOR_KINDS["host"]:
                out.append((col, rv))
        return out


def host_prior_logpdf(theta, host):
    """Sum over the host-leg components of their log densities at the rows
    of the device tensor theta [B, d]; a device tensor [B] (None if there are
    no host components)."""
    if not host:
        return None
    from . import gpu
    cols = [c for c, _ in host]
    vals = theta[:, cols].cpu().numpy()
    s = np.zeros(vals.shape[0])
    with np.errstate(divide="ignore"):
        for q, (_, rv) in enumerate(host):
            s += rv.host_logpdf(vals[:, q])
    return gpu.as_dev(s, device=theta.device)


def host_prior_draw(theta, att, host, seed, generation, idx0):
    """Replace the host-leg columns of a t = 0 prior draw (the device wrote a
    point of the support) by scipy's ppf of the candidate's own uniform from
    its prior stream (slot of the accepted attempt), in place."""
    if not host:
        return theta
    from . import gpu
    for col, rv in host:
        u = gpu.prior_uniforms(att, col, seed, generation, idx0)
        theta[:, col] = gpu.as_dev(rv.host_ppf(u.cpu().numpy()), device=theta.device)
    return theta
