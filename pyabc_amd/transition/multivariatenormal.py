"""MultivariateNormalTransition on the GPU.

Reference: pyabc/transition/multivariatenormal.py:40-113.
  fit  :72-83   weighted covariance (smart_cov) x silverman(ESS, d)^2 x scaling,
                frozen scipy mvn(cov, allow_singular=True)
  rvs  :85-97   ancestor ~ Cat(w), theta = X_j + N(0, Sigma)
  pdf  :99-113  sum_j w_j mvn.pdf(x - X_j)

fit: weighted moments (abc_weighted_moments) and the covariance, its
eigen-whitening with scipy's _PSD cut-off and the sampling factor
(abc_mvn_fit: fp64 Jacobi in one workgroup) all on the device, population
packed once into the MFMA operand image at rank d (abc_mvn_pack_population,
cut eigen-directions contribute zero columns); the fit reads nothing back --
its scalars (rank, log pdet, max w) arrive through a pinned async copy read
at the first density call, which takes the direct kernel if the covariance
turned out singular.  Custom bandwidth selectors, N = 1 and d > 64 run the
eigen-whitening on the host as before.  pdf: the fused
cross-term GEMM + log-sum-exp kernel (abc_mvn_logpdf); singular Sigma (or
rank > 59) goes through the direct fp64 kernel that applies scipy's support
mask.  rvs: the Philox proposal kernel with a flat prior.
"""
import math
from typing import Callable, Union

import numpy as np
import pandas as pd

from .. import gpu
from .. import _native as nat
from .base import Transition
from .exceptions import NotEnoughParticles

BandwidthSelector = Callable[[int, int], float]


def scott_rule_of_thumb(n_samples, dimension):
    """pyabc/transition/multivariatenormal.py:14-24."""
    return n_samples ** (-1. / (dimension + 4))


def silverman_rule_of_thumb(n_samples, dimension):
    """pyabc/transition/multivariatenormal.py:27-37."""
    return (4 / n_samples / (dimension + 2)) ** (1 / (dimension + 4))


# bandwidth rules abc_mvn_fit evaluates on the device (its bw_rule argument)
def _bw_rule(selector):
    return {silverman_rule_of_thumb: 0, scott_rule_of_thumb: 1}.get(selector)


def psd_whitening(cov):
    """scipy.stats._multivariate._PSD semantics (the frozen mvn at
    multivariatenormal.py:83): eigen cut-off 1e6 * eps * max|s|."""
    cov = np.atleast_2d(np.asarray(cov, dtype=np.float64))
    s, u = np.linalg.eigh(cov)
    eps = 1e6 * np.finfo(np.float64).eps * np.max(np.abs(s))
    if np.min(s) < -eps:
        raise ValueError("The input matrix must be symmetric positive "
                         "semidefinite.")
    keep = s > eps
    U = u[:, keep] / np.sqrt(s[keep])
    # sampling factor L L^T = cov, lower triangular (the proposal kernels
    # skip the upper triangle): LQ of the eigen factor B = u sqrt(s), i.e.
    # L = R^T of B^T = Q R, which exists for singular cov as well
    B = u * np.sqrt(np.clip(s, 0, None))[None, :]
    L = np.tril(np.linalg.qr(B.T, mode="r").T)
    return dict(U=U, V=u[:, ~keep], rank=int(keep.sum()),
                log_pdet=float(np.sum(np.log(s[keep]))), tol=1e3 * eps, L=L)


class MultivariateNormalTransition(Transition):
    """Transition via a multivariate Gaussian KDE (GPU).

    Parameters as in the reference (``scaling``, ``bandwidth_selector``), plus
    ``precision`` of the transition-density kernel:

    * "x3" (default): f16 MFMA on three-limb split operands with exact-grid
      f32 accumulation -- f32-grade accuracy (~1e-7 relative) at the highest
      throughput.  Populations outside its range (whitened norm beyond
      ~200 kernel widths, rank > 25) use "f64" automatically.
    * "f64": f64-MFMA cross term (2e-6 relative; the exp2 is f32).
    * "f32": plain f32-MFMA cross term (~3e-5 relative at N=1e5, d=10).
    """
    MFMA_MAX_RANK = 59
    X3_MAX_RANK = 25

    def __init__(self, scaling: float = 1,
                 bandwidth_selector: BandwidthSelector = silverman_rule_of_thumb,
                 precision: str = "x3"):
        self.scaling = scaling
        self.bandwidth_selector = bandwidth_selector
        self.precision = precision
        self._X_arr = None
        self.cov = None
        self._normal = None
        self._fit_future = None

    # the KDE covariance: a host array, fetched from the device fit on use
    @property
    def cov(self):
        if self.__dict__.get("_cov_host") is None and \
                self.__dict__.get("_dev_cov") is not None:
            self._cov_host = self._dev_cov.cpu().numpy()
        return self.__dict__.get("_cov_host")

    @cov.setter
    def cov(self, value):
        self._cov_host = value
        self._dev_cov = None

    # -- fit ---------------------------------------------------------------
    def fit(self, X: pd.DataFrame, w: np.ndarray) -> None:
        if len(X) == 0:
            raise NotEnoughParticles("Fitting not possible.")
        self._X_arr = X.values
        gpu.require_device()
        Xd = gpu.as_dev(self._X_arr)
        wd = gpu.as_dev(np.asarray(w, dtype=np.float64))
        self._fit_device_arrays(Xd, wd)

    def fit_device(self, Xd, wd, columns):
        """Device-resident fit used by the batched sampler: Xd [N, d], wd [N]
        float64 tensors (w normalised), columns = sorted parameter names."""
        if Xd.shape[0] == 0:
            raise NotEnoughParticles("Fitting not possible.")
        self.no_parameters = len(columns) == 0
        self._columns = list(columns)
        self.X = _LazyFrame(Xd, self._columns)
        self.w = _LazyArray(wd)
        self._X_arr = None
        self._fit_device_arrays(Xd, wd)

    def _fit_device_arrays(self, Xd, wd):
        N, d = Xd.shape
        rule = _bw_rule(self.bandwidth_selector)
        if N == 1 or rule is None or d > 64:
            return self._fit_host(Xd, wd)
        # device fit: moments -> cov, eigen-whitening, L (abc_mvn_fit); no
        # host read here (the GPU may still be busy with the generation's
        # densities: the host keeps queueing)
        mom = gpu.weighted_moments_dev(Xd, wd)
        cov, evec, evals, U, L, stats = gpu.mvn_fit(mom, d, self.scaling, rule)
        self._cov_host = None
        self._dev_cov, self._dev_evec, self._dev_evals = cov, evec, evals
        self._dev_stats = stats
        self._fit_future = gpu.HostFuture(stats)
        self._normal = None
        self._dev_X, self._dev_w = Xd, wd
        self._dev_mu = mom[2:2 + d]
        self._dev_L = L
        self._dev_U = U                       # d x d, cut directions zero
        self._dev_V = None
        self._dev_cdf = gpu.inclusive_scan(wd)
        self._dev_guide = gpu.cdf_guide(self._dev_cdf)
        self._prec = {"f32": nat.ABC_PREC_F32, "f64": nat.ABC_PREC_F64,
                      "x3": nat.ABC_PREC_X3}[self.precision]
        # tentatively full rank; _resolve_fit checks it at the first density
        self._rank = d
        self._mfma = d <= self.MFMA_MAX_RANK
        if self._prec == nat.ABC_PREC_X3 and d > self.X3_MAX_RANK:
            self._prec = nat.ABC_PREC_F64
        self._dev_packed = None
        self._x3_range = None
        if self._mfma and self._prec == nat.ABC_PREC_X3:
            # exponents <= 0: the shift -log max w read on the device
            packed, rng = gpu.mvn_pack(Xd, wd, self._dev_mu, U, 0.0, self._prec,
                                       with_range=True, shift_dev=stats[3:4])
            self._dev_packed = packed
            self._x3_range = gpu.HostFuture(rng)
        elif self._mfma:
            self._pack_f64()
        self._dev_flat_kind, self._dev_flat_params = gpu.flat_prior(d, Xd.device)
        self._seed = int(np.random.randint(0, 2 ** 62))
        self._counter = 0
        # the fused rounds' ancestor table, queued with the fit (it would
        # otherwise be built at the next generation's first round, on the
        # critical path between the epsilon read and the first launch)
        self._ancestor_table()

    def _resolve_fit(self):
        """The device fit's scalars (first use after fit_device): rank, the
        normalisation, the shift; a singular covariance switches to the direct
        kernel with scipy's support mask (compact U [d x r] and the null
        space V); a covariance that is not positive semidefinite raises as
        scipy's _PSD does (multivariatenormal.py:83)."""
        fut = self._fit_future
        if fut is None:
            return
        self._fit_future = None
        st = fut.get()
        if st[7] == 0:
            raise ValueError("The input matrix must be symmetric positive "
                             "semidefinite.")
        d = self._dev_X.shape[1]
        rank = int(st[0])
        self._rank = rank
        self._log_norm = -0.5 * (rank * gpu.LOG_2PI + float(st[1]))
        self._support_tol = float(st[2])
        if self._prec == nat.ABC_PREC_X3 and self._mfma:
            self._shift = float(st[3])
        if rank < d or rank == 0:
            self._mfma = False
            self._dev_packed = None
            self._x3_range = None
            self._dev_U = self._dev_U[:, :rank].contiguous() if rank else None
            self._dev_V = self._dev_evec[:, rank:].contiguous()

    def _fit_host(self, Xd, wd):
        """Host eigen-whitening (custom bandwidth selector, N = 1, d > 64)."""
        N, d = Xd.shape
        sw, sw2, mean, cov_b, wmax = gpu.weighted_moments(Xd, wd, with_max=True)
        self._wmax = float(wmax)
        if N == 1:
            sample_cov = np.diag(np.abs(Xd[0].cpu().numpy()))
        else:
            # np.cov(X, aweights=w): sum w (x-m)(x-m)^T / (V1 - V2 / V1)
            sample_cov = cov_b * sw / (sw - sw2 / sw)
        sample_cov = np.atleast_2d(sample_cov)
        eff_sample_size = 1 / sw2
        bw_factor = self.bandwidth_selector(eff_sample_size, d)
        self.cov = sample_cov * bw_factor ** 2 * self.scaling
        self._normal = None
        self._fit_future = None
        self._set_kernel(Xd, wd, mean)

    def _set_kernel(self, Xd, wd, mean):
        N, d = Xd.shape
        psd = psd_whitening(self.cov)
        dev = Xd.device
        self._dev_X = Xd
        self._dev_w = wd
        # one host-to-device copy for all fit constants (mu, U, V, L)
        parts = [np.asarray(mean, dtype=np.float64).ravel(),
                 np.asarray(psd["U"], dtype=np.float64).ravel() if psd["rank"] else np.zeros(0),
                 np.asarray(psd["V"], dtype=np.float64).ravel() if psd["rank"] < d else np.zeros(0),
                 np.asarray(psd["L"], dtype=np.float64).ravel()]
        blob = gpu.as_dev(np.concatenate(parts), device=dev)
        views, o = [], 0
        for a in parts:
            views.append(blob[o:o + a.size])
            o += a.size
        self._dev_mu = views[0]
        self._dev_U = views[1].view(d, psd["rank"]) if psd["rank"] else None
        self._dev_V = views[2].view(d, d - psd["rank"]) if psd["rank"] < d else None
        self._dev_L = views[3].view(d, d)
        self._dev_cdf = gpu.inclusive_scan(wd)
        self._dev_guide = gpu.cdf_guide(self._dev_cdf)
        self._rank = psd["rank"]
        self._support_tol = psd["tol"]
        self._log_norm = -0.5 * (psd["rank"] * gpu.LOG_2PI + psd["log_pdet"])
        self._prec = {"f32": nat.ABC_PREC_F32, "f64": nat.ABC_PREC_F64,
                      "x3": nat.ABC_PREC_X3}[self.precision]
        self._mfma = 1 <= psd["rank"] == d and psd["rank"] <= self.MFMA_MAX_RANK
        if self._prec == nat.ABC_PREC_X3 and psd["rank"] > self.X3_MAX_RANK:
            self._prec = nat.ABC_PREC_F64
        self._dev_packed = None
        self._x3_range = None
        if self._mfma and self._prec == nat.ABC_PREC_X3:
            # exponents <= 0: shift by -log max w (one host read per fit)
            self._shift = -math.log(self._wmax)
            packed, rng = gpu.mvn_pack(Xd, wd, self._dev_mu, self._dev_U,
                                       self._shift, self._prec, with_range=True)
            # range = [max whitened norm, grid exponent E]; E <= 8 keeps the
            # dropped limb products below 2^-19 (see abc_mvn_x3.hip).  Read
            # back at the first density call, not here (no host sync in fit)
            self._dev_packed = packed
            self._x3_range = gpu.HostFuture(rng)
        if self._mfma and self._dev_packed is None:
            self._pack_f64()
        self._dev_flat_kind, self._dev_flat_params = gpu.flat_prior(d, dev)
        self._seed = int(np.random.randint(0, 2 ** 62))
        self._counter = 0

    def _pack_f64(self):
        self._shift = math.log(self._dev_X.shape[0])
        self._dev_packed = gpu.mvn_pack(self._dev_X, self._dev_w, self._dev_mu,
                                        self._dev_U, self._shift, self._prec)

    def _check_x3_range(self):
        self._resolve_fit()
        rng = getattr(self, "_x3_range", None)
        if rng is None:
            return
        self._x3_range = None
        ymax, E = rng.get()
        if E > 8:  # population too spread for the limb grid: fp64 MFMA
            self._prec = nat.ABC_PREC_F64
            self._pack_f64()

    # -- density -----------------------------------------------------------
    def logpdf_device(self, xd, out=None, hint=None):
        """log density at device points xd [M, d] (columns in fit order).
        hint: optional device int64 [M] rows of the fitted population near
        the points (the ancestors propose_device drew them from)."""
        self._check_x3_range()
        if self._mfma:
            return gpu.mvn_logpdf(xd, self._dev_packed, self._dev_X.shape[0],
                                  self._dev_mu, self._dev_U, self._prec,
                                  self._log_norm - self._shift, out=out,
                                  X=self._dev_X, w=self._dev_w,
                                  shift=self._shift,
                                  hint=hint if self._prec == nat.ABC_PREC_X3 else None)
        return gpu.mvn_logpdf_direct(xd, self._dev_X, self._dev_w, self._dev_U,
                                     self._dev_V, self._support_tol,
                                     self._log_norm, out=out)

    def pdf(self, x: Union[pd.Series, pd.DataFrame]) -> Union[float, np.ndarray]:
        x = x[self.X.columns]
        x = np.array(x, dtype=np.float64)
        if len(x.shape) == 1:
            x = x[None, :]
        xd = gpu.as_dev(x, device=self._dev_X.device)
        dens = gpu.torch.exp(self.logpdf_device(xd)).cpu().numpy()
        return dens if dens.size != 1 else float(dens[0])

    # -- sampling ----------------------------------------------------------
    def propose_device(self, B, prior_kind=None, prior_params=None, seed=None,
                       generation=0, idx0=None, max_attempts=1):
        """Batched rvs: B candidates with ancestor ~ Cat(w), theta = X_j + L n,
        re-drawn while the prior density is 0 (when a prior is given)."""
        d = self._dev_X.shape[1]
        if prior_kind is None:
            prior_kind, prior_params = self._dev_flat_kind, self._dev_flat_params
        if idx0 is None:
            idx0 = self._counter
            self._counter += B
        return gpu.propose(self._dev_X, self._dev_cdf, self._dev_L, prior_kind,
                           prior_params, self._seed if seed is None else seed,
                           generation, idx0, B, max_attempts, d,
                           guide=self._dev_guide)

    def proposal_arrays(self):
        """Device arrays of the proposal for the fused candidate kernel
        (abc_candidate_spec): population, weight scan, guide, shared L."""
        return dict(X=self._dev_X, cdf=self._dev_cdf, guide=self._dev_guide,
                    L=self._dev_L, per_particle_L=False,
                    anc_table=self._ancestor_table())

    def rvs(self, size: int = None) -> Union[pd.Series, pd.DataFrame]:
        n = 1 if size is None else size
        theta = self.propose_device(n)[0].cpu().numpy()
        if size is None:
            return pd.Series(theta[0], index=self.X.columns)
        return pd.DataFrame(theta, columns=self.X.columns)

    def rvs_single(self):
        return self.rvs(None)

    # -- reference attribute ----------------------------------------------
    @property
    def normal(self):
        if self._normal is None and self.cov is not None:
            import scipy.stats as st
            self._normal = st.multivariate_normal(cov=self.cov,
                                                  allow_singular=True)
        return self._normal


class _LazyFrame:
    """DataFrame view of a device population, materialised on first use."""

    _index_cache = {}

    def __init__(self, Xd, columns):
        self._Xd = Xd
        key = tuple(columns)
        idx = _LazyFrame._index_cache.get(key)
        if idx is None:
            # one pandas Index per column set (building one costs ~0.1 ms,
            # once per fit otherwise)
            idx = _LazyFrame._index_cache[key] = pd.Index(columns)
        self.columns = idx
        self._df = None

    def _frame(self):
        if self._df is None:
            self._df = pd.DataFrame(self._Xd.cpu().numpy(), columns=self.columns)
        return self._df

    def __len__(self):
        return int(self._Xd.shape[0])

    def __deepcopy__(self, memo):
        # the device population is immutable after fit: share it, and do not
        # materialise the host frame just to copy it (the column Index is
        # immutable too)
        new = _LazyFrame.__new__(_LazyFrame)
        new._Xd, new.columns, new._df = self._Xd, self.columns, self._df
        return new

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        return getattr(self._frame(), item)

    def __getitem__(self, item):
        return self._frame()[item]


class _LazyArray:
    def __init__(self, wd):
        self._wd = wd
        self._a = None

    def _arr(self):
        if self._a is None:
            self._a = self._wd.cpu().numpy()
        return self._a

    def __len__(self):
        return int(self._wd.shape[0])

    def __deepcopy__(self, memo):
        new = _LazyArray(self._wd)
        new._a = self._a
        return new

    @property
    def size(self):
        return int(self._wd.numel())

    @property
    def shape(self):
        return tuple(self._wd.shape)

    def __array__(self, dtype=None, copy=None):
        a = self._arr()
        return a if dtype is None else a.astype(dtype)

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        return getattr(self._arr(), item)

    def __getitem__(self, item):
        return self._arr()[item]
