"""LocalTransition on the GPU.

Reference: pyabc/transition/local_transition.py:13-145.
  k        :60-75   max(int(k_fraction * N), MIN_K, d); ``k`` is ignored
                    unless ``k_fraction=None`` (reference behaviour kept)
  fit      :77-96   k+1-NN per particle (cKDTree), local weighted covariance
                    (:125-139), det/inv with the EPS loop (:112-123)
  pdf      :98-110  np.average(exp(-d^T inv_j d / 2) / norm_j, weights=w)
  rvs      :141-145 j ~ Cat(w), theta ~ N(X_j, cov_j)
Device kernels: abc_local_fit (exact radix-select k-NN + moments + small
fp64 linear algebra), abc_local_logpdf, abc_local_propose.  d <= 16 on the
templated kernels; d > 16 on runtime-d kernels (abc_local_wide.hip, slower,
same results; above d = 64 the per-particle matrices live in the workspace
and proposals come from the wide propose kernel); no cap on d, as in the
reference.
"""
import numpy as np
import pandas as pd

from .. import gpu
from .base import Transition
from .exceptions import NotEnoughParticles


class LocalTransition(Transition):
    EPS = 1e-3
    MIN_K = 10

    def __init__(self, k=None, k_fraction=1 / 4, scaling=1):
        if k_fraction is not None:
            self.k_fraction = k_fraction
            self._k = None
        else:
            self.k_fraction = None
            self._k = k
        self.scaling = scaling

    @property
    def k(self):
        if self.k_fraction is not None:
            if self.w is None:
                k_ = 0
            else:
                k_ = int(self.k_fraction * len(self.w))
        else:
            k_ = self._k
        try:
            dim = self.X_arr.shape[1]
        except AttributeError:
            dim = 0
        return max([k_, self.MIN_K, dim])

    def fit(self, X, w):
        if len(X) == 0:
            raise NotEnoughParticles("Fitting not possible.")
        self.X_arr = X.values
        gpu.require_device()
        Xd = gpu.as_dev(self.X_arr)
        wd = gpu.as_dev(np.asarray(w, dtype=np.float64))
        self._fit_device_arrays(Xd, wd)

    def fit_device(self, Xd, wd, columns):
        from .multivariatenormal import _LazyArray, _LazyFrame
        if Xd.shape[0] == 0:
            raise NotEnoughParticles("Fitting not possible.")
        self.no_parameters = len(columns) == 0
        self.X = _LazyFrame(Xd, list(columns))
        self.w = _LazyArray(wd)
        self.X_arr = _LazyArray(Xd)
        self._fit_device_arrays(Xd, wd)

    def _fit_device_arrays(self, Xd, wd):
        N, d = Xd.shape
        covs, inv, dets, chol, lnorm = gpu.local_fit(Xd, wd, self.k,
                                                     self.scaling, self.EPS)
        self._dev_X, self._dev_w = Xd, wd
        self._dev_covs, self._dev_inv, self._dev_dets = covs, inv, dets
        self._dev_chol, self._dev_lnorm = chol, lnorm
        self._dev_cdf = gpu.inclusive_scan(wd)
        self._dev_guide = gpu.cdf_guide(self._dev_cdf)
        self._dev_flat_kind, self._dev_flat_params = gpu.flat_prior(d, Xd.device)
        self._seed = int(np.random.randint(0, 2 ** 62))
        self._counter = 0
        self._host = None

    # reference attributes, materialised on demand
    def _host_arrays(self):
        if self._host is None:
            self._host = dict(covs=self._dev_covs.cpu().numpy(),
                              inv_covs=self._dev_inv.cpu().numpy(),
                              determinants=self._dev_dets.cpu().numpy())
            self._host["normalization"] = np.exp(self._dev_lnorm.cpu().numpy())
        return self._host

    @property
    def covs(self):
        return self._host_arrays()["covs"]

    @property
    def inv_covs(self):
        return self._host_arrays()["inv_covs"]

    @property
    def determinants(self):
        return self._host_arrays()["determinants"]

    @property
    def normalization(self):
        return self._host_arrays()["normalization"]

    def logpdf_device(self, xd, out=None, hint=None):
        return gpu.local_logpdf(xd, self._dev_X, self._dev_w, self._dev_inv,
                                self._dev_lnorm, out=out)

    def pdf(self, x):
        x = x[self.X.columns].values
        single = len(x.shape) == 1
        xa = np.atleast_2d(np.asarray(x, dtype=np.float64))
        xd = gpu.as_dev(xa, device=self._dev_X.device)
        dens = gpu.torch.exp(self.logpdf_device(xd)).cpu().numpy()
        return float(dens[0]) if single else dens

    def propose_device(self, B, prior_kind=None, prior_params=None, seed=None,
                       generation=0, idx0=None, max_attempts=1):
        d = self._dev_X.shape[1]
        if prior_kind is None:
            prior_kind, prior_params = self._dev_flat_kind, self._dev_flat_params
        if idx0 is None:
            idx0 = self._counter
            self._counter += B
        return gpu.propose(self._dev_X, self._dev_cdf, self._dev_chol,
                           prior_kind, prior_params,
                           self._seed if seed is None else seed, generation,
                           idx0, B, max_attempts, d, per_particle_L=True,
                           guide=self._dev_guide)

    def proposal_arrays(self):
        """Device arrays for the fused candidate kernel: per-particle
        Cholesky factors (local_transition.py:141-145)."""
        return dict(X=self._dev_X, cdf=self._dev_cdf, guide=self._dev_guide,
                    L=self._dev_chol, per_particle_L=True,
                    anc_table=self._ancestor_table())

    def rvs_single(self):
        theta = self.propose_device(1)[0].cpu().numpy()[0]
        return pd.Series(theta, index=self.X.columns)

    def rvs(self, size=None):
        if size is None:
            return self.rvs_single()
        theta = self.propose_device(size)[0].cpu().numpy()
        return pd.DataFrame(theta, columns=self.X.columns)
