"""Generate golden vectors by importing the pyABC 0.10.5 reference.

Runs in the BUILD container only (needs /root/reference); the outputs are
small .npz/.json fixtures committed next to this script.  Nothing here is
imported by the product or shipped to the GPU box.

    PYTHONDONTWRITEBYTECODE=1 OMP_NUM_THREADS=1 \
      PYTHONPATH=/root/reference:tests/golden python tests/golden/make_golden.py [--e2e]

Each fixture stores its inputs, seed and the reference outputs.
"""
import json
import os
import sys
import time

import numpy as np
import pandas as pd

import stub_env  # noqa: F401  (must precede pyabc)
import pyabc
from pyabc.transition import MultivariateNormalTransition, LocalTransition
from pyabc.distance import PNormDistance, AdaptivePNormDistance
from pyabc.distance.scale import (standard_deviation,
                                  median_absolute_deviation)
from pyabc.weighted_statistics import weighted_quantile
from pyabc.epsilon import QuantileEpsilon

HERE = os.path.dirname(os.path.abspath(__file__))


def names(d):
    return [f"p{k:02d}" for k in range(d)]


def mvn_case(tag, X, w, x, scaling=1.0):
    d = X.shape[1]
    cols = names(d)
    Xdf = pd.DataFrame(X, columns=cols)
    t = MultivariateNormalTransition(scaling=scaling)
    wref = w.copy()
    t.fit(Xdf, wref)
    xdf = pd.DataFrame(x, columns=cols)
    pdf = np.atleast_1d(t.pdf(xdf))
    np.savez_compressed(os.path.join(HERE, f"mvn_{tag}.npz"), X=X, w=w, x=x,
                        scaling=scaling, cov=t.cov, w_fit=wref, pdf=pdf)
    print("mvn", tag, X.shape, pdf[:3])


def gen_mvn():
    rng = np.random.default_rng(12345)
    for d, N in [(1, 1000), (2, 500), (10, 4096)]:
        X = rng.normal(0.5, 1.0, size=(N, d)) * (1 + np.arange(d))
        w = np.exp(0.5 * rng.standard_normal(N))
        w /= w.sum()
        par = rng.integers(0, N, size=256)
        x = X[par] + 0.3 * rng.standard_normal((256, d)) * (1 + np.arange(d))
        mvn_case(f"d{d}_n{N}", X, w, x)
    # un-normalised weights (fit normalises in place) and scaling != 1
    X = rng.normal(size=(300, 3))
    w = rng.uniform(0.5, 2.0, size=300)
    x = X[:64] + 0.1 * rng.standard_normal((64, 3))
    mvn_case("d3_unnorm_scaled", X, w, x, scaling=0.5)
    # singular: last coordinate constant -> rank 2 of 3
    X = rng.normal(size=(200, 3))
    X[:, 2] = 1.25
    w = np.full(200, 1 / 200)
    x = X[:40] + np.c_[0.2 * rng.standard_normal((40, 2)), np.zeros(40)]
    x[::4, 2] += 0.5     # every 4th candidate leaves the support
    mvn_case("singular", X, w, x)
    # single particle: diag(|x0|) covariance
    X = np.array([[0.7, -1.3]])
    w = np.array([1.0])
    x = X + 0.2 * rng.standard_normal((16, 2))
    mvn_case("n1", X, w, x)


def gen_local():
    rng = np.random.default_rng(99)
    N, d = 400, 5
    comp = rng.integers(0, 2, size=N)
    A = np.tril(rng.normal(size=(d, d))) * 0.3 + np.eye(d) * 0.5
    X = rng.standard_normal((N, d)) @ A.T + comp[:, None] * 2.0
    w = np.exp(0.5 * rng.standard_normal(N))
    w /= w.sum()
    x = X[rng.integers(0, N, 64)] + 0.2 * rng.standard_normal((64, d))
    cols = names(d)
    for tag, kw in [("k50", dict(k=50, k_fraction=None)),
                    ("default", dict())]:
        t = LocalTransition(**kw)
        t.fit(pd.DataFrame(X, columns=cols), w.copy())
        pdf = np.atleast_1d(t.pdf(pd.DataFrame(x, columns=cols)))
        np.savez_compressed(os.path.join(HERE, f"local_{tag}.npz"), X=X, w=w,
                            x=x, k=t.k, covs=t.covs, inv_covs=t.inv_covs,
                            dets=t.determinants,
                            normalization=t.normalization, pdf=pdf)
        print("local", tag, t.k, pdf[:3])


def gen_local_degenerate():
    """LocalTransition on populations whose neighbour weights are degenerate
    (local_transition.py:125-139 -> np.cov(aweights) with 1 - sum a^2 == 0,
    or all neighbour weights 0): one particle carries all the weight of its
    neighbourhood (the others at 1e-20 of it), and a far cluster has zero
    weights.  The reference's covariances are non-finite exactly there; its
    ``while det <= 0`` loop exits on the NaN determinant.  d = 3 (register
    kernels), 20 (runtime-d, LDS) and 80 (runtime-d, workspace matrices)."""
    import warnings
    out = {}
    for d, N, k in [(3, 160, 10), (20, 200, 30), (80, 420, 100)]:
        rng = np.random.default_rng(1000 + d)
        X = rng.standard_normal((N, d))
        w = np.exp(0.3 * rng.standard_normal(N))
        # a cluster far from the rest around particle 0, which dominates its
        # neighbours' neighbourhoods (no other particle's k nearest reach it,
        # so no covariance sits on the det <= 0 knife edge)
        m = k + 6
        X[0] = 20.0
        X[1:m] = X[0] + 0.1 * rng.standard_normal((m - 1, d))
        w[0] = 1.0
        w[1:m] = 1e-20
        # a far cluster of zero-weight particles (> k + 1 of them)
        z0, z1 = N - (k + 8), N
        X[z0:z1] = 40.0 + rng.standard_normal((z1 - z0, d))
        w[z0:z1] = 0.0
        w = w / w.sum()
        t = LocalTransition(k=k, k_fraction=None)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            with np.errstate(all="ignore"):
                t.fit(pd.DataFrame(X, columns=names(d)), w.copy())
        fin = np.isfinite(t.covs).all(axis=(1, 2))
        out[f"X{d}"], out[f"w{d}"], out[f"k{d}"] = X, w, t.k
        out[f"covs{d}"], out[f"dets{d}"] = t.covs, t.determinants
        print("local degenerate d", d, "non-finite covariances:", np.nonzero(~fin)[0])
    np.savez_compressed(os.path.join(HERE, "local_degenerate.npz"), **out)


def gen_distance():
    rng = np.random.default_rng(7)
    out = {}
    for S in (1, 10, 256):
        keys = [f"s{k:03d}" for k in range(S)][::-1]   # non-sorted key order
        x0 = {k: float(v) for k, v in zip(keys, rng.normal(size=S))}
        xs = rng.normal(size=(50, S)) * rng.uniform(0.1, 5, size=S)
        wts = {k: float(v) for k, v in zip(keys, rng.uniform(0.2, 3, size=S))}
        fac = {k: float(v) for k, v in zip(keys, rng.uniform(0.5, 2, size=S))}
        for p in (1, 2, np.inf):
            dist = PNormDistance(p=p, weights=wts, factors=fac)
            dist.initialize(0, lambda: [], x0)
            dv = [dist({k: float(v) for k, v in zip(keys, row)}, x0, 0)
                  for row in xs]
            ptag = "inf" if p == np.inf else str(p)
            out[f"S{S}_p{ptag}"] = dict(
                x=xs, x0=np.array([x0[k] for k in keys]),
                w=np.array([wts[k] for k in keys]),
                f=np.array([fac[k] for k in keys]), p=float(p),
                d=np.array(dv))
    np.savez_compressed(os.path.join(HERE, "pnorm.npz"),
                        **{f"{c}__{f}": v for c, dct in out.items()
                           for f, v in dct.items()})
    print("pnorm", list(out))
    # adaptive weights
    res = {}
    for R in (101, 100):
        S = 12
        keys = [f"y{k}" for k in range(S)]
        data = rng.normal(size=(R, S)) * 10.0 ** rng.uniform(-2, 2, size=S)
        data[:, 3] = 4.2          # zero-scale key -> weight 0
        data[:, 5] = np.round(data[:, 5])  # ties for the MAD
        x0 = {k: 0.0 for k in keys}
        ss = [{k: float(v) for k, v in zip(keys, row)} for row in data]
        for sname, sf in [("std", standard_deviation),
                          ("mad", median_absolute_deviation)]:
            for ratio in (None, 5.0):
                dist = AdaptivePNormDistance(scale_function=sf,
                                             max_weight_ratio=ratio)
                dist.initialize(0, lambda: ss, x0)
                wv = np.array([dist.weights[0][k] for k in keys])
                tag = f"R{R}_{sname}_r{ratio}"
                res[tag + "__data"] = data
                res[tag + "__w"] = wv
                res[tag + "__ratio"] = np.nan if ratio is None else ratio
    np.savez_compressed(os.path.join(HERE, "adaptive.npz"), **res)
    print("adaptive", len(res) // 3)


def gen_quantile():
    rng = np.random.default_rng(3)
    res = {}
    cases = {
        "n10k": (rng.exponential(size=10000), rng.uniform(0, 1, size=10000)),
        "ties": (np.repeat(rng.normal(size=50), 7),
                 rng.uniform(0, 1, size=350)),
        "zerow": (rng.normal(size=500),
                  np.where(rng.uniform(size=500) < 0.3, 0.0,
                           rng.uniform(size=500))),
        "n1": (np.array([3.5]), np.array([1.0])),
    }
    for name, (pts, w) in cases.items():
        w = w / w.sum()
        for a in (0.2, 0.5, 0.9, 1.0):
            q = weighted_quantile(pts, w, alpha=a)
            res[f"{name}__a{a}__q"] = q
        res[f"{name}__points"] = pts
        res[f"{name}__w"] = w
        # QuantileEpsilon update path, weighted and not, multiplier
        for weighted in (True, False):
            eps = QuantileEpsilon(alpha=0.3, quantile_multiplier=1.1,
                                  weighted=weighted)
            df = pd.DataFrame({"distance": pts, "w": w * 2.0})
            eps.initialize(0, lambda: df, None, 10, None)
            res[f"{name}__eps_w{int(weighted)}"] = eps(0)
    np.savez_compressed(os.path.join(HERE, "quantile.npz"), **res)
    print("quantile", len(cases))


def gen_step():
    """Fixed-input generation step: population, weights, candidates, eps ->
    distances, accept mask, importance weights (smc.py:768-811)."""
    rng = np.random.default_rng(2024)
    d, N, M = 4, 800, 512
    cols = names(d)
    X = rng.normal(0.5, 0.5, size=(N, d))
    w = np.exp(0.3 * rng.standard_normal(N))
    w /= w.sum()
    prior = pyabc.Distribution(**{c: pyabc.RV("norm", 0, 1) for c in cols})
    t = MultivariateNormalTransition()
    t.fit(pd.DataFrame(X, columns=cols), w.copy())
    theta = X[rng.integers(0, N, M)] + 0.4 * rng.standard_normal((M, d))
    noise = rng.standard_normal((M, d))
    xsim = theta + 0.5 * noise
    x0 = {f"y{k}": 1.0 for k in range(d)}
    dist = PNormDistance(p=2)
    dist.initialize(1, lambda: [], x0)
    dv = np.array([dist({f"y{k}": row[k] for k in range(d)}, x0, 1)
                   for row in xsim])
    eps = float(np.quantile(dv, 0.4))
    acc = dv <= eps
    prior_pd = np.array([prior.pdf(pyabc.Parameter(
        **{c: v for c, v in zip(cols, row)})) for row in theta])
    trans_pd = np.atleast_1d(t.pdf(pd.DataFrame(theta, columns=cols)))
    weight = np.where(acc, prior_pd / trans_pd, 0.0)
    np.savez_compressed(os.path.join(HERE, "step.npz"), X=X, w=w,
                        theta=theta, xsim=xsim, x0=np.ones(d), eps=eps,
                        d=dv, accept=acc, prior_pd=prior_pd,
                        trans_pd=trans_pd, weight=weight)
    print("step", acc.sum(), "accepted of", M)


def gen_e2e(seeds=(0, 1, 2, 3)):
    """End-to-end reference moments (statistical parity targets)."""
    out = {}
    for s in seeds:
        np.random.seed(s)
        t0 = time.time()

        def model(p):
            return {"y": p["x"] + 0.5 * np.random.randn()}
        abc = pyabc.ABCSMC(model, pyabc.Distribution(x=pyabc.RV("norm", 0, 1)),
                           pyabc.PNormDistance(), population_size=1000,
                           sampler=pyabc.SingleCoreSampler())
        abc.new("sqlite://", {"y": 2.0})
        h = abc.run(max_nr_populations=8)
        df, w = h.get_distribution(0, h.max_t)
        pops = h.get_all_populations()
        out[f"c1_seed{s}"] = dict(
            mean=float((df["x"].values * w).sum()),
            sd=float(np.sqrt((w * (df["x"].values
                                   - (df["x"].values * w).sum()) ** 2).sum())),
            eps=[float(e) for e in pops["epsilon"].values],
            samples=[int(n) for n in pops["samples"].values],
            seconds=time.time() - t0)
        print("e2e c1 seed", s, out[f"c1_seed{s}"])
    with open(os.path.join(HERE, "e2e_reference.json"), "w") as f:
        json.dump(out, f, indent=1)


def gen_e2e10(seeds=(0, 1, 2, 3), pop=1000, gens=5):
    """10-D conjugate model (config 2 shape at N=1000): the reference's ABC
    posterior moments per generation (statistical parity targets)."""
    d = 10
    nm = [f"p{k}" for k in range(d)]
    keys = [f"y{k}" for k in range(d)]
    out = {}
    for s in seeds:
        np.random.seed(s)
        t0 = time.time()

        def model(p):
            return {keys[k]: p[nm[k]] + 0.5 * np.random.randn()
                    for k in range(d)}
        prior = pyabc.Distribution(**{n: pyabc.RV("norm", 0, 1) for n in nm})
        abc = pyabc.ABCSMC(model, prior, pyabc.PNormDistance(),
                           population_size=pop,
                           eps=QuantileEpsilon(alpha=0.5),
                           sampler=pyabc.SingleCoreSampler())
        abc.new("sqlite://", {k: 1.0 for k in keys})
        h = abc.run(max_nr_populations=gens)
        pops = h.get_all_populations()
        means, sds = [], []
        for t in range(h.max_t + 1):
            df, w = h.get_distribution(0, t)
            v = df[nm].values
            m = (v * w[:, None]).sum(0)
            means.append([float(a) for a in m])
            sds.append([float(a) for a in
                        np.sqrt((w[:, None] * (v - m) ** 2).sum(0))])
        out[f"d10_seed{s}"] = dict(
            mean=means, sd=sds,
            eps=[float(e) for e in pops["epsilon"].values],
            samples=[int(n) for n in pops["samples"].values],
            seconds=time.time() - t0)
        print("e2e d10 seed", s, out[f"d10_seed{s}"]["eps"],
              np.mean(means[-1]), flush=True)
    with open(os.path.join(HERE, "e2e_reference_d10.json"), "w") as f:
        json.dump(out, f, indent=1)


def gen_e2e_samples(seeds=(0, 1, 2, 3)):
    """Final-population samples and weights of the reference's c1 run
    (N = 1000, 8 generations, as gen_e2e) and 10-D run (N = 1000, 5
    generations, as gen_e2e10), same seeds: the targets of the weighted
    two-sample KS tests (tests/test_gpu_e2e.py), the reference's own
    criterion being test_nondeterministic/test_abc_smc_algorithm.py:309-394."""
    out = {}
    for s in seeds:
        np.random.seed(s)

        def model(p):
            return {"y": p["x"] + 0.5 * np.random.randn()}
        abc = pyabc.ABCSMC(model, pyabc.Distribution(x=pyabc.RV("norm", 0, 1)),
                           pyabc.PNormDistance(), population_size=1000,
                           sampler=pyabc.SingleCoreSampler())
        abc.new("sqlite://", {"y": 2.0})
        h = abc.run(max_nr_populations=8)
        df, w = h.get_distribution(0, h.max_t)
        out[f"c1_seed{s}__x"] = df["x"].values
        out[f"c1_seed{s}__w"] = w
        out[f"c1_seed{s}__eps"] = h.get_all_populations()["epsilon"].values
        print("samples c1", s, float((df["x"].values * w).sum()), flush=True)
    d = 10
    nm = [f"p{k}" for k in range(d)]
    keys = [f"y{k}" for k in range(d)]
    for s in seeds:
        np.random.seed(s)

        def model(p):
            return {keys[k]: p[nm[k]] + 0.5 * np.random.randn()
                    for k in range(d)}
        prior = pyabc.Distribution(**{n: pyabc.RV("norm", 0, 1) for n in nm})
        abc = pyabc.ABCSMC(model, prior, pyabc.PNormDistance(),
                           population_size=1000, eps=QuantileEpsilon(alpha=0.5),
                           sampler=pyabc.SingleCoreSampler())
        abc.new("sqlite://", {k: 1.0 for k in keys})
        h = abc.run(max_nr_populations=5)
        df, w = h.get_distribution(0, h.max_t)
        out[f"d10_seed{s}__X"] = df[nm].values
        out[f"d10_seed{s}__w"] = w
        out[f"d10_seed{s}__eps"] = h.get_all_populations()["epsilon"].values
        print("samples d10", s, (df[nm].values * w[:, None]).sum(0).mean(), flush=True)
    np.savez_compressed(os.path.join(HERE, "e2e_reference_samples.npz"), **out)


def gen_e2e_large(seeds=(0, 1, 2), pop=10_000, n_procs=8):
    """Final populations of reference runs at N = 1e4 (MulticoreEval on this
    container's cores): the c1 model (1-D, x_0 = 2, 8 generations, as
    gen_e2e) and the 10-D conjugate model (x_0 = 1, QuantileEpsilon(0.5), 4
    generations).  Targets of the N = 1e4 KS / moment tests
    (tests/test_gpu_e2e.py), whose thresholds are the reference's
    test_abc_smc_algorithm.py:354-394.  Samples stored as float32 (the KS
    statistic needs no more), weights as float64."""
    from pyabc.sampler import MulticoreEvalParallelSampler
    out = {}
    d = 10
    nm = [f"p{k}" for k in range(d)]
    keys = [f"y{k}" for k in range(d)]
    for s in seeds:
        np.random.seed(s)
        t0 = time.time()

        def model1(p):
            return {"y": p["x"] + 0.5 * np.random.randn()}
        abc = pyabc.ABCSMC(model1, pyabc.Distribution(x=pyabc.RV("norm", 0, 1)),
                           pyabc.PNormDistance(), population_size=pop,
                           sampler=MulticoreEvalParallelSampler(n_procs=n_procs))
        abc.new("sqlite://", {"y": 2.0})
        h = abc.run(max_nr_populations=8)
        df, w = h.get_distribution(0, h.max_t)
        out[f"c1_seed{s}__x"] = df["x"].values.astype(np.float32)
        out[f"c1_seed{s}__w"] = w
        out[f"c1_seed{s}__eps"] = h.get_all_populations()["epsilon"].values
        print("large c1", s, float((df["x"].values * w).sum()),
              round(time.time() - t0, 1), "s", flush=True)
    for s in seeds:
        np.random.seed(s)
        t0 = time.time()

        def model10(p):
            return {keys[k]: p[nm[k]] + 0.5 * np.random.randn() for k in range(d)}
        prior = pyabc.Distribution(**{n: pyabc.RV("norm", 0, 1) for n in nm})
        abc = pyabc.ABCSMC(model10, prior, pyabc.PNormDistance(),
                           population_size=pop, eps=QuantileEpsilon(alpha=0.5),
                           sampler=MulticoreEvalParallelSampler(n_procs=n_procs))
        abc.new("sqlite://", {k: 1.0 for k in keys})
        h = abc.run(max_nr_populations=4)
        df, w = h.get_distribution(0, h.max_t)
        out[f"d10_seed{s}__X"] = df[nm].values.astype(np.float32)
        out[f"d10_seed{s}__w"] = w
        out[f"d10_seed{s}__eps"] = h.get_all_populations()["epsilon"].values
        print("large d10", s, (df[nm].values * w[:, None]).sum(0).mean(),
              out[f"d10_seed{s}__eps"], round(time.time() - t0, 1), "s", flush=True)
    np.savez_compressed(os.path.join(HERE, "e2e_reference_large.npz"), **out)


def gen_cv(seeds=tuple(range(24))):
    """Bootstrapped KDE CV (pyabc/cv/bootstrap.py:44-110) and the population
    size predicted from it (transition/predict_population_size.py).
    Deterministic part: fixed bootstrap samples (drawn once with the
    reference's own rvs) -> fit + pdf + scipy.stats.variation + weighted
    sum.  Statistical part: the reference's calc_cv / required_nr_samples
    over seeds (their RNG is numpy's, so the GPU matches in distribution)."""
    from pyabc.cv.bootstrap import calc_cv
    import scipy.stats as st
    rng = np.random.default_rng(777)
    N, d = 400, 2
    X = rng.normal(size=(N, d)) @ np.array([[1.0, 0.4], [0.0, 0.7]])
    w = np.exp(0.4 * rng.standard_normal(N))
    w /= w.sum()
    cols = names(d)
    Xdf = pd.DataFrame(X, columns=cols)
    t = MultivariateNormalTransition()
    t.fit(Xdf, w.copy())
    np.random.seed(4242)
    B, n = 6, 300
    samples = np.stack([t.rvs(size=n).values for _ in range(B)])
    dens = []
    for b in range(B):
        tt = MultivariateNormalTransition()
        tt.fit(pd.DataFrame(samples[b], columns=cols), np.ones(n) / n)
        dens.append(tt.pdf(Xdf))
    dens = np.array(dens)
    variation = st.variation(dens, axis=0)
    cv_fixed = float((variation * w).sum())
    stat_n = [100, 400]
    cvs = np.zeros((len(stat_n), len(seeds)))
    for i, nn in enumerate(stat_n):
        for j, s in enumerate(seeds):
            np.random.seed(s)
            cvs[i, j] = calc_cv(nn, np.array([1.0]), 10, [t.w], [t],
                                [t.X])[0]
    n_est = np.zeros(8)
    for j in range(len(n_est)):
        np.random.seed(100 + j)
        tr = MultivariateNormalTransition()
        tr.fit(Xdf, w.copy())
        n_est[j] = tr.required_nr_samples(0.1)
    np.savez_compressed(os.path.join(HERE, "cv.npz"), X=X, w=w,
                        samples=samples, dens=dens, variation=variation,
                        cv_fixed=cv_fixed, stat_n=np.array(stat_n), cvs=cvs,
                        n_est=n_est, n_est_target=0.1)
    print("cv", cv_fixed, cvs.mean(axis=1), cvs.std(axis=1), n_est)


def gen_stochastic():
    """StochasticKernel values, StochasticAcceptor decisions, pdf norms and
    temperature schemes (kernel.py, acceptor.py, pdf_norm.py,
    temperature.py)."""
    from pyabc.distance import (NormalKernel, IndependentNormalKernel,
                                IndependentLaplaceKernel, BinomialKernel,
                                PoissonKernel, NegativeBinomialKernel,
                                SCALE_LIN, SCALE_LOG)
    from pyabc.epsilon.temperature import (
        match_acceptance_rate, EssScheme, AcceptanceRateScheme,
        ExpDecayFixedIterScheme, ExpDecayFixedRatioScheme,
        PolynomialDecayFixedIterScheme, DalyScheme, FrielPettittScheme,
        Temperature)
    from pyabc.acceptor import (StochasticAcceptor, pdf_norm_max_found,
                                pdf_norm_from_kernel, ScaledPDFNorm)
    rng = np.random.default_rng(2024)
    keys = ["s0", "s1", "s2", "s3"]
    B = 64
    out = {}

    def run(kern, X, x0):
        x0d = dict(zip(keys, x0))
        kern.initialize(0, None, x0d)
        v = np.array([kern(dict(zip(keys, row)), x0d) for row in X],
                     dtype=float)
        pm = np.nan if kern.pdf_max is None else float(kern.pdf_max)
        return v, pm

    x0 = rng.normal(size=4)
    X = x0 + 1.5 * rng.normal(size=(B, 4))
    var = np.array([0.5, 1.0, 2.0, 0.7])
    A = rng.normal(size=(4, 4))
    cov = A @ A.T + np.eye(4)
    out.update(cont_x=X, cont_x0=x0, var=var, cov=cov)
    for tag, kern in [
            ("inorm", IndependentNormalKernel(var=var)),
            ("inorm1", IndependentNormalKernel()),
            ("ilap", IndependentLaplaceKernel(scale=var)),
            ("normal", NormalKernel(cov=cov)),
            ("normal_lin", NormalKernel(cov=cov, ret_scale=SCALE_LIN))]:
        out[tag], out[tag + "_pdfmax"] = run(kern, X, x0)
    k0 = rng.integers(0, 12, size=4).astype(float)
    Xc = rng.integers(0, 20, size=(B, 4)) + 0.6 * (rng.random((B, 4)) < 0.3)
    out.update(count_x=Xc, count_x0=k0, p_binom=0.7, p_nbinom=0.4)
    for tag, kern in [
            ("poisson", PoissonKernel()),
            ("poisson_lin", PoissonKernel(ret_scale=SCALE_LIN)),
            ("binom", BinomialKernel(p=0.7)),
            ("binom_lin", BinomialKernel(p=0.7, ret_scale=SCALE_LIN)),
            ("nbinom", NegativeBinomialKernel(p=0.4))]:
        with np.errstate(all="ignore"):
            out[tag], out[tag + "_pdfmax"] = run(kern, Xc, k0)

    # accept decisions: the reference draws u with np.random.uniform
    kern = IndependentNormalKernel(var=var)
    x0d = dict(zip(keys, x0))
    kern.initialize(0, None, x0d)
    for tag, scale in (("acc_log", SCALE_LOG), ("acc_lin", SCALE_LIN)):
        acc = StochasticAcceptor()
        acc.pdf_norms = {0: -3.0 if scale == SCALE_LOG else 0.01}
        kk = kern if scale == SCALE_LOG else NormalKernel(
            cov=np.diag(var), ret_scale=SCALE_LIN)
        kk.initialize(0, None, x0d)
        us, ds, accs, ws = [], [], [], []
        for i in range(B):
            np.random.seed(1000 + i)
            us.append(np.random.uniform(low=0, high=1))
            np.random.seed(1000 + i)
            r = acc(kk, lambda t: 2.5, dict(zip(keys, X[i])), x0d, 0, None)
            ds.append(r.distance)
            accs.append(r.accept)
            ws.append(r.weight)
        out[tag + "_u"] = np.array(us)
        out[tag + "_dens"] = np.array(ds)
        out[tag + "_accept"] = np.array(accs)
        out[tag + "_weight"] = np.array(ws)
        out[tag + "_pdf_norm"] = acc.pdf_norms[0]

    # match_acceptance_rate: log and linear scale, and the corner cases
    R = 500
    pds = rng.normal(-3.0, 2.0, R)
    wts = np.exp(0.5 * rng.standard_normal(R))
    out.update(mar_pds=pds, mar_w=wts)
    out["mar_log"] = match_acceptance_rate(wts / wts.sum(), pds, pds.max(),
                                           SCALE_LOG, 0.3)
    out["mar_log_low"] = match_acceptance_rate(wts / wts.sum(), pds,
                                               pds.max() + 1.0, SCALE_LOG, 0.05)
    out["mar_log_one"] = match_acceptance_rate(wts / wts.sum(), pds, pds.min(),
                                               SCALE_LOG, 0.3)
    lpds = np.exp(pds)
    out["mar_lin"] = match_acceptance_rate(wts / wts.sum(), lpds, lpds.max(),
                                           SCALE_LIN, 0.3)
    # EssScheme
    N = 400
    ep = rng.normal(-2.0, 1.5, N)
    ew = np.exp(0.3 * rng.standard_normal(N))
    out.update(ess_pds=ep, ess_w=ew)

    def wd():
        return pd.DataFrame({"distance": ep, "w": ew})
    for tag, prev in (("ess_prev", 7.53), ("ess_none", None)):
        out[tag] = float(np.ravel(EssScheme()(
            t=1, get_weighted_distances=wd, get_all_records=None,
            max_nr_populations=5, pdf_norm=ep.max(), kernel_scale=SCALE_LOG,
            prev_temperature=prev, acceptance_rate=0.3))[0])
    # deterministic schemes at a few (t, prev_temperature, acceptance rate)
    sch = []
    for t, prev, ar in ((1, 7.53, 0.4), (2, 3.0, 0.6), (3, 12.0, 5e-5)):
        args = dict(t=t, get_weighted_distances=wd, get_all_records=None,
                    max_nr_populations=5, pdf_norm=0.0,
                    kernel_scale=SCALE_LOG, prev_temperature=prev,
                    acceptance_rate=ar)
        row = [ExpDecayFixedIterScheme()(**args),
               ExpDecayFixedRatioScheme()(**args),
               PolynomialDecayFixedIterScheme()(**args),
               DalyScheme()(**args), FrielPettittScheme()(**args)]
        sch.append([t, prev, ar] + row)
    out["schemes"] = np.array(sch)
    # Temperature orchestration with list records
    recs = [dict(distance=pds[i], transition_pd_prev=1.0,
                 transition_pd=wts[i], accepted=bool(i % 3 == 0))
            for i in range(R)]
    temp = Temperature()
    cfg = dict(pdf_norm=pds.max(), kernel_scale=SCALE_LOG)
    temp.initialize(0, wd, lambda: recs, 4, cfg)
    for t in (1, 2, 3):
        temp.update(t, wd, lambda: recs, 0.2, cfg)
    out["temp_seq"] = np.array([temp(t) for t in range(4)])
    # pdf norms
    pn = dict(kernel_val=42, prev_pdf_norm=3.5, get_weighted_distances=wd,
              prev_temp=10.3, acceptance_rate=0.05)
    out["pdfnorm"] = np.array([pdf_norm_max_found(**pn),
                               pdf_norm_from_kernel(**pn),
                               ScaledPDFNorm()(**pn)])
    np.savez_compressed(os.path.join(HERE, "stochastic.npz"), **out)
    print("stochastic", out["mar_log"], out["mar_lin"], out["ess_prev"],
          out["temp_seq"], out["pdfnorm"])


def gen_history():
    """A small run stored by pyABC's own History (read back by our
    read_run), and a file written by our bulk writer read by pyABC's
    History (history.py readers over db_model.py)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from pyabc_amd.storage.sqlite_store import SQLiteStore
    ref_db = os.path.join(HERE, "ref_history.db")
    if os.path.exists(ref_db):
        os.remove(ref_db)
    np.random.seed(0)

    def model(p):
        return {"y": p["x"] + 0.5 * np.random.randn(), "z": 2 * p["x"]}
    prior = pyabc.Distribution(x=pyabc.RV("norm", 0, 1))
    abc = pyabc.ABCSMC(model, prior, pyabc.PNormDistance(), population_size=40,
                       sampler=pyabc.sampler.SingleCoreSampler())
    abc.new("sqlite:///" + ref_db, {"y": 2.0, "z": 4.0},
            gt_par={"x": 1.5})
    h = abc.run(max_nr_populations=2)
    out = {}
    for t in range(h.max_t + 1):
        df, w = h.get_distribution(0, t)
        out[f"theta_{t}"] = df["x"].values
        out[f"w_{t}"] = w
        wd = h.get_weighted_distances(t)
        out[f"dist_{t}"] = wd["distance"].values
    pops = h.get_all_populations()
    out["pops"] = pops[["t", "samples", "epsilon", "particles"]].values.astype(float)
    # our writer -> pyABC's reader
    ours_db = "/tmp/ours_history_golden.db"
    if os.path.exists(ours_db):
        os.remove(ours_db)
    rng = np.random.default_rng(3)
    n, d, S = 50, 3, 2
    th = rng.normal(size=(n, d))
    w = rng.random(n)
    w /= w.sum()
    dist = rng.random(n)
    ss = rng.normal(size=(n, S))
    st = SQLiteStore(ours_db)
    abc_id = st.new_run({}, "{}", "{}", "{}")
    st.store_pre_population(abc_id, 0, {"s0": 1.0, "s1": 2.0}, {"a": 0.5},
                            ["m0"])
    st.submit(abc_id, 0, 0.7, 123, lambda: dict(
        theta=th, w=w, distance=dist, sum_stats=ss, names=["a", "b", "c"],
        keys=["s0", "s1"]), "m0")
    st.update_nr_samples(abc_id, -1, 77)
    st.done(abc_id)
    st.close()
    hr = pyabc.History("sqlite:///" + ours_db)
    hr.id = abc_id
    df, wr = hr.get_distribution(0, 0)
    ws, sss = hr.get_weighted_sum_stats(0)
    out.update(ours_theta=th, ours_w=w, ours_dist=dist, ours_ss=ss,
               ours_ref_theta=df[["a", "b", "c"]].values, ours_ref_w=wr,
               ours_ref_ss=np.array([[s["s0"], s["s1"]] for s in sss]),
               ours_ref_dist=hr.get_weighted_distances(0)["distance"].values,
               ours_ref_x0=np.array([hr.observed_sum_stat()["s0"],
                                     hr.observed_sum_stat()["s1"]]),
               ours_ref_pops=hr.get_all_populations()[
                   ["t", "samples", "epsilon", "particles"]].values.astype(float),
               ours_ref_nsim=hr.total_nr_simulations)
    np.savez_compressed(os.path.join(HERE, "history.npz"), **out)
    print("history", out["pops"], out["ours_ref_pops"])


if __name__ == "__main__":
    if "--history" in sys.argv:
        gen_history()
        sys.exit(0)
    if "--stochastic" in sys.argv:
        gen_stochastic()
        sys.exit(0)
    if "--cv" in sys.argv:
        gen_cv()
        sys.exit(0)
    if "--e2e10" in sys.argv:
        gen_e2e10()
        sys.exit(0)
    if "--e2e-large" in sys.argv:
        gen_e2e_large()
        sys.exit(0)
    if "--local-degenerate" in sys.argv:
        gen_local_degenerate()
        sys.exit(0)
    if "--e2e-samples" in sys.argv:
        gen_e2e_samples()
        sys.exit(0)
    gen_mvn()
    gen_local()
    gen_distance()
    gen_quantile()
    gen_step()
    if "--e2e" in sys.argv:
        gen_e2e()
