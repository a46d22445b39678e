"""Stochastic acceptance stack: noise-model kernels (distance/kernel.py),
StochasticAcceptor + pdf norms (acceptor/acceptor.py:309-476,
acceptor/pdf_norm.py), temperatures (epsilon/temperature.py).

Pinning: tests/golden/stochastic.npz, produced by importing pyABC 0.10.5
(tests/golden/make_golden.py --stochastic).  CPU tests check the oracle and
the host-side scheme logic against it; GPU tests run the device kernels
through the C ABI.  Tolerances: kernel values 1e-12 relative (1e-10 for the
lgamma-based count models and the linear scale), accept masks exact,
temperatures 1e-9 relative (bisection to xtol 2e-12 on log beta), EssScheme
1e-5 (scipy's L-BFGS-B stopping rule on a rounded objective).
"""
import json
import os
import tempfile

import numpy as np
import pandas as pd
import pytest

import oracle.stochastic as ost
from conftest import GOLDEN

G = np.load(os.path.join(GOLDEN, "stochastic.npz"))
KEYS = ["s0", "s1", "s2", "s3"]


def close(a, b, rtol):
    a, b = np.asarray(a, float), np.asarray(b, float)
    fin = np.isfinite(b)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    assert np.array_equal(a[~fin & ~np.isnan(b)], b[~fin & ~np.isnan(b)])
    np.testing.assert_allclose(a[fin], b[fin], rtol=rtol, atol=1e-300)


# ---- CPU: oracle vs the reference -------------------------------------------

CONT = [("inorm", "independent_normal", "var", None, True),
        ("ilap", "independent_laplace", "var", None, True),
        ("normal", "normal", None, "cov", True),
        ("normal_lin", "normal", None, "cov", False)]
COUNT = [("poisson", "poisson", None, True), ("poisson_lin", "poisson", None, False),
         ("binom", "binomial", "p_binom", True),
         ("binom_lin", "binomial", "p_binom", False),
         ("nbinom", "negative_binomial", "p_nbinom", True)]


@pytest.mark.parametrize("tag,kind,par,cov,log", CONT)
def test_oracle_continuous_kernels(tag, kind, par, cov, log):
    v = ost.kernel_values(kind, G["cont_x"], G["cont_x0"],
                          par=None if par is None else G[par],
                          cov=None if cov is None else G[cov], ret_log=log)
    close(v, G[tag], 1e-12)
    close(ost.kernel_values("independent_normal", G["cont_x"], G["cont_x0"],
                            par=1.0), G["inorm1"], 1e-12)


@pytest.mark.parametrize("tag,kind,par,log", COUNT)
def test_oracle_count_kernels(tag, kind, par, log):
    with np.errstate(all="ignore"):
        v = ost.kernel_values(kind, G["count_x"], G["count_x0"],
                              par=None if par is None else float(G[par]),
                              ret_log=log)
    close(v, G[tag], 1e-12)


@pytest.mark.parametrize("tag,log", [("acc_log", True), ("acc_lin", False)])
def test_oracle_accept_step(tag, log):
    acc, w = ost.stochastic_accept(G[tag + "_dens"], float(G[tag + "_pdf_norm"]),
                                   2.5, log, True, G[tag + "_u"])
    assert np.array_equal(acc, G[tag + "_accept"])
    close(w, G[tag + "_weight"], 1e-13)


def test_oracle_match_acceptance_rate_and_ess():
    pds, w = G["mar_pds"], G["mar_w"]
    close(ost.match_acceptance_rate(w, pds, pds.max(), True, 0.3), G["mar_log"], 1e-12)
    close(ost.match_acceptance_rate(w, pds, pds.max() + 1, True, .05),
          G["mar_log_low"], 1e-12)
    assert ost.match_acceptance_rate(w, pds, pds.min(), True, .3) == G["mar_log_one"] == 1.0
    lp = np.exp(pds)
    close(ost.match_acceptance_rate(w, lp, lp.max(), False, .3), G["mar_lin"], 1e-10)
    ep, ew = G["ess_pds"], G["ess_w"]
    close(ost.ess_temperature(ep, ew, ep.max(), True, 7.53), G["ess_prev"], 1e-9)
    close(ost.ess_temperature(ep, ew, ep.max(), True, None), G["ess_none"], 1e-9)


# ---- CPU: host-side scheme logic of pyabc_amd ---------------------------------

def _wd():
    return pd.DataFrame({"distance": G["ess_pds"], "w": G["ess_w"]})


def test_deterministic_schemes_match_reference():
    import pyabc_amd as pa
    for t, prev, ar, *ref in G["schemes"]:
        args = dict(t=int(t), get_weighted_distances=_wd, get_all_records=None,
                    max_nr_populations=5, pdf_norm=0.0,
                    kernel_scale=pa.distance.SCALE_LOG,
                    prev_temperature=prev, acceptance_rate=ar)
        got = [pa.ExpDecayFixedIterScheme()(**args),
               pa.ExpDecayFixedRatioScheme()(**args),
               pa.PolynomialDecayFixedIterScheme()(**args),
               pa.DalyScheme()(**args), pa.FrielPettittScheme()(**args)]
        np.testing.assert_allclose(got, ref, rtol=1e-14)


def test_scheme_none_and_errors():
    """test_epsilon.py:150-163 behaviour."""
    import pyabc_amd as pa
    args = dict(t=0, get_weighted_distances=_wd, get_all_records=None,
                max_nr_populations=3, pdf_norm=10,
                kernel_scale=pa.distance.SCALE_LOG, prev_temperature=None,
                acceptance_rate=0.4)
    for s in (pa.ExpDecayFixedIterScheme(), pa.ExpDecayFixedRatioScheme(),
              pa.PolynomialDecayFixedIterScheme(), pa.DalyScheme(),
              pa.FrielPettittScheme()):
        assert s(**args) == np.inf
    args["prev_temperature"] = 7.53
    assert 1.0 < pa.ExpDecayFixedIterScheme()(**args) < np.inf
    args["t"] = 2
    assert pa.ExpDecayFixedIterScheme()(**args) == 1.0
    args["max_nr_populations"] = np.inf
    with pytest.raises(ValueError):
        pa.ExpDecayFixedIterScheme()(**args)


def test_temperature_orchestration_and_log():
    """test_epsilon.py:56-100 with a fixed initial temperature and a
    deterministic scheme (no device reductions)."""
    import pyabc_amd as pa
    eps = pa.ListTemperature(values=[10, 5, 1.5])
    assert eps(0) == 10 and eps(2) == 1.5
    log_file = tempfile.mkstemp(suffix=".json")[1]
    cfg = {"pdf_norm": 5, "kernel_scale": pa.distance.SCALE_LOG}
    eps = pa.Temperature(schemes=[pa.ExpDecayFixedIterScheme()],
                         initial_temperature=42, log_file=log_file)
    eps.initialize(0, _wd, None, 3, cfg)
    assert eps(0) == 42
    eps.update(1, _wd, None, 0.4, cfg)
    assert 1 < eps(1) < 42
    eps.update(2, _wd, None, 0.2, cfg)
    assert eps(2) == 1
    prop = pa.storage.load_dict_from_json(log_file)
    assert prop[0][0] == 42 and len(prop[1]) == 1 and len(prop[2]) == 1
    os.remove(log_file)


def test_pdf_norm_methods():
    """test_acceptor.py:131-160 (host DataFrame path)."""
    import pyabc_amd as pa

    def wd():
        return pd.DataFrame({'distance': [1, 2, 3, 4], 'w': [2, 1, 1, 0]})
    args = dict(kernel_val=42, prev_pdf_norm=3.5, get_weighted_distances=wd,
                prev_temp=10.3, acceptance_rate=0.3)
    assert pa.pdf_norm_max_found(**args) == 4
    assert pa.pdf_norm_from_kernel(**args) == 42
    assert pa.ScaledPDFNorm()(**args) == 4
    args["prev_pdf_norm"] = 4.5
    args["acceptance_rate"] = 0.05
    assert pa.pdf_norm_max_found(**args) == 4.5
    assert pa.ScaledPDFNorm()(**args) == 4.5 - np.log(10) * 0.5 * 10.3
    # the reference's golden values (prev 3.5, rate 0.05)
    args = dict(kernel_val=42, prev_pdf_norm=3.5, get_weighted_distances=_wd,
                prev_temp=10.3, acceptance_rate=0.05)
    got = [pa.pdf_norm_max_found(**args), pa.pdf_norm_from_kernel(**args),
           pa.ScaledPDFNorm()(**args)]
    np.testing.assert_allclose(got, G["pdfnorm"], rtol=1e-15)


def test_kernel_keys_and_errors():
    import pyabc_amd as pa
    with pytest.raises(ValueError):
        pa.BinomialKernel(p=1.5)
    with pytest.raises(ValueError):
        pa.NormalKernel(ret_scale="bad")
    k = pa.IndependentNormalKernel(var=lambda par: 1.0)
    k.initialize(0, None, {"b": 1.0, "a": 2.0})
    assert k.keys == ["a", "b"] and k.pdf_max is None
    assert not k.batched_capable


# ---- GPU: device kernels through the C ABI ----------------------------------

gpu_mark = pytest.mark.gpu


def _kernel(tag):
    import pyabc_amd as pa
    SL = pa.distance.SCALE_LIN
    return {"inorm": pa.IndependentNormalKernel(var=G["var"]),
            "inorm1": pa.IndependentNormalKernel(),
            "ilap": pa.IndependentLaplaceKernel(scale=G["var"]),
            "normal": pa.NormalKernel(cov=G["cov"]),
            "normal_lin": pa.NormalKernel(cov=G["cov"], ret_scale=SL),
            "poisson": pa.PoissonKernel(),
            "poisson_lin": pa.PoissonKernel(ret_scale=SL),
            "binom": pa.BinomialKernel(p=0.7),
            "binom_lin": pa.BinomialKernel(p=0.7, ret_scale=SL),
            "nbinom": pa.NegativeBinomialKernel(p=0.4)}[tag]


ALL = ["inorm", "inorm1", "ilap", "normal", "normal_lin", "poisson",
       "poisson_lin", "binom", "binom_lin", "nbinom"]


@gpu_mark
@pytest.mark.parametrize("tag", ALL)
def test_kernel_device_call_golden(tag):
    """Batched values with the sum-stat columns in a different (x_0) order
    plus an unused column; per-particle __call__ on a few rows."""
    from pyabc_amd import gpu
    cont = tag in ("inorm", "inorm1", "ilap", "normal", "normal_lin")
    X, x0 = (G["cont_x"], G["cont_x0"]) if cont else (G["count_x"], G["count_x0"])
    kern = _kernel(tag)
    order = ["s2", "extra", "s0", "s3", "s1"]
    x0d = dict(zip(KEYS, x0))
    kern.initialize(0, None, x0d)
    if not np.isnan(G[tag + "_pdfmax"]):
        np.testing.assert_allclose(kern.pdf_max, G[tag + "_pdfmax"], rtol=1e-10)
    full = {k: X[:, i] for i, k in enumerate(KEYS)}
    full["extra"] = np.full(X.shape[0], 123.0)
    xmat = np.stack([full[k] for k in order], axis=1)
    x0vec = np.array([x0d.get(k, 7.0) for k in order])
    dev = gpu.require_device()
    got = kern.device_call(gpu.as_dev(xmat), gpu.as_dev(x0vec), 0, order)
    rtol = 1e-12 if tag in ("inorm", "inorm1", "ilap", "normal") else 1e-10
    close(got.cpu().numpy(), G[tag], rtol)
    for i in (0, 5, 17):
        v = kern(dict(zip(KEYS, X[i])), x0d)
        close([v], [G[tag][i]], rtol)
    assert dev is not None


@gpu_mark
def test_kernel_callable_and_array_keys():
    """kernel.py callables of the parameters and array-valued keys
    (test_distance_function.py:258-330)."""
    import pyabc_amd as pa
    x0 = {'y0': np.array([1, 2]), 'y1': 2.5}
    x = {'y0': np.array([0, 0]), 'y1': 7}
    exp = -0.5 * (3 * np.log(2 * np.pi) + np.log(1) + np.log(2) + np.log(3)
                  + 1 ** 2 / 1 + 2 ** 2 / 2 + 4.5 ** 2 / 3)
    k = pa.IndependentNormalKernel(lambda p: np.array([p['th0'], p['th1'], 3]))
    k.initialize(0, None, x0)
    assert np.isclose(k(x, x0, par={'th0': 1, 'th1': 2}), exp)
    k = pa.NormalKernel(cov=np.diag([1, 2, 3]))
    k.initialize(0, None, x0)
    assert np.isclose(k(x, x0), exp)
    k = pa.IndependentLaplaceKernel()
    k.initialize(0, None, x0)
    assert np.isclose(k(x, x0), -(3 * np.log(2) + 1 + 2 + 4.5))
    x0 = {'y0': np.array([4, 5]), 'y1': 7}
    x = {'y0': np.array([7, 7]), 'y1': 7}
    from scipy import stats
    k = pa.BinomialKernel(p=lambda par: np.array([0.9, 0.8, 0.7]))
    k.initialize(0, None, x0)
    assert np.isclose(k(x, x0), np.sum(stats.binom.logpmf(
        k=[4, 5, 7], n=[7, 7, 7], p=[0.9, 0.8, 0.7])))
    k = pa.BinomialKernel(p=0.9)
    k.initialize(0, None, x0)
    assert k(x, {'y0': np.array([4, 10]), 'y1': 7}) == -np.inf


@gpu_mark
@pytest.mark.parametrize("log", [True, False])
def test_stochastic_accept_replay(log):
    """abc_stochastic_accept vs the oracle replay of the same Philox
    uniforms: exact accept masks, 1e-13 weights; then compaction."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(5)
    B = 20000
    dens = rng.normal(-4, 2, B) if log else np.exp(rng.normal(-4, 2, B))
    dens[:3] = [np.nan, -np.inf if log else 0.0, 5.0 if log else 1e3]
    c = -3.0 if log else np.exp(-3.0)
    seed, gen, idx0 = 987654321, 3, 4096
    key, accw = gpu.stochastic_accept(gpu.as_dev(dens), c, 2.5, log, True,
                                      seed, gen, idx0)
    u = ost.accept_uniform(seed, gen, idx0, B)
    acc, w = ost.stochastic_accept(dens, c, 2.5, log, True, u)
    assert np.array_equal(key.cpu().numpy() <= 0, acc)
    close(accw.cpu().numpy()[acc], w[acc], 1e-13)
    idx, cnt = gpu.accept_compact(key, 0.0)
    n = int(cnt.item())
    assert np.array_equal(idx[:n].cpu().numpy(), np.nonzero(acc)[0])


@gpu_mark
def test_match_acceptance_rate_device():
    import pyabc_amd as pa
    from pyabc_amd import gpu
    from pyabc_amd.epsilon.temperature import match_acceptance_rate
    pds, w = G["mar_pds"], G["mar_w"]
    SL, SG = pa.distance.SCALE_LIN, pa.distance.SCALE_LOG
    # log-form device records: weights exp(log t_pd - log t_pd_prev)
    d, lw = gpu.as_dev(pds), gpu.as_dev(np.log(w) + 3.0)
    lprev = gpu.as_dev(np.full(w.size, 3.0))
    close(match_acceptance_rate(d, lw, pds.max(), SG, 0.3, lprev), G["mar_log"], 1e-9)
    close(match_acceptance_rate(d, lw, pds.max() + 1, SG, .05, lprev),
          G["mar_log_low"], 1e-9)
    assert match_acceptance_rate(d, lw, pds.min(), SG, .3, lprev) == 1.0
    lp = np.exp(pds)
    close(match_acceptance_rate(gpu.as_dev(lp), gpu.as_dev(w), lp.max(), SL,
                                0.3, None, log_form=False), G["mar_lin"], 1e-9)
    # through the scheme with the reference's list-of-dicts records
    recs = [dict(distance=pds[i], transition_pd_prev=2.0,
                 transition_pd=2.0 * w[i], accepted=True) for i in range(w.size)]
    t = pa.AcceptanceRateScheme()(
        t=1, get_weighted_distances=None, get_all_records=lambda: recs,
        max_nr_populations=5, pdf_norm=pds.max(), kernel_scale=SG,
        prev_temperature=None, acceptance_rate=0.3)
    close(t, G["mar_log"], 1e-9)
    recd = pa.epsilon.DeviceRecords(d, lprev, lw, gpu.as_dev(np.zeros(w.size)))
    t = pa.AcceptanceRateScheme()(
        t=1, get_weighted_distances=None, get_all_records=lambda: recd,
        max_nr_populations=5, pdf_norm=pds.max(), kernel_scale=SG,
        prev_temperature=None, acceptance_rate=0.3)
    close(t, G["mar_log"], 1e-9)


@gpu_mark
def test_ess_scheme_and_temperature_sequence():
    import pyabc_amd as pa
    SG = pa.distance.SCALE_LOG
    ep = G["ess_pds"]
    for tag, prev in (("ess_prev", 7.53), ("ess_none", None)):
        got = pa.EssScheme()(t=1, get_weighted_distances=_wd,
                             get_all_records=None, max_nr_populations=5,
                             pdf_norm=ep.max(), kernel_scale=SG,
                             prev_temperature=prev, acceptance_rate=0.3)
        close(np.ravel(got)[0], G[tag], 1e-5)
    pds, w = G["mar_pds"], G["mar_w"]
    recs = [dict(distance=pds[i], transition_pd_prev=1.0, transition_pd=w[i],
                 accepted=bool(i % 3 == 0)) for i in range(pds.size)]
    temp = pa.Temperature()
    cfg = dict(pdf_norm=pds.max(), kernel_scale=SG)
    temp.initialize(0, _wd, lambda: recs, 4, cfg)
    for t in (1, 2, 3):
        temp.update(t, _wd, lambda: recs, 0.2, cfg)
    close([temp(t) for t in range(4)], G["temp_seq"], 1e-9)


def _stochastic_abc(pop, seed, sampler=None, pdf_norm=None, max_pop=4):
    import pyabc_amd as pa
    np.random.seed(seed)
    model = pa.LinearGaussianModel(["x"], ["y"], src=[0], sigma=[0.0])
    prior = pa.Distribution(x=pa.RV("norm", 0, 1))
    kern = pa.IndependentNormalKernel(var=[0.25])
    acc = pa.StochasticAcceptor(pdf_norm_method=pdf_norm)
    abc = pa.ABCSMC(model, prior, kern, population_size=pop,
                    sampler=sampler or pa.BatchedGPUSampler(seed=77 + seed),
                    eps=pa.Temperature(), acceptor=acc)
    abc.new("sqlite://", {"y": 2.0})
    return abc


@gpu_mark
def test_stochastic_abc_exact_posterior_batched():
    """Noise-model ABC is exact at T = 1 (Wilkinson 2013): y = x, x_0 = 2,
    noise var 0.25, prior N(0, 1) -> posterior N(1.6, 0.2).  Runs every
    device piece: kernel, stochastic accept, acceptance weights, device
    records with both transition densities, AcceptanceRateScheme bisection."""
    import pyabc_amd as pa
    from test_gpu_e2e import posterior_check
    abc = _stochastic_abc(4000, 0)
    h = abc.run(max_nr_populations=4)
    assert abc.minimum_epsilon == 1.0
    temps = abc.eps.temperatures
    assert temps[max(temps)] == 1.0
    assert all(temps[t] >= temps[t + 1] for t in range(max(temps)))
    posterior_check(h, 1.6, np.sqrt(0.2), cdf_tol=0.06, mean_tol=0.04,
                    sd_tol=0.04)
    assert isinstance(abc.sampler, pa.BatchedGPUSampler)


@gpu_mark
def test_stochastic_abc_gave_up_proposals():
    """A narrow bounded prior with max_attempts = 2: some proposals exhaust
    their prior re-draws.  Under a StochasticAcceptor the "distance" is a
    density, so such a proposal must get the zero-probability density (never
    accepted, acceptance weight 0) and stay out of the temperature records --
    not +inf, which would accept it with an infinite weight and NaN the
    population's normalisation."""
    import pyabc_amd as pa
    from pyabc_amd import gpu
    np.random.seed(3)
    model = pa.LinearGaussianModel(["x"], ["y"], src=[0], sigma=[0.0])
    prior = pa.Distribution(x=pa.RV("uniform", 1.2, 0.3))
    sampler = pa.BatchedGPUSampler(seed=91, max_attempts=2)
    # a wide perturbation kernel: many proposals leave the narrow support
    abc = pa.ABCSMC(model, prior, pa.IndependentNormalKernel(var=[0.25]),
                    population_size=3000, sampler=sampler,
                    transitions=pa.MultivariateNormalTransition(scaling=50),
                    eps=pa.Temperature(initial_temperature=8.0),
                    acceptor=pa.StochasticAcceptor())
    abc.new("sqlite://", {"y": 2.0})
    gave_up = []
    orig = gpu.mask_gave_up

    def spy(dist, att, max_attempts, value=float("nan")):
        gave_up.append(int((att > max_attempts).sum()))
        return orig(dist, att, max_attempts, value)
    gpu.mask_gave_up = spy
    try:
        h = abc.run(max_nr_populations=4)
    finally:
        gpu.mask_gave_up = orig
    assert sum(gave_up) > 0
    for t in range(h.max_t + 1):
        df, w = h.get_distribution(0, t)
        assert np.isfinite(w).all() and (w > 0).all()
        np.testing.assert_allclose(w.sum(), 1.0, rtol=1e-12)
        x = df["x"].to_numpy()
        assert ((x >= 1.2) & (x <= 1.5)).all()
    assert h.max_t >= 1
    temps = abc.eps.temperatures
    assert all(np.isfinite(v) and v >= 1.0 for v in temps.values())


@gpu_mark
def test_prior_logpdf_wide_vs_scipy():
    """abc_prior_logpdf above d = 64 (the StochasticAcceptor's temperature
    records need the prior density of every recorded theta): d = 80, mixed
    families, points inside and outside the supports, vs scipy (1e-12)."""
    from scipy import stats
    from pyabc_amd import gpu
    d, B = 80, 777
    rng = np.random.default_rng(17)
    kinds = np.array([0, 1, 2, 3] * (d // 4), dtype=np.int32)
    params = np.zeros((d, 4))
    params[:, 0] = rng.uniform(-1, 1, d)
    params[:, 1] = rng.uniform(0.5, 2, d)
    theta = rng.normal(0, 2, (B, d))
    inside = kinds == 1      # uniform [loc, loc + scale]: mostly inside
    theta[:, inside] = params[inside, 0] + params[inside, 1] * rng.uniform(0, 1, (B, inside.sum()))
    expo = kinds == 2        # expon: support [loc, inf)
    theta[:, expo] = params[expo, 0] + rng.exponential(1.0, (B, expo.sum()))
    theta[:10, np.nonzero(inside)[0][0]] = params[inside, 0][0] - 1.0   # outside
    theta[10:20, np.nonzero(expo)[0][0]] = params[expo, 0][0] - 0.5     # outside
    lp = gpu.prior_logpdf(gpu.as_dev(theta), gpu.as_dev(kinds, dtype=gpu.torch.int32),
                          gpu.as_dev(params.ravel())).cpu().numpy()
    fam = {0: stats.norm, 1: stats.uniform, 2: stats.expon, 3: stats.laplace}
    ref = sum(fam[int(kinds[k])].logpdf(theta[:, k], params[k, 0], params[k, 1])
              for k in range(d))
    fin = np.isfinite(ref)
    assert 0 < fin.sum() < B
    np.testing.assert_array_equal(np.isfinite(lp), fin)
    np.testing.assert_allclose(lp[fin], ref[fin], rtol=1e-12)


@gpu_mark
def test_stochastic_abc_wide_records():
    """d = 80 under a StochasticAcceptor and a Temperature: generation 1
    weighs the records of generation 0 with the prior density on the device
    (above d = 64) and both transition densities; the populations are finite
    and normalised and the temperatures stay >= 1."""
    import pyabc_amd as pa
    d = 80
    names = [f"p{i:02d}" for i in range(d)]
    keys = [f"y{i:02d}" for i in range(d)]
    model = pa.LinearGaussianModel(names, keys, src=list(range(d)), sigma=[0.0] * d)
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    abc = pa.ABCSMC(model, prior, pa.IndependentNormalKernel(var=[4.0] * d),
                    population_size=400, sampler=pa.BatchedGPUSampler(seed=23),
                    eps=pa.Temperature(), acceptor=pa.StochasticAcceptor())
    abc.new("sqlite://", {k: 0.3 for k in keys})
    h = abc.run(max_nr_populations=3)
    assert h.max_t >= 1
    for t in range(h.max_t + 1):
        df, w = h.get_distribution(0, t)
        assert df.shape[1] == d and np.isfinite(df.to_numpy()).all()
        assert np.isfinite(w).all() and (w >= 0).all()
        np.testing.assert_allclose(w.sum(), 1.0, rtol=1e-12)
    temps = abc.eps.temperatures
    assert all(np.isfinite(v) and v >= 1.0 for v in temps.values())


@gpu_mark
def test_stochastic_abc_per_particle_and_pdf_norms():
    """test_acceptor.py:72-128 on the per-particle path (array-valued sum
    stats, user model) for every pdf normalisation."""
    import pyabc_amd as pa

    def model(par):
        return {'s0': par['p0'] + np.array([0.3, 0.7])}
    x_0 = {'s0': np.array([0.4, -0.6])}
    for pdf_norm in [pa.pdf_norm_max_found, pa.pdf_norm_from_kernel,
                     pa.ScaledPDFNorm()]:
        pnorm_file = tempfile.mkstemp(suffix=".json")[1]
        acceptor = pa.StochasticAcceptor(pdf_norm_method=pdf_norm,
                                         log_file=pnorm_file)
        abc = pa.ABCSMC(model, pa.Distribution(p0=pa.RV('uniform', -1, 2)),
                        pa.IndependentNormalKernel(var=np.array([1, 1])),
                        eps=pa.Temperature(), acceptor=acceptor,
                        population_size=20)
        abc.new(pa.create_sqlite_db_id(), x_0)
        h = abc.run(max_nr_populations=3)
        pnorms = pa.storage.load_dict_from_json(pnorm_file)
        assert len(pnorms) == h.max_t + 2
        assert abc.minimum_epsilon == 1.0
        os.remove(pnorm_file)
