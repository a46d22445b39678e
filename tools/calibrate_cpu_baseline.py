"""Calibrate bench.py's CPU baseline (the oracle's vectorised numpy port)
against the reference's own samplers on identical work, in THIS container
(the reference does not travel to the GPU box).

    PYTHONPATH=/root/reference:tests/golden PYTHONDONTWRITEBYTECODE=1 \
        OMP_NUM_THREADS=1 python tools/calibrate_cpu_baseline.py

Config: the 10-D conjugate model (c2 shape) at population 1000,
QuantileEpsilon(0.5), PNormDistance, MultivariateNormalTransition, 5
generations (t = 1..3 compared: proposals from the transition and a density
per accepted particle).  For each reference sampler (SingleCoreSampler,
MulticoreEvalParallelSampler(n_procs=8)) the sample_until_n_accepted call of
every generation is timed together with its evaluation count.  The port is
timed on the same work: n_sim candidates (proposal, prior, simulation,
distance; oracle/sampler.py) + n accepted transition densities against the
population (oracle/transition.py), one core.  At the c3 population (N =
1e6, d = 10) the density dominates; one reference MultivariateNormalTransition
.pdf call (smc.py:743 evaluates one per accepted particle) is timed against
the port's density of one point.  Writes profiles/r02_cpu_calibration.json.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import stub_env  # noqa: E402,F401  (before pyabc)
import pyabc  # noqa: E402
from pyabc.epsilon import QuantileEpsilon  # noqa: E402

D, POP, GENS = 10, 1000, 5


def run_reference(sampler):
    nm = [f"p{k}" for k in range(D)]
    keys = [f"y{k}" for k in range(D)]
    np.random.seed(7)

    def model(p):
        return {keys[k]: p[nm[k]] + 0.5 * np.random.randn() for k in range(D)}
    prior = pyabc.Distribution(**{n: pyabc.RV("norm", 0, 1) for n in nm})
    abc = pyabc.ABCSMC(model, prior, pyabc.PNormDistance(), population_size=POP,
                       eps=QuantileEpsilon(alpha=0.5), sampler=sampler)
    calls = []
    orig = sampler.sample_until_n_accepted

    def timed(n, simulate_one, *a, **k):
        t0 = time.perf_counter()
        s = orig(n, simulate_one, *a, **k)
        calls.append(dict(n=int(n), n_sim=int(sampler.nr_evaluations_),
                          seconds=time.perf_counter() - t0))
        return s
    sampler.sample_until_n_accepted = timed
    abc.new("sqlite://", {k: 1.0 for k in keys})
    h = abc.run(max_nr_populations=GENS)
    df, w = h.get_distribution(0, h.max_t - 1)
    return calls, df.values, w


def port_rates(X, w):
    import oracle
    import oracle.sampler as osamp
    cov, wn = oracle.mvn_fit(X, w)
    L = np.linalg.cholesky(cov)
    t0 = time.perf_counter()
    n_c = 0
    while time.perf_counter() - t0 < 3.0:
        th, lp, _, _ = osamp.propose_mvn(X, wn, L, 1, 1, n_c, 4096, ["norm"] * D,
                                         np.tile([0, 1, 0, 0], (D, 1)))
        x = osamp.simulate_linear_gaussian(th, np.arange(D), np.ones(D),
                                           np.full(D, .5), 1, 1, n_c)
        oracle.pnorm(x, np.ones(D))
        n_c += 4096
    t_cand = (time.perf_counter() - t0) / n_c
    t1 = time.perf_counter()
    n_p = 0
    while time.perf_counter() - t1 < 3.0:
        oracle.mvn_logpdf(th[:256], X, wn, cov, block=64)
        n_p += 256
    t_pdf = (time.perf_counter() - t1) / n_p
    return t_cand, t_pdf


def main():
    from pyabc.sampler import MulticoreEvalParallelSampler, SingleCoreSampler
    res = {"config": dict(d=D, population=POP, generations=GENS,
                          model="10-D conjugate Gaussian, PNorm p=2, QuantileEpsilon(0.5), "
                                "MultivariateNormalTransition"),
           "host_cpus": os.cpu_count()}
    single, X, w = run_reference(SingleCoreSampler())
    multi, _, _ = run_reference(MulticoreEvalParallelSampler(n_procs=8))
    t_cand, t_pdf = port_rates(X, w)
    rows = []
    for g, (s, m) in enumerate(zip(single, multi)):
        if g <= 1:
            continue   # calibration sample and t = 0 (prior draws, no density)
        port_s = s["n_sim"] * t_cand + s["n"] * t_pdf
        rows.append(dict(generation=g - 1, n=s["n"], n_sim_single=s["n_sim"],
                         n_sim_multi=m["n_sim"],
                         reference_single_s=s["seconds"], reference_multi8_s=m["seconds"],
                         port_1core_s=port_s,
                         single_over_port=s["seconds"] / port_s,
                         multi8_over_port=m["seconds"] / port_s))
    res["port_seconds_per_candidate"] = t_cand
    res["port_seconds_per_density_N1000"] = t_pdf
    res["generations"] = rows
    # generations t >= 1 (proposal from the transition + density per accepted)
    res["ratio_single_over_port"] = float(np.median([r["single_over_port"] for r in rows]))
    res["ratio_multi8_over_port"] = float(np.median([r["multi8_over_port"] for r in rows]))
    # c3-sized density: the reference's per-particle pdf vs the port's
    import pandas as pd
    import oracle
    from pyabc.transition import MultivariateNormalTransition
    rng = np.random.default_rng(3)
    N = 1_000_000
    Xb = rng.normal(0.8, 0.45, (N, D))
    wb = np.full(N, 1.0 / N)
    cols = [f"p{k}" for k in range(D)]
    tr = MultivariateNormalTransition()
    tr.fit(pd.DataFrame(Xb, columns=cols), wb.copy())
    pt = pd.Series(Xb[0] + 0.1, index=cols)
    tr.pdf(pt)
    t0 = time.perf_counter()
    for _ in range(5):
        tr.pdf(pt)
    t_ref = (time.perf_counter() - t0) / 5
    t0 = time.perf_counter()
    for _ in range(5):
        oracle.mvn_logpdf(Xb[:1] + 0.1, Xb, wb, tr.cov, block=1)
    t_port = (time.perf_counter() - t0) / 5
    res["density_N1e6"] = dict(reference_pdf_call_s=t_ref, port_density_s=t_port,
                               reference_over_port=t_ref / t_port)
    out = os.path.join(ROOT, "profiles", "r02_cpu_calibration.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
