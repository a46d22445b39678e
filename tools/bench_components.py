"""Per-component measurements of the §8 rows beside the transition density.

    python tools/bench_components.py [--only c4,quantile,c5,sampler] [--reps 5]

One JSON line per kernel: the BASELINE.json config it is measured on, the
average time per call (torch.cuda.Event on the launch stream = torch's
current stream, which libabcgpu launches on), the algorithmic bytes or FLOP
per call and the fraction of the HBM (8 TB/s) or fp64 VALU
peak.  Inputs are synthetic, generated on the device or from seeded numpy.

  c4        AdaptivePNormDistance on 256-dim summary stats, pop 2e5:
            pnorm over R candidates (R = 6.7e5 recorded at acceptance 0.3),
            column std and MAD over the recorded [R x 256] matrix
  quantile  QuantileEpsilon weighted quantile at N = 1e6 (c3) and 1e5 (c2)
  c5        LocalTransition d = 5, N = 1e5: k-NN covariance fit (k = 50 and
            the default k = N/4 = 25000), density of 1e5 candidates
  sampler   propose + simulate + pnorm + accept at the c3 batch (4.6e6)
  cv        AdaptivePopulationSize.update on the c2 population (wall time)
  e2e       whole-run generation times of c1, c4 (MAD / std), c5
  history   History file store: a c2 population written in pyABC's schema
  stochastic StochasticAcceptor stack at the c3 batch (4.6e6 candidates):
            IndependentNormalKernel values (S = 10), tempered accept step,
            one AcceptanceRateScheme objective over 4.6e6 records, the full
            bisection; plus wall time per generation of a c2-size
            (N = 1e5, d = 10) stochastic ABCSMC run
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM_PEAK = 8.0e12          # B/s (MI355X_MICROARCH.md)
F64_VALU_PEAK = 78.6e12    # FLOP/s fp64 vector = fp64 matrix on MI355X (spec)


def timed(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def emit(component, config, ms, bytes_=None, flop=None, extra=None):
    rec = {"component": component, "config": config, "ms": round(ms, 4)}
    if bytes_ is not None:
        bw = bytes_ / (ms * 1e-3)
        rec.update(algorithmic_bytes=bytes_, achieved_GBps=round(bw / 1e9, 1),
                   bound="hbm", frac=round(bw / HBM_PEAK, 4))
    if flop is not None:
        fl = flop / (ms * 1e-3)
        rec.update(algorithmic_flop=flop, achieved_TFLOPs=round(fl / 1e12, 3),
                   bound="fp64 valu", frac=round(fl / F64_VALU_PEAK, 4))
    if extra:
        rec.update(extra)
    print(json.dumps(rec), flush=True)


def c4(reps):
    import torch
    from pyabc_amd import gpu
    rng = np.random.default_rng(1234)
    S, R = 256, 670_000
    a = rng.uniform(0.5, 2.0, S)
    sig = 10.0 ** rng.uniform(-2, 2, S)
    theta = torch.randn(R, 4, dtype=torch.float64, device="cuda")
    src = torch.as_tensor(np.arange(S) % 4, device="cuda")
    X = theta[:, src] * torch.as_tensor(a, device="cuda") + \
        torch.randn(R, S, dtype=torch.float64, device="cuda") * torch.as_tensor(sig, device="cuda")
    X = X.contiguous()
    x0 = gpu.as_dev(a * 0.5)
    wf = gpu.as_dev(1.0 / sig)
    out = torch.empty(R, dtype=torch.float64, device="cuda")
    ms = timed(lambda: gpu.pnorm(X, x0, wf, 2.0, out=out), reps)
    emit("pnorm (AdaptivePNormDistance.__call__)", "c4: S=256, 6.7e5 candidates",
         ms, bytes_=R * (8 * S + 8))
    ms = timed(lambda: gpu.column_std(X), reps)
    emit("column std (scale update)", "c4: [6.7e5 x 256] recorded", ms,
         bytes_=R * S * 8 * 2, extra={"note": "two-pass: mean, then squares"})
    ms = timed(lambda: gpu.column_mad(X), max(1, reps // 2))
    emit("column MAD (scale update)", "c4: [6.7e5 x 256] recorded", ms,
         bytes_=R * S * 8 * 2,
         extra={"note": "algorithmic = median pass + deviation pass, 8 B each"})


def quantile(reps):
    import torch
    from pyabc_amd import gpu
    for N, tag in ((1_000_000, "c3"), (100_000, "c2")):
        d = torch.rand(N, dtype=torch.float64, device="cuda") * 4 + 1
        w = torch.rand(N, dtype=torch.float64, device="cuda")
        ms = timed(lambda: gpu.weighted_quantile(d, w, 0.5), reps)
        emit("weighted quantile (QuantileEpsilon)", f"{tag}: N={N}", ms,
             bytes_=N * 16)


def c5(reps):
    import torch
    import pandas as pd
    from pyabc_amd.transition import LocalTransition
    rng = np.random.default_rng(99)
    N, d = 100_000, 5
    comp = rng.integers(0, 2, N)
    A = rng.standard_normal((d, d)) * 0.3 + np.eye(d)
    X = rng.standard_normal((N, d)) @ A.T + np.where(comp[:, None] == 1, 2.0, -1.0)
    w = np.exp(0.5 * rng.standard_normal(N))
    w /= w.sum()
    cols = [f"p{k}" for k in range(d)]
    for kw, tag in ((dict(k=50, k_fraction=None), "k=50"), (dict(), "k=N/4=25000")):
        t = LocalTransition(**kw)
        t.fit(pd.DataFrame(X, columns=cols), w.copy())
        Xd, wd = t._dev_X, t._dev_w
        ms = timed(lambda: t._fit_device_arrays(Xd, wd), 1)
        pair_flop = 3 * d + 2 * (2 + d + d * (d + 1) // 2)
        emit("LocalTransition.fit (k-NN covariances)", f"c5: N=1e5, d=5, {tag}", ms,
             flop=N * N * pair_flop,
             extra={"note": "per (n, j) pair: 3d distance + masked moments"})
    x = t.propose_device(N)[0]
    ms = timed(lambda: t.logpdf_device(x), reps)
    # the pair term as a GEMM over K0 = d(d+1)/2 + d + 1 quadratic features
    # (abc_local.hip), priced against the fp64 MFMA peak
    k0 = d * (d + 1) // 2 + d + 1
    fl = N * N * 2 * k0
    emit("LocalTransition.pdf", "c5: 1e5 candidates x 1e5 particles", ms,
         extra=dict(algorithmic_flop=fl, flop_per_pair=2 * k0,
                    achieved_TFLOPs=round(fl / (ms * 1e-3) / 1e12, 3),
                    bound="fp64 mfma", peak_TFLOPs=78.6,
                    frac=round(fl / (ms * 1e-3) / F64_VALU_PEAK, 4),
                    note="quadratic-feature GEMM on v_mfma_f64_16x16x4_f64 + "
                         "exp2/sum; per-pair VALU form is d^2+2d+4 FLOP"))


def sampler(reps):
    import torch
    import pandas as pd
    from pyabc_amd import gpu
    from pyabc_amd.transition import MultivariateNormalTransition
    rng = np.random.default_rng(5)
    N, d, B = 1_000_000, 10, 4_600_000
    X = 0.8 + np.sqrt(0.2) * rng.standard_normal((N, d))
    w = np.exp(0.5 * rng.standard_normal(N))
    w /= w.sum()
    t = MultivariateNormalTransition()
    t.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(d)]), w.copy())
    kind = torch.zeros(d, dtype=torch.int32, device="cuda")
    params = gpu.as_dev(np.tile([0.0, 1.0, 0.0, 0.0], d))
    res = {}

    def prop():
        res["p"] = t.propose_device(B, kind, params, seed=3, generation=2,
                                    idx0=0, max_attempts=100)
    ms = timed(prop, reps)
    emit("propose (MVN rvs + prior)", "c3 batch: 4.6e6 candidates", ms,
         bytes_=B * (8 * d + 8 + 8 + 4 + 8 * d),
         extra={"note": "theta/lp/ancestor/attempts written + ancestor row read"})
    th = res["p"][0]
    src = torch.arange(d, dtype=torch.int32, device="cuda")
    one, half = gpu.as_dev(np.ones(d)), gpu.as_dev(np.full(d, 0.5))
    xs = {}
    ms = timed(lambda: xs.__setitem__("x", gpu.simulate_linear_gaussian(
        th, src, one, half, 3, 2, 0)), reps)
    emit("simulate (vectorised linear Gaussian)", "c3 batch", ms,
         bytes_=B * 16 * d)
    x = xs["x"]
    dd = torch.empty(B, dtype=torch.float64, device="cuda")
    ms = timed(lambda: gpu.pnorm(x, one, one, 2.0, out=dd), reps)
    emit("pnorm (PNormDistance, S=10)", "c3 batch", ms, bytes_=B * (8 * d + 8))
    eps = float(dd.median())
    ms = timed(lambda: gpu.accept_compact(dd, eps), reps)
    emit("accept + compaction", "c3 batch", ms, bytes_=B * 8 * 2)


def cv(reps):
    """AdaptivePopulationSize.update at c2 size (N = 1e5, d = 10): the
    bootstrapped KDE CV on range(N/3, 2N, N/10) x 10 bootstraps, each an
    rvs + fit + N x n transition-density launch."""
    import time
    import pandas as pd
    import torch
    import pyabc_amd as pa
    from pyabc_amd import gpu
    N, d = 100_000, 10
    rng = np.random.default_rng(8)
    X = rng.normal(0.8, 0.45, size=(N, d))
    w = np.exp(0.3 * rng.standard_normal(N))
    w /= w.sum()
    tr = pa.MultivariateNormalTransition()
    tr.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(d)]), w)
    ns = list(range(N // 3, 2 * N, N // 10))
    pairs = 10 * N * sum(ns)
    for r in range(max(1, reps // 2) + 1):
        ps = pa.AdaptivePopulationSize(N, mean_cv=0.02, n_bootstrap=10,
                                       max_population_size=10 ** 6)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ps.update([tr], np.array([1.0]), t=1)
        torch.cuda.synchronize()
        sec = time.perf_counter() - t0
    # reference: 7.8e6 transition-density pair-evals/s per core (BASELINE.md,
    # multivariatenormal.py:99-113 at N = 1e6)
    emit("AdaptivePopulationSize.update (bootstrapped KDE CV)",
         "c2 population: N=1e5, d=10, 17 sizes x 10 bootstraps",
         sec * 1e3, extra=dict(pair_evals=pairs,
                               pair_evals_per_s=round(pairs / sec, 1),
                               new_size=ps.nr_particles,
                               reference_core_s_extrapolated=round(pairs / 7.8e6)))


def stochastic(reps):
    import time
    import torch
    import pyabc_amd as pa
    from pyabc_amd import gpu
    from pyabc_amd.epsilon.temperature import match_acceptance_rate
    B, S = 4_600_000, 10
    x = torch.randn(B, S, dtype=torch.float64, device="cuda")
    keys = [f"y{k}" for k in range(S)]
    x0 = {k: 0.5 for k in keys}
    kern = pa.IndependentNormalKernel(var=np.full(S, 0.3))
    kern.initialize(0, None, x0)
    x0v = gpu.as_dev(np.full(S, 0.5))
    out = torch.empty(B, dtype=torch.float64, device="cuda")
    ms = timed(lambda: kern.device_call(x, x0v, 0, keys, out=out), reps)
    emit("kernel values (IndependentNormalKernel, S=10)", "c3 batch: 4.6e6",
         ms, bytes_=B * (8 * S + 8))
    res = {}
    ms = timed(lambda: res.__setitem__("a", gpu.stochastic_accept(
        out, float(out.max()), 3.0, True, True, 7, 2, 0)), reps)
    emit("stochastic accept (u, acc, weight)", "c3 batch", ms,
         bytes_=B * (8 + 16))
    lr = torch.randn(B, dtype=torch.float64, device="cuda").mul_(0.3)
    lp = torch.zeros(B, dtype=torch.float64, device="cuda")
    c = float(out.max())
    ms = timed(lambda: gpu.temper_sums(out, lr, c, True, gpu.TEMPER_ACCEPTANCE,
                                       0.3, 0.0, lr_sub=lp), reps)
    emit("AcceptanceRateScheme objective (one bisection step)",
         "c3 records: 4.6e6", ms, bytes_=B * 24,
         extra={"note": "includes the 16-byte host read of the two sums"})
    t0 = time.perf_counter()
    T = match_acceptance_rate(out, lr, c, pa.distance.SCALE_LOG, 0.3, lp)
    emit("match_acceptance_rate (full bisection)", "c3 records: 4.6e6",
         (time.perf_counter() - t0) * 1e3, extra={"temperature": T})
    # end to end: c2-size noise-model ABC (y = theta, IndependentNormal
    # noise), StochasticAcceptor + Temperature(), batched sampler
    d = 10
    names = [f"p{k}" for k in range(d)]
    model = pa.LinearGaussianModel(names, keys, src=list(range(d)),
                                   sigma=[0.0] * d)
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    abc = pa.ABCSMC(model, prior, pa.IndependentNormalKernel(var=np.full(S, 0.25)),
                    population_size=100_000, eps=pa.Temperature(),
                    acceptor=pa.StochasticAcceptor(),
                    sampler=pa.BatchedGPUSampler(seed=5))
    abc.new("sqlite://", {k: 1.0 for k in keys})
    abc.run(max_nr_populations=6)
    log = abc.generation_log
    emit("stochastic ABCSMC generation (c2 size)",
         "N=1e5, d=S=10, IndependentNormalKernel(var .25), Temperature()",
         1e3 * float(np.median([g["seconds"] for g in log[1:]])),
         extra={"temperatures": [round(abc.eps(g["t"]), 3) for g in log],
                "n_sim": [g["n_sim"] for g in log]})


def history(reps):
    """History file store: one c2 population (1e5 particles, d = S = 10)
    through libabcstore into pyABC's SQLite schema (host code; the
    reference's SQLAlchemy writer takes 2.9 ms per particle)."""
    import tempfile
    import time
    from pyabc_amd.storage.sqlite_store import SQLiteStore
    n, d, S = 100_000, 10, 10
    rng = np.random.default_rng(0)
    h = dict(theta=rng.normal(size=(n, d)), w=np.full(n, 1 / n),
             distance=rng.random(n), sum_stats=rng.normal(size=(n, S)),
             names=[f"p{k}" for k in range(d)], keys=[f"y{k}" for k in range(S)])
    path = os.path.join(tempfile.mkdtemp(), "w.db")
    st = SQLiteStore(path)
    i = st.new_run({}, "", "", "")
    t0 = time.perf_counter()
    st.submit(i, 0, 1.0, n, lambda: h, "m")
    st.flush()
    sec = time.perf_counter() - t0
    st.close()
    emit("History population write (libabcstore, pyABC schema)",
         "c2 population: 1e5 particles, d=S=10 (22 rows per particle)",
         sec * 1e3, extra=dict(us_per_particle=round(sec / n * 1e6, 2),
                               reference_ms_per_particle=2.9,
                               file_MB=round(os.path.getsize(path) / 1e6, 1)))


def e2e(reps):
    """Whole runs of the BASELINE.json configs on one GPU (wall time per
    generation from ABCSMC.generation_log; History in HBM):
      c1  d=1, N=1000, 8 generations, MVN + PNorm + MedianEpsilon
      c4  S=256 heterogeneous-scale model, N=2e5, AdaptivePNormDistance with
          the MAD scale (and the default std scale), record_rejected on
      c5  LocalTransition (k=50) as the transition of a 5-D run, N=1e5"""
    import time
    import torch
    import pyabc_amd as pa
    # c1 (after one untimed run: the first kernel launches of a process load
    # libabcgpu's code objects, a one-time cost of ~0.1 s)
    w = pa.ABCSMC(pa.LinearGaussianModel(["x"], ["y"], src=[0], sigma=[0.5]),
                  pa.Distribution(x=pa.RV("norm", 0, 1)), pa.PNormDistance(),
                  population_size=1000, sampler=pa.BatchedGPUSampler(seed=9))
    w.new("sqlite://", {"y": 2.0})
    w.run(max_nr_populations=2)
    np.random.seed(0)
    abc = pa.ABCSMC(pa.LinearGaussianModel(["x"], ["y"], src=[0], sigma=[0.5]),
                    pa.Distribution(x=pa.RV("norm", 0, 1)), pa.PNormDistance(),
                    population_size=1000, sampler=pa.BatchedGPUSampler(seed=1))
    abc.new("sqlite://", {"y": 2.0})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    abc.run(max_nr_populations=8)
    torch.cuda.synchronize()
    sec = time.perf_counter() - t0
    emit("c1 end to end (8 generations)", "d=1, N=1000, MVN + PNorm + MedianEpsilon",
         sec * 1e3, extra=dict(accepted_per_s=round(8000 / sec, 1),
                               reference_accepted_per_s={"SingleCore": 229,
                                                         "MulticoreEval(8)": 912}))
    # c4
    rng = np.random.default_rng(1234)
    S = 256
    a = rng.uniform(0.5, 2.0, S)
    sig = 10.0 ** rng.uniform(-2, 2, S)
    names = [f"th{k}" for k in range(4)]
    keys = [f"s{k:03d}" for k in range(S)]
    model = pa.LinearGaussianModel(names, keys, src=np.arange(S) % 4, a=a,
                                   sigma=sig)
    x0 = {k: float(a[i] * 0.5) for i, k in enumerate(keys)}
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    for tag, scale in (("MAD", pa.distance.median_absolute_deviation),
                       ("std", None)):
        dist = (pa.AdaptivePNormDistance(scale_function=scale) if scale
                else pa.AdaptivePNormDistance())
        abc = pa.ABCSMC(model, prior, dist, population_size=200_000,
                        sampler=pa.BatchedGPUSampler(seed=2))
        abc.new("sqlite://", x0)
        abc.run(max_nr_populations=5)
        log = abc.generation_log
        emit(f"c4 generation (AdaptivePNormDistance, {tag} scale)",
             "S=256, N=2e5, record_rejected, MedianEpsilon",
             1e3 * float(np.median([g["seconds"] for g in log[1:]])),
             extra=dict(n_sim=[g["n_sim"] for g in log],
                        accepted_per_s=round(2e5 / float(np.median(
                            [g["seconds"] for g in log[1:]])), 1)))
    # c5: LocalTransition in a 5-D run
    d = 5
    names = [f"p{k}" for k in range(d)]
    keys = [f"y{k}" for k in range(d)]
    abc = pa.ABCSMC(pa.LinearGaussianModel(names, keys, src=list(range(d)),
                                           sigma=[0.5] * d),
                    pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names}),
                    pa.PNormDistance(), population_size=100_000,
                    transitions=pa.LocalTransition(k=50, k_fraction=None),
                    eps=pa.QuantileEpsilon(alpha=0.5),
                    sampler=pa.BatchedGPUSampler(seed=3))
    abc.new("sqlite://", {k: 1.0 for k in keys})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    abc.run(max_nr_populations=4)
    torch.cuda.synchronize()
    sec = time.perf_counter() - t0
    log = abc.generation_log
    emit("c5 generation (LocalTransition k=50)", "d=5, N=1e5, PNorm, QuantileEpsilon(.5)",
         1e3 * float(np.median([g["seconds"] for g in log[1:]])),
         extra=dict(n_sim=[g["n_sim"] for g in log],
                    run_total_ms=round(sec * 1e3, 1),
                    note="run_total: calibration + 4 generations + 4 fits, synchronized"))
    # the fit alone on this run's last population
    cols = abc.history.get_population_device()
    tr = pa.LocalTransition(k=50, k_fraction=None)
    tr.fit_device(cols.theta, cols.weights, cols.param_names)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.fit_device(cols.theta, cols.weights, cols.param_names)
    torch.cuda.synchronize()
    emit("c5 LocalTransition fit on the run's population", "N=1e5, d=5, k=50",
         (time.perf_counter() - t0) * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c4,quantile,c5,sampler,cv")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    for name in a.only.split(","):
        globals()[name](a.reps)


if __name__ == "__main__":
    main()
