"""Fused candidate rounds (abc_candidates_round / abc_candidates_regen).

The fused kernel runs the per-candidate closure (pyabc/smc.py:588-724:
proposal + prior re-draw, LinearGaussianModel, PNormDistance, d <= eps) in
one launch and keeps one accept bit per candidate; accepted rows are
regenerated.  Parity bar: the accept set, ancestors, theta, prior
log-density, sum stats and distances are BIT-IDENTICAL to the staged kernels
(abc_propose -> abc_simulate_linear_gaussian -> abc_pnorm ->
abc_accept_compact) on the same inputs (distances of rows wider than 32
statistics to 1e-13: abc_pnorm sums those in another order), in plain and
early-reject (filter)
modes, for the MVN, LocalTransition and prior (t = 0) proposals; and the
accept set equals the numpy oracle's replay of the same Philox streams away
from |d - eps| < 1e-12 (oracle/sampler.py).
"""
import numpy as np
import pytest

import oracle
import oracle.sampler as osamp

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    from pyabc_amd import gpu
    return gpu.require_device()


def T(a, dtype=None):
    from pyabc_amd import gpu
    return gpu.as_dev(a, dtype=dtype)


KIND = {"norm": 0, "uniform": 1, "expon": 2, "laplace": 3, "lognorm": 4,
        "gamma": 5, "beta": 6}


def _case(d, S, N=3000, mode="mvn", seed=0, kinds=None, params=None, p=2.0,
          src=None, a=None, sigma=None, x0=1.0):
    """Device arrays of one generation's closure + the staged reference."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(seed)
    X = rng.normal(0.5, 0.8, (N, d))
    w = np.exp(0.5 * rng.standard_normal(N))
    w /= w.sum()
    kinds = kinds or ["norm"] * d
    params = (np.tile([0.0, 1.0, 0, 0], (d, 1)) if params is None
              else np.asarray(params, float))
    src = np.arange(S) % d if src is None else np.asarray(src)
    a = np.ones(S) if a is None else np.asarray(a, float)
    sigma = np.full(S, 0.5) if sigma is None else np.asarray(sigma, float)
    wf = np.ones(S)
    c = dict(d=d, S=S, kind=T([KIND[k] for k in kinds], torch.int32),
             params=T(params.ravel()), src=T(src, torch.int32), a=T(a),
             sigma=T(sigma), x0=T(np.full(S, x0)), wf=T(wf), p=p,
             host=dict(X=X, w=w, kinds=kinds, params=params, src=src, a=a,
                       sigma=sigma, x0=np.full(S, x0), wf=wf))
    if mode == "prior":
        c.update(X=None, cdf=None, guide=None, L=None, ppl=False)
        return c
    Xd, wd = T(X), T(w)
    cdf = gpu.inclusive_scan(wd)
    c.update(X=Xd, cdf=cdf, guide=gpu.cdf_guide(cdf))
    if mode == "mvn":
        Lh = np.linalg.cholesky(0.2 * np.eye(d) + 0.05)
        c.update(L=T(Lh), ppl=False)
        c["host"]["L"] = Lh
    else:   # per-particle factors (LocalTransition)
        A = rng.normal(0, 0.3, (N, d, d))
        cov = A @ np.transpose(A, (0, 2, 1)) + 0.05 * np.eye(d)
        Lh = np.linalg.cholesky(cov)
        c.update(L=T(Lh), ppl=True)
        c["host"]["L"] = Lh
    return c


def _round(c, seed=11, gen=3, max_attempts=1000):
    from pyabc_amd import gpu
    return gpu.CandidateRound(c["d"], c["S"], c["kind"], c["params"], c["src"],
                              c["a"], c["sigma"], c["x0"], c["wf"], c["p"],
                              seed, gen, max_attempts, X=c["X"], cdf=c["cdf"],
                              guide=c["guide"], L=c["L"],
                              per_particle_L=c["ppl"])


def _staged(c, lo, B, eps, seed=11, gen=3, max_attempts=1000):
    from pyabc_amd import gpu
    th, lp, anc, att = gpu.propose(c["X"], c["cdf"], c["L"], c["kind"], c["params"],
                                   seed, gen, lo, B, max_attempts, c["d"],
                                   per_particle_L=c["ppl"], guide=c["guide"])
    x = gpu.simulate_linear_gaussian(th, c["src"], c["a"], c["sigma"], seed, gen, lo)
    dist = gpu.pnorm(x, c["x0"], c["wf"], c["p"])
    gpu.mask_gave_up(dist, att, max_attempts)
    idx, cnt = gpu.accept_compact(dist, eps)
    n = int(cnt.cpu())
    return dict(theta=th, lp=lp, anc=anc, x=x, dist=dist, idx=idx[:n], n=n)


def _eps_for(dist, rate):
    return float(torch.quantile(dist[torch.isfinite(dist)][:200000], rate))


def _check_equal(c, fr, ref, lo, B, eps, filt):
    idx, cnt = fr.run(lo, B, eps, cap=max(ref["n"], 1), filter=filt)
    n = int(cnt.cpu())
    assert n == ref["n"]
    assert torch.equal(idx[:n], ref["idx"])
    th, lp, anc, x, dist = fr.regen(lo, idx[:n])
    sel = ref["idx"]
    assert torch.equal(th, ref["theta"][sel])
    assert torch.equal(x, ref["x"][sel])
    if c["S"] <= 32:
        assert torch.equal(dist, ref["dist"][sel])
    else:   # abc_pnorm sums wide rows lane-strided + wave tree (other order)
        torch.testing.assert_close(dist, ref["dist"][sel], rtol=1e-13, atol=0)
    assert torch.equal(lp, ref["lp"][sel])
    if c["X"] is not None:
        assert torch.equal(anc, ref["anc"][sel])
    return n


@pytest.mark.parametrize("mode,d,S", [("mvn", 10, 10), ("mvn", 1, 1), ("mvn", 3, 7),
                                      ("local", 5, 5), ("prior", 10, 10),
                                      ("mvn", 4, 256), ("mvn", 7, 13)])
@pytest.mark.parametrize("rate", [0.3, 0.01])
def test_fused_equals_staged(dev, mode, d, S, rate):
    c = _case(d, S, mode=mode, seed=d + S)
    lo, B = 123_456_789, 100_003
    probe = _staged(c, lo, B, np.inf)
    eps = _eps_for(probe["dist"], rate)
    ref = _staged(c, lo, B, eps)
    fr = _round(c)
    for filt in (False, True):
        n = _check_equal(c, fr, ref, lo, B, eps, filt)
    assert n > 0


@pytest.mark.parametrize("wkind", ["zeros", "heavy", "tiny", "n1", "n2", "n65"])
def test_ancestor_table_edge_weights(dev, wkind):
    """The fused rounds draw ancestors through abc_ancestor_table (padded
    records + exact-bin guide); the staged kernels through the cdf guide.
    Both must give np.searchsorted's ancestor: runs of zero weights (flat
    scan, leading and trailing), one row with most of the weight (a row
    spanning many bins), weights over 300 decades, N = 1, 2, 65."""
    from pyabc_amd import gpu
    N = {"n1": 1, "n2": 2, "n65": 65}.get(wkind, 4000)
    c = _case(3, 3, N=N, seed=4)
    rng = np.random.default_rng(8)
    w = rng.uniform(size=N)
    if wkind == "zeros":
        w[rng.uniform(size=N) < 0.7] = 0.0
        w[:5] = 0.0
        w[-5:] = 0.0
    elif wkind == "heavy":
        w[N // 3] = 1e6
    elif wkind == "tiny":
        w = 10.0 ** rng.uniform(-300, 0, N)
    cdf = gpu.inclusive_scan(T(w))
    c.update(cdf=cdf, guide=gpu.cdf_guide(cdf))
    lo, B = 99, 40_000
    ref = _staged(c, lo, B, 1e300)
    assert ref["n"] == B
    n = _check_equal(c, _round(c), ref, lo, B, 1e300, False)
    assert n == B
    anc = ref["anc"].cpu().numpy()
    if wkind == "zeros":    # zero-weight rows are never drawn
        assert (w[anc] > 0).all()
    if wkind == "heavy":
        assert (anc == N // 3).mean() > 0.9


@pytest.mark.parametrize("p", [1.0, np.inf, 3.0])
def test_fused_pnorm_orders(dev, p):
    c = _case(6, 11, p=p, seed=5)
    lo, B = 0, 50_000
    eps = _eps_for(_staged(c, lo, B, np.inf)["dist"], 0.05)
    ref = _staged(c, lo, B, eps)
    fr = _round(c)
    for filt in (False, True):
        _check_equal(c, fr, ref, lo, B, eps, filt)


def test_fused_prior_kinds_and_gave_up(dev):
    """Bounded priors: proposals outside the support are re-drawn with the
    same streams; with max_attempts = 2 some exhaust it and are rejected in
    both paths (never accepted with zero prior density)."""
    kinds = ["uniform", "expon", "gamma", "beta", "lognorm", "laplace"]
    params = [[0.0, 1.0, 0, 0], [0.2, 0.5, 0, 0], [2.0, 0.0, 1.0, 0],
              [2.0, 3.0, 0.0, 1.0], [0.5, 0.0, 1.0, 0], [0.0, 1.0, 0, 0]]
    c = _case(6, 6, kinds=kinds, params=params, seed=9)
    c["host"]["X"] = np.abs(c["host"]["X"]) * 0.5 + 0.1
    from pyabc_amd import gpu
    c["X"] = T(c["host"]["X"])
    lo, B = 77, 60_000
    for max_att in (1000, 2):
        # eps = inf too: a proposal that gave up is NaN, never <= eps
        for eps in (1e300, np.inf):
            ref = _staged(c, lo, B, eps, max_attempts=max_att)
            fr = _round(c, max_attempts=max_att)
            n = _check_equal(c, fr, ref, lo, B, eps, False)
            assert _check_equal(c, fr, ref, lo, B, eps, True) == n
            if max_att == 2:
                assert 0 < n < B     # some gave up and were rejected
            assert torch.isfinite(fr.regen(lo, ref["idx"][:1000])[1]).all()
    # prior mode (t = 0) with the same bounded kinds
    c0 = _case(6, 6, mode="prior", kinds=kinds, params=params, seed=9)
    ref = _staged(c0, lo, B, 1e300)
    _check_equal(c0, _round(c0), ref, lo, B, 1e300, False)


@pytest.mark.parametrize("p", [2.0, 1.0, np.inf, 3.0])
def test_fused_eps_on_a_distance(dev, p):
    """eps equal to some candidates' distances exactly: those candidates are
    accepted (d <= eps) by the round's accept bit and by the staged
    pipeline alike, and their regenerated distances are <= eps -- the round
    (p = 2: pnorm_acc<2>), the regeneration and the staged p-norm must
    round identically (no contraction anywhere, abc_candidate.h)."""
    c = _case(10, 10, p=p, seed=21)
    lo, B = 5_000, 80_000
    d = _staged(c, lo, B, np.inf)["dist"].cpu().numpy()
    fr = _round(c)
    for q in (100, 1000, 5000, 20000):
        eps = float(np.sort(d[np.isfinite(d)])[q])
        ref = _staged(c, lo, B, eps)
        hit = np.nonzero(d == eps)[0]
        assert len(hit) >= 1
        assert set(hit.tolist()) <= set(ref["idx"].cpu().numpy().tolist())
        n = _check_equal(c, fr, ref, lo, B, eps, False)
        assert n >= q + 1
        dist = fr.regen(lo, ref["idx"][:n])[4]
        assert bool((dist <= eps).all())


@pytest.mark.parametrize("variant", ["wide_uniform", "narrow_uniform", "src_late",
                                     "huge_x", "d5_S6", "w_zeros", "w_heavy", "w_tiny",
                                     "n65", "n1"])
def test_fused_lazy_filter(dev, variant):
    """The lazy early reject (filter mode, MVN, d > 4): theta_0..3 of attempt
    0 and statistics 0..3 decide the rejection when every coordinate k >= 4
    of any proposal lies in the support (lazy_filter_ok); otherwise the full
    proposal runs first.  Both must give the staged pipeline's accept set
    and rows bit for bit: bounded priors wide enough for the lazy head
    (uniform(-50, 100)), narrow ones (the head is refused, attempt 0 may be
    re-drawn), early-reject statistics reading theta_7 (refused), a
    population far out (|X| ~ 1e6: refused by the bound), and d = 5.  The
    lazy head reads its ancestor from the head bins (one record per scan
    bin with up to three candidate rows, abc_candidate.h): weights with runs
    of zeros, one dominant row, weights over 300 decades, N = 65 and N = 1
    exercise the bins holding more than three rows and the last rows."""
    d, S = (5, 6) if variant == "d5_S6" else (8, 9)
    N = {"n65": 65, "n1": 1}.get(variant, 3000)
    kinds, params, src = None, None, None
    if variant == "wide_uniform":
        kinds, params = ["uniform"] * d, [[-50.0, 150.0, 0, 0]] * d
    elif variant == "narrow_uniform":
        kinds, params = ["uniform"] * d, [[-1.0, 3.0, 0, 0]] * d
    elif variant == "src_late":
        src = [7, 1, 2, 3, 4, 5, 6, 0, 1]
    c = _case(d, S, N=N, kinds=kinds, params=params, src=src, seed=21)
    if variant.startswith("w_"):
        from pyabc_amd import gpu
        rng = np.random.default_rng(8)
        w = rng.uniform(size=N)
        if variant == "w_zeros":
            w[rng.uniform(size=N) < 0.7] = 0.0
            w[:5] = 0.0
            w[-5:] = 0.0
        elif variant == "w_heavy":
            w[N // 3] = 1e4
        else:
            w = 10.0 ** rng.uniform(-300, 0, N)
        cdf = gpu.inclusive_scan(T(w))
        c.update(cdf=cdf, guide=gpu.cdf_guide(cdf))
    if variant == "huge_x":
        c["host"]["X"] = c["host"]["X"] + 1e6
        c["X"] = T(c["host"]["X"])
        c["x0"] = T(np.full(S, 1e6 + 1.0))
    lo, B = 31, 120_000
    fr = _round(c)
    for rate in (0.2, 0.003):
        eps = _eps_for(_staged(c, lo, B, np.inf)["dist"], rate)
        ref = _staged(c, lo, B, eps)
        assert ref["n"] > 0
        for filt in (True, False):
            _check_equal(c, fr, ref, lo, B, eps, filt)


def test_fused_edges(dev):
    """Ragged B (1, 63, 64, 65, 2047, 2049), cap below the count, count 0,
    record rows for every candidate."""
    c = _case(3, 4, seed=1)
    fr = _round(c)
    for B in (1, 63, 64, 65, 2047, 2049, 10_000):
        ref = _staged(c, 5, B, 1.0)
        idx, cnt = fr.run(5, B, 1.0, cap=max(ref["n"], 1))
        assert int(cnt.cpu()) == ref["n"]
        assert torch.equal(idx[:ref["n"]], ref["idx"])
    ref = _staged(c, 5, 10_000, 1.5)
    assert ref["n"] > 20
    idx, cnt = fr.run(5, 10_000, 1.5, cap=7)
    assert int(cnt.cpu()) == ref["n"] and torch.equal(idx[:7], ref["idx"][:7])
    idx, cnt = fr.run(5, 10_000, -1.0, cap=3)
    assert int(cnt.cpu()) == 0
    rec = torch.empty((10_000, 4), dtype=torch.float64, device=dev)
    idx, cnt = fr.run(5, 10_000, 1.5, cap=ref["n"], rec_x=rec)
    assert torch.equal(rec, ref["x"]) and int(cnt.cpu()) == ref["n"]


def test_regen_device_sized(dev):
    """abc_candidates_regen sized on the device (the sampler queues it before
    reading the round's count): rows = min(n, *n_dev), identical to the
    host-sized regeneration; rows past them untouched; count 0 writes
    nothing."""
    from pyabc_amd import gpu
    c = _case(4, 6, seed=3)
    fr = _round(c)
    lo, B = 77, 20_000
    for eps, cap in ((1.2, 50), (1.2, 100_000), (-1.0, 10)):
        idx, cnt = fr.run(lo, B, eps, cap=cap)
        n = min(int(cnt.cpu()), cap)
        ref = fr.regen(lo, idx[:n]) if n else None
        outs = (torch.full((cap, 4), 7.0, dtype=torch.float64, device=dev),
                torch.full((cap,), 7.0, dtype=torch.float64, device=dev),
                torch.full((cap,), 7, dtype=torch.int64, device=dev),
                torch.full((cap, 6), 7.0, dtype=torch.float64, device=dev),
                torch.full((cap,), 7.0, dtype=torch.float64, device=dev))
        fr.regen_into(lo, idx.data_ptr(), min(cap, B), [o.data_ptr() for o in outs], n_dev=cnt)
        for o, r in zip(outs, ref if ref else (None,) * 5):
            if n:
                assert torch.equal(o[:n], r)
            assert bool((o[n:] == 7).all())


def test_round_keep_vs_cutoff(dev):
    """abc_round_keep (the multi-rank cutoff on the device) against the
    host's dd.cutoff: ranks 1..8, counts with zeros, need below / at / above
    the total."""
    from pyabc_amd import gpu
    from pyabc_amd.sampler import distributed as dd
    rng = np.random.default_rng(9)
    for ws in (1, 2, 3, 8):
        for _ in range(20):
            counts = rng.integers(0, 50, ws) * rng.integers(0, 2, ws)
            tot = int(counts.sum())
            for need in (0, 1, max(tot // 2, 1), tot, tot + 7):
                c = torch.as_tensor(counts, dtype=torch.int64, device=dev)
                want = dd.cutoff(counts, need)
                got = [int(gpu.round_keep(c, need, r).cpu()) for r in range(ws)]
                assert got == list(want), (counts, need)


def test_fused_vs_oracle_replay(dev):
    """Accept set against the numpy oracle's replay of the same streams
    (theta, x to 1e-12; masks equal away from |d - eps| < 1e-12)."""
    c = _case(10, 10, N=2000, seed=4)
    h = c["host"]
    lo, B, seed, gen = 999, 20_000, 11, 3
    th, lp, anc, att = osamp.propose_mvn(h["X"], h["w"], h["L"], seed, gen, lo, B,
                                         h["kinds"], h["params"])
    x = osamp.simulate_linear_gaussian(th, h["src"], h["a"], h["sigma"], seed, gen, lo)
    d = oracle.pnorm(x, h["x0"], p=2)
    eps = float(np.quantile(d, 0.05))
    fr = _round(c)
    idx, cnt = fr.run(lo, B, eps, cap=B)
    n = int(cnt.cpu())
    got = np.zeros(B, bool)
    got[idx[:n].cpu().numpy()] = True
    want = d <= eps
    near = np.abs(d - eps) < 1e-12
    assert np.array_equal(got[~near], want[~near])
    tg, lpg, ancg, xg, dg = fr.regen(lo, idx[:n])
    sel = idx[:n].cpu().numpy()
    np.testing.assert_array_equal(ancg.cpu().numpy(), anc[sel])
    np.testing.assert_allclose(tg.cpu().numpy(), th[sel], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(xg.cpu().numpy(), x[sel], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(dg.cpu().numpy(), d[sel], rtol=1e-12)
    np.testing.assert_allclose(lpg.cpu().numpy(), lp[sel], rtol=1e-12)


def _abc(fused, adaptive=False, pop=4000, max_fused=1 << 31, local=False, S=10,
         filter_below=0.01, dim=None):
    import pyabc_amd as pa
    d = dim or (4 if local else 10)
    names = [f"p{k}" for k in range(d)]
    keys = [f"y{k}" for k in range(S)]
    rng = np.random.default_rng(1234)
    model = pa.LinearGaussianModel(names, keys, src=[k % d for k in range(S)],
                                   a=rng.uniform(0.5, 2, S),
                                   sigma=10 ** rng.uniform(-1, 0.5, S))
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    dist = (pa.AdaptivePNormDistance(p=2) if adaptive else pa.PNormDistance(p=2))
    tr = pa.LocalTransition(k=50, k_fraction=None) if local else pa.MultivariateNormalTransition()
    sampler = pa.BatchedGPUSampler(seed=77, fused=fused,
                                   max_fused_batch_size=max_fused,
                                   filter_below=filter_below, filter_min_stats=5)
    np.random.seed(3)
    abc = pa.ABCSMC(model, prior, dist, population_size=pop, transitions=tr,
                    eps=pa.QuantileEpsilon(alpha=0.5), sampler=sampler)
    abc.new("sqlite://", {k: 0.5 for k in keys})
    return abc


@pytest.mark.parametrize("adaptive,local,max_fused,S,filt,dim",
                         [(False, False, 1 << 31, 10, 0.01, None),
                          (True, False, 1 << 31, 24, 0.01, None),
                          (False, False, 5000, 10, 0.01, None),
                          (False, True, 1 << 31, 6, 0.01, None),
                          (False, False, 1 << 31, 10, 1.0, None),
                          (False, False, 20000, 10, 1.0, None),
                          (False, True, 1 << 31, 12, 0.01, 12)])
def test_sampler_fused_equals_staged(dev, adaptive, local, max_fused, S, filt, dim):
    """Whole generations: fused and staged samplers give the same populations,
    weights, epsilons and evaluation counts (several rounds per generation
    with a small fused batch; every round in early-reject mode with
    filter_below = 1; LocalTransition at d = 12)."""
    runs = []
    for fused in (False, True):
        abc = _abc(fused, adaptive=adaptive, max_fused=max_fused, local=local, S=S,
                   filter_below=filt, dim=dim)
        h = abc.run(max_nr_populations=4)
        pops = [h.get_population_device(t) for t in range(h.max_t + 1)]
        runs.append((abc, pops, [g["n_sim"] for g in abc.generation_log],
                     [g["eps"] for g in abc.generation_log]))
        if fused:
            assert abc.sampler.last_stats.get("fused")
            if filt == 1.0:
                assert abc.sampler.last_stats.get("filtered_rounds", 0) > 0
    (_, p0, n0, e0), (_, p1, n1, e1) = runs
    assert n0 == n1 and e0 == e1
    for a, b in zip(p0, p1):
        assert torch.equal(a.theta, b.theta)
        assert torch.equal(a.weights, b.weights)
        assert torch.equal(a.distances, b.distances)
        assert torch.equal(a.sum_stats, b.sum_stats)


def unit_scale(data, x_0=None):
    """An adaptive distance's scale that keeps every weight at 1 (host scale
    function): record_rejected on, distances unchanged."""
    return 1.0


@pytest.mark.parametrize("adaptive", [False, True])
def test_sampler_fused_quantile_rerun(dev, adaptive):
    """Every candidate's statistics are 0 (a = 0, sigma = 0), so every
    distance is the same and QuantileEpsilon's knots sit in a tie run of
    4000 equal keys: the device select leaves the quantile undecided (NaN),
    each generation's first fused round runs at the NaN threshold, accepts
    nothing and is re-run at the host value (batched.py,
    last_stats["quantile_reruns"]).  The fused sampler's populations,
    weights, epsilons and evaluation counts equal the staged sampler's bit
    for bit -- also with record_rejected on (an adaptive distance whose
    scale keeps the weights at 1)."""
    import pyabc_amd as pa
    d, S = 4, 10
    names = [f"p{k}" for k in range(d)]
    keys = [f"y{k}" for k in range(S)]
    runs = []
    for fused in (False, True):
        model = pa.LinearGaussianModel(names, keys, src=[k % d for k in range(S)],
                                       a=np.zeros(S), sigma=np.zeros(S))
        prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
        dist = (pa.AdaptivePNormDistance(p=2, scale_function=unit_scale) if adaptive
                else pa.PNormDistance(p=2))
        sampler = pa.BatchedGPUSampler(seed=5, fused=fused)
        np.random.seed(3)
        abc = pa.ABCSMC(model, prior, dist, population_size=4000,
                        transitions=pa.MultivariateNormalTransition(),
                        eps=pa.QuantileEpsilon(alpha=0.5), sampler=sampler)
        abc.new("sqlite://", {k: 0.5 for k in keys})
        h = abc.run(max_nr_populations=3)
        if fused:
            st = abc.sampler.last_stats
            assert st.get("fused") and st["quantile_reruns"] == 1
        assert abc.sampler.sample_factory.record_rejected == adaptive
        pops = [h.get_population_device(t) for t in range(h.max_t + 1)]
        runs.append((pops, [g["n_sim"] for g in abc.generation_log],
                     [g["eps"] for g in abc.generation_log]))
    (p0, n0, e0), (p1, n1, e1) = runs
    assert n0 == n1 and e0 == e1
    for a, b in zip(p0, p1):
        assert torch.equal(a.theta, b.theta)
        assert torch.equal(a.weights, b.weights)
        assert torch.equal(a.distances, b.distances)
        assert torch.equal(a.sum_stats, b.sum_stats)


def test_box_muller_accuracy(dev):
    """The fp32 Box-Muller transform (abc_common.h): on 4M draws (the
    simulator with a = 0, sigma = 1 returns the raw normals) the device
    normals equal the oracle's float32 replay (oracle/philox.py
    normal_pairs) BIT FOR BIT, and are within 4 fp32 ulp of R of an 80-bit
    long-double evaluation of R cos / R sin, R = sqrt(-2 ln u1), u1 = (a | 1)
    2^-32, below 2^-23 ((a << 9 | b & 511) | 1) 2^-41 (normals reach 7.54)."""
    from pyabc_amd import gpu
    from oracle.philox import normal_pairs, philox4x32_10
    B, S = 1 << 20, 4
    th = torch.zeros((B, 1), dtype=torch.float64, device=dev)
    x = gpu.simulate_linear_gaussian(th, T(np.zeros(S), torch.int32), T(np.zeros(S)),
                                     T(np.ones(S)), 5, 6, 7).cpu().numpy()
    idx = np.arange(7, 7 + B, dtype=np.uint64)
    r = philox4x32_10(idx, 0x40000000, 6, 5)
    ld = np.longdouble
    for h in range(2):
        ref = np.stack(normal_pairs(r[:, 2 * h], r[:, 2 * h + 1]), 1)
        np.testing.assert_array_equal(x[:, 2 * h:2 * h + 2], ref)
        rr = r.astype(np.uint64)
        a, b = rr[:, 2 * h], rr[:, 2 * h + 1]
        u1 = np.where(a < np.uint64(512),
                      ((a << np.uint64(9)) | (b & np.uint64(511)) | np.uint64(1)).astype(ld)
                      * ld(2.0) ** -41, (a | np.uint64(1)).astype(ld) * ld(2.0) ** -32)
        m2 = ((b >> np.uint64(9)) * 2 + 1).astype(ld)
        R = np.sqrt(-2 * np.log(u1))
        ang = ld("3.14159265358979323846264338327950288") * m2 * ld(2.0) ** -23
        exact = np.stack([(R * np.cos(ang)).astype(np.float64),
                          (R * np.sin(ang)).astype(np.float64)], 1)
        ulp = np.abs(x[:, 2 * h:2 * h + 2] - exact) / \
            np.spacing(R.astype(np.float32)).astype(np.float64)[:, None]
        assert ulp.max() <= 4, ulp.max()


def test_box_muller_tail_words(dev):
    """The 41-bit u1 branch (first word < 2^9: u1 takes the angle word's 9
    low bits) on the device: simulator draws at Philox indices whose u1 word
    is below 512 (found by scanning oracle.philox4x32_10 for seed 5,
    generation 6, the simulator slot) equal the oracle replay bit for bit,
    and their radius lies beyond the 2^-23 edge (sqrt(46 ln 2) = 5.64)."""
    from pyabc_amd import gpu
    from oracle.philox import normal_pairs, philox4x32_10
    hits = [4877494, 8440393, 12144803, 20704936, 22109970, 22722510]
    S = 4
    for h in hits:
        r = philox4x32_10(np.array([h], dtype=np.uint64), 0x40000000, 6, 5)[0]
        assert r[0] < 512 or r[2] < 512
        th = torch.zeros((1, 1), dtype=torch.float64, device=dev)
        x = gpu.simulate_linear_gaussian(th, T(np.zeros(S), torch.int32), T(np.zeros(S)),
                                         T(np.ones(S)), 5, 6, h).cpu().numpy()[0]
        for q in (0, 2):
            n0, n1 = normal_pairs(r[q:q + 1], r[q + 1:q + 2])
            np.testing.assert_array_equal(x[q:q + 2], [n0[0], n1[0]])
            if r[q] < 512:
                assert np.hypot(n0[0], n1[0]) > np.sqrt(46 * np.log(2)) - 1e-6


@pytest.mark.parametrize("mode,d", [("mvn", 10), ("mvn", 3), ("local", 5), ("prior", 10),
                                    ("mvn", 7), ("mvn", 20)])
def test_proposal_only_round_equals_propose(dev, mode, d):
    """abc_candidates_propose (the staged sampler path's proposals through
    the fused kernel's propose_one: ancestor table, support box once per
    launch, theta rows leaving through LDS) returns gpu.propose's rows bit
    for bit: theta, prior log-density, ancestor, attempts -- including
    ragged block tails, d > 16 (runtime-d kernel) and bounded priors that
    exhaust max_attempts = 2."""
    from pyabc_amd import gpu
    c = _case(d, 1, mode=mode, seed=d)
    lo = 12345
    for B, max_att in ((1, 1000), (1023, 1000), (70_001, 1000)):
        fr = _round(c, max_attempts=max_att)
        th, lp, anc, att = fr.propose(lo, B)
        th2, lp2, anc2, att2 = gpu.propose(c["X"], c["cdf"], c["L"], c["kind"], c["params"],
                                           11, 3, lo, B, max_att, d,
                                           per_particle_L=c["ppl"], guide=c["guide"])
        assert torch.equal(th, th2) and torch.equal(lp, lp2) and torch.equal(att, att2)
        if mode != "prior":
            assert torch.equal(anc, anc2)
    # bounded priors, attempts exhausted
    kinds = ["uniform", "expon", "gamma", "beta", "lognorm", "laplace"]
    params = [[0.0, 1.0, 0, 0], [0.2, 0.5, 0, 0], [2.0, 0.0, 1.0, 0],
              [2.0, 3.0, 0.0, 1.0], [0.5, 0.0, 1.0, 0], [0.0, 1.0, 0, 0]]
    c = _case(6, 1, kinds=kinds, params=params, seed=9)
    c["host"]["X"] = np.abs(c["host"]["X"]) * 0.5 + 0.1
    c["X"] = T(c["host"]["X"])
    fr = _round(c, max_attempts=2)
    th, lp, anc, att = fr.propose(77, 50_000)
    th2, lp2, anc2, att2 = gpu.propose(c["X"], c["cdf"], c["L"], c["kind"], c["params"],
                                       11, 3, 77, 50_000, 2, 6, guide=c["guide"])
    assert (att > 2).any() and torch.isinf(lp[att > 2]).all()
    assert torch.equal(th, th2) and torch.equal(lp, lp2) and torch.equal(att, att2)
    assert torch.equal(anc, anc2)
