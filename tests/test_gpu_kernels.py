"""GPU parity: every kernel, through the C ABI, against the CPU oracle and the
reference golden vectors (tests/golden).  Tolerances are stated per test:
integer / index / accept-mask work is exact; fp64 arithmetic 1e-10..1e-12;
the transition density 2e-6 relative in the f64-MFMA mode (exp2 of the
shifted exponent is fp32) and 1e-4 in the f32-MFMA fast mode.
"""
import os

import numpy as np
import pytest

import oracle
import oracle.sampler as osamp
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    from pyabc_amd import gpu
    return gpu.require_device()


def g(name):
    return np.load(os.path.join(GOLDEN, name))


def T(a, dtype=None):
    from pyabc_amd import gpu
    return gpu.as_dev(a, dtype=dtype)


MVN = ["d1_n1000", "d2_n500", "d10_n4096", "d3_unnorm_scaled"]


@pytest.mark.parametrize("tag", MVN)
@pytest.mark.parametrize("precision,rtol", [("x3", 1e-6), ("f64", 2e-6),
                                            ("f32", 1e-4)])
def test_mvn_pdf_golden(dev, tag, precision, rtol):
    import pandas as pd
    from pyabc_amd.transition import MultivariateNormalTransition
    gg = g(f"mvn_{tag}.npz")
    d = gg["X"].shape[1]
    cols = [f"p{k:02d}" for k in range(d)]
    t = MultivariateNormalTransition(scaling=float(gg["scaling"]),
                                     precision=precision)
    w = gg["w"].copy()
    t.fit(pd.DataFrame(gg["X"], columns=cols), w)
    np.testing.assert_allclose(w, gg["w_fit"], rtol=1e-13)
    np.testing.assert_allclose(t.cov, gg["cov"], rtol=1e-10, atol=1e-14)
    assert t._mfma
    pdf = t.pdf(pd.DataFrame(gg["x"], columns=cols))
    np.testing.assert_allclose(pdf, gg["pdf"], rtol=rtol, atol=0)


@pytest.mark.parametrize("d,rule,rank,tiny", [(1, 0, 1, 1), (2, 1, 2, 1), (10, 0, 10, 1),
                                              (10, 0, 7, 1), (25, 1, 25, 1), (40, 0, 40, 1),
                                              (64, 0, 64, 1), (6, 0, 6, 1e-7), (8, 1, 8, 3e-4),
                                              (7, 0, 7, 1.8e-4), (7, 1, 7, 2.5e-4)])
def test_mvn_fit_device_vs_host(dev, d, rule, rank, tiny):
    """abc_mvn_fit (the fit's covariance, PSD eigen-whitening and sampling
    factor on the device, parallel Jacobi in fp64) against the host path it
    replaces (np.cov * bw^2 * scaling and scipy's _PSD via numpy eigh):
    covariance 1e-12 relative, eigenvalues 1e-12 of the largest, rank
    equal, log pdet 1e-11 (plus d eps sum s_max / s_i for ill-conditioned
    fits), U U^T = cov^+ (the pseudo-inverse on the kept eigenspace) to 1e-9
    (or 8 d eps kappa) of its largest entry, L lower with L L^T = cov to
    1e-12 of the largest entry; rank-deficient populations (rank < d: the
    points span a subspace), a direction 1e-7 thinner than the others
    (scipy's cut-off drops it: rank d - 1) and one 3e-4 thinner (kept, but
    the Cholesky path cannot certify it: the eigen path decides); at d = 7
    directions 1.8e-4 / 2.5e-4 thinner put the smallest eigenvalue at ~0.8 /
    ~1.5 x the cut-off (dropped / kept): L L^T = cov still to 1e-12 (L from
    the eigen factor, as the host's psd_whitening; a semidefinite Cholesky
    zeroing near-cut pivots left off-diagonal terms up to sqrt(cut c_ii)
    out).
    Well-conditioned full-rank covariances take the Cholesky path (U = L^-T,
    no eigenvectors: evec / evals NaN)."""
    from pyabc_amd import gpu
    from pyabc_amd.transition.multivariatenormal import (
        psd_whitening, silverman_rule_of_thumb, scott_rule_of_thumb)
    rng = np.random.default_rng(7 * d + rank)
    N = 3000
    B = rng.standard_normal((rank, d)) * rng.uniform(0.2, 3.0, (rank, 1))
    B[0] *= tiny
    X = rng.standard_normal((N, rank)) @ B + 0.3
    w = np.exp(0.5 * rng.standard_normal(N))
    w /= w.sum()
    Xd, wd = T(X), T(w)
    mom = gpu.weighted_moments_dev(Xd, wd)
    cov, evec, evals, U, L, st = (a.cpu().numpy() for a in gpu.mvn_fit(mom, d, 1.3, rule))
    sw, sw2, mean, cov_b = gpu.weighted_moments(Xd, wd)
    bw = (silverman_rule_of_thumb, scott_rule_of_thumb)[rule](1 / sw2, d)
    ref = cov_b * sw / (sw - sw2 / sw) * bw ** 2 * 1.3
    scale = max(np.abs(ref).max(), 1e-300)
    np.testing.assert_allclose(cov, ref, rtol=1e-12, atol=1e-14 * scale)
    assert st[7] == 1.0
    psd = psd_whitening(ref)
    s_ref = np.sort(np.linalg.eigvalsh(ref))[::-1]
    eigen_path = not np.isnan(evals).all()
    assert eigen_path == (psd["rank"] < d or tiny < 1)
    if eigen_path:
        np.testing.assert_allclose(evals, s_ref, rtol=0, atol=1e-12 * s_ref[0])
        np.testing.assert_allclose(np.abs(evec.T @ evec), np.eye(d), atol=1e-12)
    assert int(st[0]) == psd["rank"] == (rank - 1 if tiny < 2e-4 else rank)
    # both eigensolvers are backward stable (eigenvalue errors ~ d eps s_max),
    # so the kept small eigenvalues carry relative errors ~ d eps s_max / s_i
    kept = s_ref[:psd["rank"]]
    eps = np.finfo(float).eps
    assert st[1] == pytest.approx(psd["log_pdet"], rel=1e-11,
                                  abs=1e-11 + d * eps * (kept[0] / kept).sum())
    assert st[3] == pytest.approx(-np.log(w.max()), rel=1e-15)
    P = U @ U.T
    P_ref = psd["U"] @ psd["U"].T
    kappa = kept[0] / kept[-1]
    assert np.abs(P - P_ref).max() <= max(1e-9, 8 * d * eps * kappa) * np.abs(P_ref).max()
    assert np.all(np.triu(L, 1) == 0)
    np.testing.assert_allclose(L @ L.T, ref, rtol=0, atol=1e-12 * scale)


@pytest.mark.parametrize("tag", ["singular", "n1"])
def test_mvn_pdf_direct_golden(dev, tag):
    import pandas as pd
    from pyabc_amd.transition import MultivariateNormalTransition
    gg = g(f"mvn_{tag}.npz")
    d = gg["X"].shape[1]
    cols = [f"p{k:02d}" for k in range(d)]
    t = MultivariateNormalTransition()
    t.fit(pd.DataFrame(gg["X"], columns=cols), gg["w"].copy())
    np.testing.assert_allclose(t.cov, gg["cov"], rtol=1e-10, atol=1e-14)
    pdf = np.atleast_1d(t.pdf(pd.DataFrame(gg["x"], columns=cols)))
    # singular -> direct fp64 kernel (1e-10); n1 is full rank -> f64 MFMA
    np.testing.assert_allclose(pdf, gg["pdf"], rtol=2e-6 if t._mfma else 1e-10,
                               atol=1e-300)
    if tag == "singular":
        assert not t._mfma
        assert (pdf[::4] == 0).all() and (pdf[1::4] > 0).all()


def test_mvn_pdf_large_vs_oracle(dev):
    """N = 1e5, d = 10 (the c2 shape): subset of candidates vs the oracle."""
    import pandas as pd
    from pyabc_amd.transition import MultivariateNormalTransition
    rng = np.random.default_rng(5)
    N, d = 100_000, 10
    X = 0.8 + np.sqrt(0.2) * rng.standard_normal((N, d))
    w = np.exp(0.5 * rng.standard_normal(N))
    w /= w.sum()
    cols = [f"p{k}" for k in range(d)]
    t = MultivariateNormalTransition()
    t.fit(pd.DataFrame(X, columns=cols), w.copy())
    assert t.precision == "x3" and t._prec == 2
    cand = t.rvs(4096).values
    ref = oracle.mvn_logpdf(cand[:200], X, w, t.cov)
    lp = t.logpdf_device(T(cand)).cpu().numpy()
    np.testing.assert_allclose(np.exp(lp[:200] - ref), 1.0, rtol=1e-6)
    t64 = MultivariateNormalTransition(precision="f64")
    t64.fit(pd.DataFrame(X, columns=cols), w.copy())
    lp64 = t64.logpdf_device(T(cand)).cpu().numpy()
    np.testing.assert_allclose(np.exp(lp64[:200] - ref), 1.0, rtol=2e-6)
    # all 4096: x3 against the f64-MFMA kernel
    np.testing.assert_allclose(np.exp(lp - lp64), 1.0, rtol=3e-6)
    t32 = MultivariateNormalTransition(precision="f32")
    t32.fit(pd.DataFrame(X, columns=cols), w.copy())
    lp32 = t32.logpdf_device(T(cand)).cpu().numpy()
    np.testing.assert_allclose(np.exp(lp32 - lp), 1.0, rtol=1e-4)


def test_mvn_x3_rescue_and_edges(dev):
    """x3 kernel: candidates outside the limb range and candidates whose
    density underflows are recomputed in fp64; zero weights; ragged sizes."""
    import pandas as pd
    from pyabc_amd.transition import MultivariateNormalTransition
    rng = np.random.default_rng(11)
    for N, d in [(1, 3), (17, 2), (1000, 5), (4099, 10)]:
        X = rng.normal(0, 1, (N, d))
        w = np.exp(rng.standard_normal(N))
        if N > 10:
            w[::7] = 0.0
        w /= w.sum()
        cols = [f"p{k}" for k in range(d)]
        t = MultivariateNormalTransition()
        t.fit(pd.DataFrame(X, columns=cols), w.copy())
        near = X[rng.integers(0, N, 300)] + 0.5 * rng.standard_normal((300, d))
        far = np.vstack([np.full(d, 40.0), np.full(d, -1e3),
                         X[0] + 8.0 * np.sqrt(np.diag(t.cov)) * 12])
        x = np.vstack([near, far])
        lp = t.logpdf_device(T(x)).cpu().numpy()
        ref = oracle.mvn_logpdf(x, X, w, t.cov)
        ok = np.isfinite(ref)
        assert (np.isfinite(lp) == ok).all()
        if t._prec == 2:
            np.testing.assert_allclose(np.exp(lp[:300] - ref[:300]), 1.0,
                                       rtol=1e-6)
        np.testing.assert_allclose(lp[300:][ok[300:]], ref[300:][ok[300:]],
                                   rtol=1e-9)


@pytest.mark.parametrize("d", [1, 7, 11, 12, 16, 25])
def test_mvn_x3_ranks_vs_oracle(dev, d):
    """The x3 density against the fp64 oracle over whitened ranks 1..25 (the
    largest x3 rank; KB = 2..6 MFMA blocks per tile pair), unhinted (max
    pre-pass) and hinted by the proposals' ancestors; 1e-6 / 2e-6."""
    import pandas as pd
    from pyabc_amd.transition import MultivariateNormalTransition
    rng = np.random.default_rng(100 + d)
    N = 5000
    X = 0.5 + 0.7 * rng.standard_normal((N, d))
    w = np.exp(0.7 * rng.standard_normal(N))
    w /= w.sum()
    cols = [f"p{k:02d}" for k in range(d)]
    t = MultivariateNormalTransition()
    t.fit(pd.DataFrame(X, columns=cols), w.copy())
    assert t._prec == 2
    th, _, anc, _ = t.propose_device(1500)
    x = th.cpu().numpy()
    ref = oracle.mvn_logpdf(x, X, w, t.cov)
    lp = t.logpdf_device(th).cpu().numpy()
    np.testing.assert_allclose(np.exp(lp - ref), 1.0, rtol=1e-6)
    lph = t.logpdf_device(th, hint=anc).cpu().numpy()
    np.testing.assert_allclose(np.exp(lph - ref), 1.0, rtol=2e-6)


def test_mvn_x3_hinted_offsets(dev):
    """x3 with per-candidate offsets from a hint row (the sampler passes the
    proposal's ancestor) instead of the max pre-pass: ancestors, random rows,
    far rows (offset clamped, rescue) and invalid rows (-> fp64 rescue) all
    match the oracle within 2e-6 relative (the offset adds up to
    2^-24 * 20 * ln 2 = 8e-7 to the pre-pass path's rounding)."""
    import pandas as pd
    from pyabc_amd.transition import MultivariateNormalTransition
    rng = np.random.default_rng(21)
    for N, d in [(50, 2), (3000, 10), (20_000, 10)]:
        X = 0.8 + np.sqrt(0.2) * rng.standard_normal((N, d))
        w = np.exp(0.5 * rng.standard_normal(N))
        w[::11] = 0.0
        w /= w.sum()
        cols = [f"p{k}" for k in range(d)]
        t = MultivariateNormalTransition()
        t.fit(pd.DataFrame(X, columns=cols), w.copy())
        assert t._prec == 2
        M = 700
        th, _, anc, _ = t.propose_device(M)
        x = th.cpu().numpy()
        ref = oracle.mvn_logpdf(x, X, w, t.cov)
        base = t.logpdf_device(th).cpu().numpy()
        hints = {
            "ancestor": anc,
            "random": torch.as_tensor(rng.integers(0, N, M), device=dev),
            "far": torch.as_tensor(np.argmax(((X - X.mean(0)) ** 2).sum(1))
                                   * np.ones(M, dtype=np.int64), device=dev),
            "invalid": torch.as_tensor(np.where(np.arange(M) % 3 == 0, -1,
                                                np.where(np.arange(M) % 3 == 1,
                                                         N + 5, 0)),
                                       device=dev),
        }
        for name, h in hints.items():
            lp = t.logpdf_device(th, hint=h.to(torch.int64)).cpu().numpy()
            np.testing.assert_allclose(np.exp(lp - ref), 1.0, rtol=2e-6,
                                       err_msg=f"N={N} hint={name}")
        np.testing.assert_allclose(np.exp(base - ref), 1.0, rtol=1e-6)
    with pytest.raises(ValueError):
        t.logpdf_device(th, hint=torch.zeros(3, dtype=torch.int64, device=dev))


def test_mvn_x3_rescue_overflow(dev):
    """More rescued rows than the nested exact pass holds (X3_NEST_CAP =
    16384, abc_mvn_x3.hip): every hint invalid, so all M = 20000 candidates
    are rescued; the first 16384 list entries take the nested x3 pass, the
    rest the fp64 rescue kernel.  Both match the oracle within the hinted
    bar (2e-6)."""
    import pandas as pd
    from pyabc_amd.transition import MultivariateNormalTransition
    rng = np.random.default_rng(5)
    N, d, M = 3000, 10, 20_000
    X = 0.8 + np.sqrt(0.2) * rng.standard_normal((N, d))
    w = np.exp(0.5 * rng.standard_normal(N))
    w /= w.sum()
    t = MultivariateNormalTransition()
    t.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(d)]), w.copy())
    assert t._prec == 2
    th, _, _, _ = t.propose_device(M)
    ref = oracle.mvn_logpdf(th.cpu().numpy(), X, w, t.cov)
    for h in (-1, N + 7):
        hint = torch.full((M,), h, dtype=torch.int64, device=dev)
        lp = t.logpdf_device(th, hint=hint).cpu().numpy()
        np.testing.assert_allclose(np.exp(lp - ref), 1.0, rtol=2e-6, err_msg=f"hint {h}")


@pytest.mark.parametrize("tag,kw", [("k50", dict(k=50, k_fraction=None)),
                                    ("default", dict())])
def test_local_golden(dev, tag, kw):
    import pandas as pd
    from pyabc_amd.transition import LocalTransition
    gg = g(f"local_{tag}.npz")
    d = gg["X"].shape[1]
    cols = [f"p{k:02d}" for k in range(d)]
    t = LocalTransition(**kw)
    t.fit(pd.DataFrame(gg["X"], columns=cols), gg["w"].copy())
    assert t.k == int(gg["k"])
    np.testing.assert_allclose(t.covs, gg["covs"], rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(t.determinants, gg["dets"], rtol=1e-8)
    np.testing.assert_allclose(t.inv_covs, gg["inv_covs"], rtol=1e-8, atol=1e-10)
    pdf = t.pdf(pd.DataFrame(gg["x"], columns=cols))
    # the density's log-sum-exp runs on the f32 exp2 unit (exponents fp64):
    # ~1e-7 relative; the north star's fp32 bar is 1e-5
    np.testing.assert_allclose(pdf, gg["pdf"], rtol=1e-6)


@pytest.mark.parametrize("d", [2, 3])
def test_local_fit_singular_neighbourhoods(dev, d):
    """d + 1 particles: every neighbour covariance is exactly singular and
    local_transition.py:112-123 ("while det <= 0: cov += EPS I") runs on
    rounding noise.  Whatever the noise decides, det and inverse must come
    from one factorisation (la.det / la.inv share getrf in the reference):
    a covariance kept with det > 0 has an inverse with a positive diagonal,
    and the densities stay finite and below the largest kernel's peak."""
    import pandas as pd
    from pyabc_amd.transition import LocalTransition
    rng = np.random.default_rng(77 + d)
    cols = [f"p{k}" for k in range(d)]
    for rep in range(150):
        X = rng.random((d + 1, d))
        t = LocalTransition()
        t.fit(pd.DataFrame(X, columns=cols), np.ones(d + 1) / (d + 1))
        dets = t._dev_dets.cpu().numpy()
        inv = t._dev_inv.cpu().numpy()
        assert (dets > 0).all()
        assert (np.einsum("nii->ni", inv) > 0).all(), (rep, dets, inv)
        ld = t.logpdf_device(gpu_as(rng.random((4, d)), dev)).cpu().numpy()
        peak = (-0.5 * (d * np.log(2 * np.pi) + np.log(dets))).max()
        assert np.all(ld <= peak + 1e-6 * abs(peak)), (rep, ld, peak)


def gpu_as(a, dev):
    from pyabc_amd import gpu
    return gpu.as_dev(a, device=dev)


@pytest.mark.parametrize("grid,N,d,k", [(None, 3000, 5, 50), (None, 3000, 5, 700),
                                         (7, 2000, 3, 50), (2, 1500, 3, 40),
                                         (None, 12000, 5, 3000), (None, 4096, 2, 10),
                                         (3, 5000, 4, 200), (None, 3000, 10, 50),
                                         (None, 2500, 16, 300), (3, 3000, 9, 100),
                                         (None, 9000, 13, 2500), (2, 1500, 3, 400),
                                         (3, 3000, 4, 1000), (None, 2048, 1, 600),
                                         (None, 1000, 8, 999), (None, 70, 6, 20)])
def test_local_fit_selection_paths_vs_oracle(dev, grid, N, d, k):
    """k-NN selection: the sample-bracketed path (N >= 2048), the LDS bucket
    path (small and large k) and the radix-pass fallback (a {0,1}^3 grid: buckets of hundreds of exact ties,
    taken by index) against the oracle's (distance, index) order.  d = 9..16
    run the 4-particle selection blocks and the sliced moments (several
    kernels over one moment list each).  k > N / 16 at d <= 5 takes the f16-limb moments
    GEMM (mm_moments_kernel), including grids of ties and d = 1."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(N + k)
    if grid is None:
        X = rng.normal(size=(N, d))
    else:
        X = rng.integers(0, grid, size=(N, d)).astype(float)
    w = np.exp(0.3 * rng.standard_normal(N))
    w /= w.sum()
    ref = oracle.local_fit(X, w, k=k, k_fraction=None)
    covs, inv, dets, chol, lnorm = gpu.local_fit(gpu.as_dev(X), gpu.as_dev(w), k,
                                                 1.0, 1e-3)
    np.testing.assert_allclose(covs.cpu().numpy(), ref["covs"], rtol=1e-9,
                               atol=1e-12)
    np.testing.assert_allclose(dets.cpu().numpy(), ref["dets"], rtol=1e-8)


@pytest.mark.parametrize("scale", [1e3, 1e7])
def test_local_fit_dense_outlier(dev, scale):
    """k > N / 16 at d <= 5 takes the f16-limb moments GEMM (abc_local.hip
    mm_moments_kernel), whose block exponents come from the population's
    largest |x - x_0|.  One far outlier stretches them: the per-particle
    rounding bound then decides between the GEMM and the VALU kernel (at
    1e7 it sends the fit back), and either way the covariances must be the
    oracle's."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(int(scale))
    N, d, k = 3000, 3, 700
    X = rng.normal(size=(N, d))
    X[17] = scale
    w = np.exp(0.3 * rng.standard_normal(N))
    w /= w.sum()
    ref = oracle.local_fit(X, w, k=k, k_fraction=None)
    covs, inv, dets, chol, lnorm = gpu.local_fit(gpu.as_dev(X), gpu.as_dev(w), k, 1.0, 1e-3)
    # the outlier's own neighbourhood covariance is (S2/sw - mean^2) with
    # |delta| ~ scale: a cancellation both the oracle and the kernels round
    # at ~1e-16 scale^2 / var, so it is left out
    keep = np.arange(N) != 17
    np.testing.assert_allclose(covs.cpu().numpy()[keep], ref["covs"][keep], rtol=1e-9,
                               atol=1e-12)


@pytest.mark.parametrize("offset,spread,k", [(1e3, 0.01, 50), (1e3, 0.01, 700),
                                             (-3e5, 1.0, 50), (0.0, 1e-6, 50)])
def test_local_fit_fp32_prefilter_stress(dev, offset, spread, k):
    """The moments sweep decides membership in fp32 where a rigorous bound
    allows it (abc_local.hip f32_bound).  Populations far from the origin
    relative to their spread (fp32 keeps ~1e-3 of the distances' bits, so
    most pairs fall between the cuts) and tiny spreads must still give the
    oracle's exact neighbourhoods."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(int(abs(offset)) + k)
    N, d = 4000, 5
    X = offset + spread * rng.normal(size=(N, d))
    w = np.exp(0.3 * rng.standard_normal(N))
    w /= w.sum()
    ref = oracle.local_fit(X, w, k=k, k_fraction=None)
    covs, inv, dets, chol, lnorm = gpu.local_fit(gpu.as_dev(X), gpu.as_dev(w), k, 1.0, 1e-3)
    np.testing.assert_allclose(covs.cpu().numpy(), ref["covs"], rtol=1e-8,
                               atol=1e-12 * spread ** 2)


@pytest.mark.parametrize("d,N,M,offset", [(5, 3001, 777, 0.0), (2, 17, 5, 40.0),
                                            (8, 1000, 130, 5.0), (1, 64, 64, 0.0),
                                            (10, 700, 130, 2.0), (13, 333, 65, 1.0),
                                            (16, 500, 70, 0.0)])
def test_local_logpdf_mfma_vs_oracle(dev, d, N, M, offset):
    """fp64-MFMA quadratic-feature GEMM vs the fp64 oracle: ragged N / M
    (tiles of 16 rows, 64-candidate waves), a population far from the origin
    (centring), zero weights, a far-away candidate (pdf underflows to 0)."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(d * 1000 + N)
    X = offset + rng.normal(size=(N, d)) * (1 + np.arange(d))
    w = rng.random(N)
    w[::7] = 0.0
    w /= w.sum()
    A = rng.normal(size=(N, d, d)) * 0.3
    covs = np.einsum("nij,nkj->nik", A, A) + 0.2 * np.eye(d)
    inv = np.linalg.inv(covs)
    norm = np.sqrt((2 * np.pi) ** d * np.linalg.det(covs))
    x = X[rng.integers(0, N, M)] + 0.5 * rng.normal(size=(M, d))
    x[0] += 1e4
    fit = dict(w=w, inv_covs=inv, normalization=norm)
    ref = oracle.local_logpdf(x, X, fit)
    got = gpu.local_logpdf(gpu.as_dev(x), gpu.as_dev(X), gpu.as_dev(w),
                           gpu.as_dev(inv), gpu.as_dev(np.log(norm))).cpu().numpy()
    # far candidate: the reference's pdf underflows to 0 (log -inf); the
    # log-space sum keeps the exact log, whose exp is the same 0
    assert ref[0] == -np.inf and got[0] < -1e5 and np.exp(got[0]) == 0.0
    got, ref = got[1:], ref[1:]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin)
    # log density: absolute 1e-6 ~ relative 1e-6 of the density
    np.testing.assert_allclose(got[fin], ref[fin], rtol=0, atol=2e-6)


def test_pnorm_golden(dev):
    from pyabc_amd import gpu
    gg = g("pnorm.npz")
    for c in sorted({k.split("__")[0] for k in gg.files}):
        wf = gg[c + "__w"] * gg[c + "__f"]
        dd = gpu.pnorm(T(gg[c + "__x"]), T(gg[c + "__x0"]), T(wf),
                       float(gg[c + "__p"])).cpu().numpy()
        np.testing.assert_allclose(dd, gg[c + "__d"], rtol=1e-12, err_msg=c)


@pytest.mark.parametrize("B,S", [(1, 33), (3, 256), (17, 100), (1001, 256), (64, 700)])
def test_pnorm_wave_rows_vs_oracle(dev, B, S):
    """Wide-row PNorm (S > 32: several rows per wave, ragged last wave)."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(B * 1000 + S)
    x = rng.standard_normal((B, S)) * 10 ** rng.uniform(-2, 2, S)
    x0 = rng.standard_normal(S)
    w = rng.uniform(0.1, 2.0, S)
    for p in (1.0, 2.0, 3.0, np.inf):
        dd = gpu.pnorm(T(x), T(x0), T(w), p).cpu().numpy()
        np.testing.assert_allclose(dd, oracle.pnorm(x, x0, w=w, p=p), rtol=1e-12,
                                   err_msg=f"p={p}")


def test_weighted_quantile_golden(dev):
    from pyabc_amd import gpu
    gg = g("quantile.npz")
    for name in ("n10k", "ties", "zerow", "n1"):
        pts, w = gg[f"{name}__points"], gg[f"{name}__w"]
        for a in (0.2, 0.5, 0.9, 1.0):
            P, W = T(pts), T(w)
            q = gpu.resolve_quantile(gpu.weighted_quantile(P, W, a).cpu()[0], P, W, a)
            ref = oracle.weighted_quantile(pts, w, a, kind="stable")
            assert q == pytest.approx(ref, rel=1e-12, abs=1e-15), (name, a)
            if name != "ties":
                assert q == pytest.approx(float(gg[f"{name}__a{a}__q"]),
                                          rel=1e-12), (name, a)


@pytest.mark.parametrize("case", ["normal", "skewed_w", "heavy_ties", "one_value",
                                  "two_spikes", "zero_w", "big", "one_max", "dense_core",
                                  "crowded", "discrete", "tiny"])
def test_weighted_quantile_select(dev, case):
    """The weighted MSD select (abc_quantile.hip) against the oracle's stable
    sort + cumsum + interp (weighted_statistics.py:27-43): continuous data,
    skewed weights, ties by the thousand (the final block's refinement), one
    value for every point (the run summary), two spikes straddling the
    quantile, zero weights, N = 2e6 (four launches), N = 2^20 (the one-launch
    path's largest grid), half the points in 1e-4 of the range (the
    one-launch path's third level), the bulk crowded next to two extreme
    points (the segment keeps its lone neighbours, no level narrows it: left
    to the sorted path), integer-valued distances, N <= 3; alpha
    at 0, 1, at a knot and between knots.  1e-12 relative.  Continuous data
    is decided by the select itself; knots inside ties by the thousand leave
    NaN and are resolved on the sort-based kernel (gpu.resolve_quantile)."""
    import zlib
    from pyabc_amd import gpu
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    N = {"big": 2_000_000, "one_max": 1 << 20, "tiny": 3}.get(case, 200_003)
    pts = rng.gamma(2.0, 1.5, N)
    w = rng.uniform(0.5, 1.5, N)
    if case == "skewed_w":
        w = np.exp(3.0 * rng.standard_normal(N))
    elif case == "heavy_ties":
        pts[rng.uniform(size=N) < 0.3] = 2.5
    elif case == "one_value":
        pts[:] = 1.25
    elif case == "two_spikes":
        pts = np.where(rng.uniform(size=N) < 0.5, 1.0, np.nextafter(1.0, 2.0))
    elif case == "zero_w":
        w[rng.uniform(size=N) < 0.4] = 0.0
    elif case == "dense_core":
        pts = np.where(rng.uniform(size=N) < 0.5, 1.0 + rng.uniform(size=N),
                       1.5 + 1e-4 * rng.uniform(size=N))
    elif case == "crowded":
        pts = 1.0 + 1e-3 * rng.uniform(size=N)
        pts[7], pts[N // 2] = 1e-300, 1e300
    elif case == "discrete":
        pts = rng.integers(0, 40, N).astype(np.float64)
    w = w / w.sum()
    order = np.argsort(pts, kind="stable")
    knot = float(((np.cumsum(w[order]) - 0.5 * w[order]))[N // 3])
    decided = case in ("normal", "skewed_w", "zero_w", "big", "one_max", "dense_core", "tiny")
    P, W = T(pts), T(w)
    for a in (0.0, 0.1, 0.5, knot, 0.9, 1.0):
        raw = float(gpu.weighted_quantile(P, W, a).cpu()[0])
        q = gpu.resolve_quantile(raw, P, W, a)
        ref = oracle.weighted_quantile(pts, w, a, kind="stable")
        assert q == pytest.approx(ref, rel=1e-12, abs=1e-300), (case, a, q, ref)
        if decided:
            assert raw == q, (case, a, raw)
    # deterministic: the same bits twice
    q1 = gpu.weighted_quantile(T(pts), T(w), 0.5).cpu().numpy()
    q2 = gpu.weighted_quantile(T(pts), T(w), 0.5).cpu().numpy()
    assert q1.tobytes() == q2.tobytes()


def test_sort_pairs(dev):
    from pyabc_amd import gpu
    rng = np.random.default_rng(1)
    for n in (1, 7, 2048, 2049, 100_003):
        k = rng.standard_normal(n) * 10 ** rng.uniform(-5, 5, n)
        k[::13] = 0.0
        k[::17] = -0.0 if n > 17 else k[::17]
        k[1::7] = k[::7][:len(k[1::7])]        # ties
        v = np.arange(n, dtype=np.float64)
        ko, vo = gpu.sort_pairs(T(k), T(v))
        order = np.argsort(k, kind="stable")
        np.testing.assert_array_equal(ko.cpu().numpy(), k[order])
        np.testing.assert_array_equal(vo.cpu().numpy(), v[order])


def test_column_stats_golden(dev):
    from pyabc_amd import gpu
    gg = g("adaptive.npz")
    for R in (101, 100):
        data = gg[f"R{R}_std_rNone__data"]
        sd = gpu.column_std(T(data)).cpu().numpy()
        np.testing.assert_allclose(sd, oracle.standard_deviation(data),
                                   rtol=1e-12, atol=1e-15)
        mad = gpu.column_mad(T(data)).cpu().numpy()
        np.testing.assert_array_equal(mad, oracle.median_absolute_deviation(data))


def test_column_mad_large(dev):
    from pyabc_amd import gpu
    rng = np.random.default_rng(2)
    for R, S in ((4097, 3), (20000, 256)):
        X = rng.standard_normal((R, S)) * 10 ** rng.uniform(-2, 2, S)
        X[:, 0] = np.round(X[:, 0])
        mad = gpu.column_mad(T(X)).cpu().numpy()
        np.testing.assert_array_equal(mad, oracle.median_absolute_deviation(X))


def test_column_mad_select_edges(dev):
    """Radix-select MAD: R = 1, 2, 3, constant columns, +-0, sign mixes,
    heavy ties, tiny/huge magnitudes, R across several select levels --
    bit-exact against np.median(|x - np.median(x)|)."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(8)
    cols = []
    for R in (1, 2, 3, 4, 5, 1000, 4096, 65537):
        X = np.empty((R, 9))
        X[:, 0] = 3.25                                  # constant
        X[:, 1] = rng.choice([-0.0, 0.0, 1.0, -1.0], R)  # signed zeros, ties
        X[:, 2] = rng.standard_normal(R)                 # sign mix
        X[:, 3] = np.round(rng.standard_normal(R) * 3)   # heavy ties
        X[:, 4] = rng.standard_normal(R) * 1e-300        # subnormal-ish scale
        X[:, 5] = rng.standard_normal(R) * 1e300
        X[:, 6] = np.exp(rng.standard_normal(R) * 20)    # many exponents
        X[:, 7] = 1.0 + rng.integers(0, 3, R) * 2.0 ** -52  # last-bit ties
        X[:, 8] = -np.abs(rng.standard_normal(R))
        if R >= 8192:
            # sample-bracket misses: huge values exactly at the kernel's
            # sample rows ((2q+1)R / 4096, q < 2048) -> full radix fallback
            X = np.concatenate([X, rng.standard_normal((R, 1))], 1)
            X[(2 * np.arange(2048) + 1) * R // 4096, 9] = 1e9
        mad = gpu.column_mad(T(X)).cpu().numpy()
        np.testing.assert_array_equal(mad, oracle.median_absolute_deviation(X),
                                      err_msg=f"R={R}")


@pytest.mark.parametrize("N,d", [(10_001, 7), (10_001, 10), (1, 10), (300, 1),
                                 (100_000, 3), (77, 20)])
def test_weighted_moments(dev, N, d):
    """np.cov(X, aweights=w) pieces; d in {1..6, 8, 10, 12, 16} run the
    register fast path, others the generic LDS path."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(3)
    X = rng.standard_normal((N, d)) + 5
    w = rng.uniform(size=N)
    sw, sw2, mean, cov_b, wmax = gpu.weighted_moments(T(X), T(w), with_max=True)
    assert wmax == w.max()
    assert sw == pytest.approx(w.sum(), rel=1e-13)
    assert sw2 == pytest.approx((w ** 2).sum(), rel=1e-13)
    np.testing.assert_allclose(mean, w @ X / w.sum(), rtol=1e-13)
    if N > 1:
        cov_ref = np.cov(X, aweights=w, rowvar=False)
        np.testing.assert_allclose(cov_b * sw / (sw - sw2 / sw), cov_ref,
                                   rtol=1e-10, atol=1e-13)
    # bitwise reproducible run to run
    again = gpu.weighted_moments(T(X), T(w))
    assert np.array_equal(again[3], cov_b) and again[0] == sw


def test_scan(dev):
    from pyabc_amd import gpu
    rng = np.random.default_rng(4)
    for n in (1, 5, 2048, 2049, 1_000_001):
        x = rng.uniform(size=n)
        c = gpu.inclusive_scan(T(x)).cpu().numpy()
        np.testing.assert_allclose(c, np.cumsum(x), rtol=1e-12)


def test_propose_replay(dev):
    """Philox draws bit-compatible with the oracle replay; prior re-draws."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(6)
    N, d = 1000, 3
    X = rng.standard_normal((N, d))
    w = rng.uniform(size=N)
    w /= w.sum()
    L = np.linalg.cholesky(np.array([[1, .3, 0], [.3, 1, .2], [0, .2, .5]])) * .4
    kinds = ["uniform", "norm", "expon"]
    params = np.array([[-1.0, 2.0, 0, 0], [0.0, 1.0, 0, 0], [-0.5, 1.0, 0, 0]])
    ref = osamp.propose_mvn(X, w, L, 123, 4, 1000, 5000, kinds, params)
    cdf = gpu.inclusive_scan(T(w))
    th, lp, anc, att = gpu.propose(
        T(X), cdf, T(L),
        T([osamp.KIND[k] for k in kinds], dtype=torch.int32), T(params.ravel()),
        123, 4, 1000, 5000, 1000, d)
    np.testing.assert_array_equal(anc.cpu().numpy(), ref[2])
    # the guide-table search returns the same ancestors (bit-exact draws)
    th_g, lp_g, anc_g, att_g = gpu.propose(
        T(X), cdf, T(L),
        T([osamp.KIND[k] for k in kinds], dtype=torch.int32), T(params.ravel()),
        123, 4, 1000, 5000, 1000, d, guide=gpu.cdf_guide(cdf))
    assert torch.equal(anc_g, anc) and torch.equal(th_g, th)
    np.testing.assert_array_equal(att.cpu().numpy(), ref[3])
    np.testing.assert_allclose(th.cpu().numpy(), ref[0], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(lp.cpu().numpy(), ref[1], rtol=1e-12)
    assert (att.cpu().numpy() > 1).any()     # re-draws happened


def test_prior_sampling_moments(dev):
    """t = 0 draws from the prior itself: moments of every supported kind."""
    from pyabc_amd import gpu
    from scipy import stats
    kinds = ["norm", "uniform", "expon", "laplace", "lognorm", "gamma", "beta"]
    params = np.array([[1, 2, 0, 0], [-1, 3, 0, 0], [0.5, 2, 0, 0],
                       [0, 1, 0, 0], [0.5, 0, 1, 0], [2.5, 0, 1, 0],
                       [2, 3, 0, 1]], dtype=float)
    B = 200_000
    th, lp, _, att = gpu.propose(None, None, None,
                                 T([osamp.KIND[k] for k in kinds], dtype=torch.int32),
                                 T(params.ravel()), 9, 0, 0, B, 10, len(kinds))
    th = th.cpu().numpy()
    dists = [stats.norm(1, 2), stats.uniform(-1, 3), stats.expon(0.5, 2),
             stats.laplace(0, 1), stats.lognorm(0.5, 0, 1), stats.gamma(2.5, 0, 1),
             stats.beta(2, 3, 0, 1)]
    for k, dist in enumerate(dists):
        ks = stats.kstest(th[:, k], dist.cdf).statistic
        assert ks < 0.01, (kinds[k], ks)
    ref_lp = osamp.prior_logpdf(th[:1000], kinds, params)
    np.testing.assert_allclose(lp.cpu().numpy()[:1000], ref_lp, rtol=1e-10)


def test_simulate_replay(dev):
    from pyabc_amd import gpu
    rng = np.random.default_rng(7)
    th = rng.standard_normal((777, 4))
    S = 13
    src = np.arange(S) % 4
    a = rng.uniform(0.5, 2, S)
    sig = 10 ** rng.uniform(-2, 2, S)
    x = gpu.simulate_linear_gaussian(T(th), T(src, dtype=torch.int32), T(a), T(sig),
                                     55, 3, 10).cpu().numpy()
    ref = osamp.simulate_linear_gaussian(th, src, a, sig, 55, 3, 10)
    np.testing.assert_allclose(x, ref, rtol=1e-12, atol=1e-12)


def test_accept_compact(dev):
    from pyabc_amd import gpu
    rng = np.random.default_rng(8)
    for B in (1, 100, 2048, 2049, 300_001):
        dd = rng.uniform(size=B)
        eps = 0.37
        idx, cnt = gpu.accept_compact(T(dd), eps)
        n = int(cnt.cpu())
        ref = np.nonzero(dd <= eps)[0]
        assert n == len(ref)
        np.testing.assert_array_equal(idx.cpu().numpy()[:n], ref)


@pytest.mark.parametrize("S", [3, 10, 32, 33, 100])
def test_pnorm_accept_tail(dev, S):
    """abc_pnorm_accept (the user-simulator accept tail): the first cap
    accepted positions and the count equal abc_pnorm + abc_mask_gave_up +
    abc_accept_compact on the same rows, bit for bit, for p in {1, 2, 3,
    inf}, ragged B, exact eps ties, gave-up proposals and cap < count."""
    import torch
    from pyabc_amd import gpu
    rng = np.random.default_rng(S)
    for B in (1, 2047, 2049, 100_003):
        x = T(rng.normal(size=(B, S)))
        x0 = T(rng.normal(size=S))
        wf = T(rng.uniform(0.2, 2.0, size=S))
        att = torch.as_tensor(np.where(rng.uniform(size=B) < 0.05, 11, 1),
                              dtype=torch.int32, device=x.device)
        for pv in (1.0, 2.0, 3.0, np.inf):
            d = gpu.pnorm(x, x0, wf, pv)
            eps = float(d.cpu().numpy()[B // 2])          # an exact tie
            gpu.mask_gave_up(d, att, 10)
            ref_idx, ref_cnt = gpu.accept_compact(d, eps)
            n = int(ref_cnt.cpu())
            for cap in (B, max(n // 2, 1)):
                idx, cnt = gpu.pnorm_accept(x, x0, wf, pv, eps, cap, att=att, max_attempts=10)
                assert int(cnt.cpu()) == n
                k = min(cap, n)
                np.testing.assert_array_equal(idx.cpu().numpy()[:k], ref_idx.cpu().numpy()[:k])


def test_step_golden(dev):
    """Fixed-input generation step (tests/golden/step.npz): distances,
    accept mask and importance weights against the reference."""
    import pandas as pd
    from pyabc_amd import gpu
    from pyabc_amd.transition import MultivariateNormalTransition
    gg = g("step.npz")
    d = gg["X"].shape[1]
    cols = [f"p{k:02d}" for k in range(d)]
    t = MultivariateNormalTransition()
    t.fit(pd.DataFrame(gg["X"], columns=cols), gg["w"].copy())
    dd = gpu.pnorm(T(gg["xsim"]), T(gg["x0"]), T(np.ones(d)), 2.0)
    np.testing.assert_allclose(dd.cpu().numpy(), gg["d"], rtol=1e-13)
    idx, cnt = gpu.accept_compact(dd, float(gg["eps"]))
    n = int(cnt.cpu())
    acc = np.zeros(len(gg["d"]), bool)
    acc[idx.cpu().numpy()[:n]] = True
    np.testing.assert_array_equal(acc, gg["accept"])
    theta = T(gg["theta"])
    kind = T([0] * d, dtype=torch.int32)
    params = T(np.tile([0.0, 1.0, 0, 0], d))
    lp = gpu.prior_logpdf(theta, kind, params)
    lt = t.logpdf_device(theta)
    wts = gpu.importance_weights(lp, lt).cpu().numpy()
    np.testing.assert_allclose(wts[acc], gg["weight"][acc], rtol=2e-6)


@pytest.mark.parametrize("d,N,M", [(65, 300, 7), (80, 1000, 33), (130, 257, 5)])
def test_wide_moments_and_direct_density(dev, d, N, M):
    """MultivariateNormalTransition above d = 64: abc_weighted_moments' wide
    path vs numpy (sum w, mean, biased covariance, max w: 1e-12) and the
    direct fp64 density kernel vs the oracle's MVN mixture (1e-10), full rank
    and singular (rank d - 5: scipy's support mask)."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(d)
    X = rng.normal(0, 1, (N, d)) * rng.uniform(0.5, 2, d)
    w = rng.uniform(0.1, 1, N)
    sw, sw2, mean, cov_b, wmax = gpu.weighted_moments(T(X), T(w), with_max=True)
    np.testing.assert_allclose([sw, sw2, wmax], [w.sum(), (w ** 2).sum(), w.max()], rtol=1e-12)
    mu = (w[:, None] * X).sum(0) / w.sum()
    np.testing.assert_allclose(mean, mu, rtol=1e-12, atol=1e-14)
    C = ((X - mu).T * w) @ (X - mu) / w.sum()
    np.testing.assert_allclose(cov_b, C, rtol=1e-11, atol=1e-13 * np.abs(C).max())
    wn = w / w.sum()
    x = X[rng.integers(0, N, M)] + 0.3 * rng.normal(0, 1, (M, d))
    for rank in (d, d - 5):
        B = rng.normal(0, 1, (d, rank))
        cov = B @ B.T / rank + (np.eye(d) * 0.5 if rank == d else 0.0)
        from pyabc_amd.transition.multivariatenormal import psd_whitening
        psd = psd_whitening(cov)
        Xs = X if rank == d else mu + (X - mu) @ B @ np.linalg.pinv(B)   # on the subspace
        xs = x if rank == d else mu + (x - mu) @ B @ np.linalg.pinv(B)
        U, V = psd["U"], psd.get("V")
        nv = 0 if V is None or psd["rank"] == d else V.shape[1]
        log_norm = -0.5 * (psd["rank"] * np.log(2 * np.pi) + psd["log_pdet"])
        got = gpu.mvn_logpdf_direct(T(xs), T(Xs), T(wn), T(U),
                                    T(V) if nv else None, psd["tol"], log_norm).cpu().numpy()
        ref = np.log(oracle.mvn_pdf(xs, Xs, wn, cov))
        np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-10)


def test_gather_rows_batch(dev):
    """One-launch gather of several column groups (fp64 matrices, fp64
    vectors, int64 ancestors) == index_select, for ragged sizes."""
    from pyabc_amd import gpu
    g = torch.Generator(device="cpu").manual_seed(3)
    for B, n in ((1, 1), (1000, 0), (4097, 1234), (100_000, 65_537)):
        th = torch.randn(B, 10, dtype=torch.float64, generator=g).to(dev)
        lp = torch.randn(B, dtype=torch.float64, generator=g).to(dev)
        x = torch.randn(B, 3, dtype=torch.float64, generator=g).to(dev)
        anc = torch.randint(0, 1 << 40, (B,), generator=g).to(dev)
        idx = torch.randperm(B, generator=g)[:n].sort().values.to(dev)
        got = gpu.gather_rows_batch([th, lp, x, anc], idx)
        for a, b in zip(got, (th, lp, x, anc)):
            assert a.dtype == b.dtype and a.shape == (n,) + tuple(b.shape[1:])
            assert torch.equal(a, b.index_select(0, idx))


def test_cdf_guide_search_edges(dev):
    """Guide-table ancestor search == searchsorted(side='right') clamped to
    N-1, for weights with zeros, one dominant weight, tiny weights, N = 1."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(12)
    cases = {"n1": np.array([1.0]),
             "zeros": np.where(rng.uniform(size=5000) < 0.5, 0.0, rng.uniform(size=5000)),
             "dominant": np.r_[np.full(3000, 1e-12), [1.0], np.full(3000, 1e-12)],
             "tiny": np.exp(-40 * rng.uniform(size=20000)),
             "uniform": np.ones(70001)}
    d = 2
    for name, w in cases.items():
        N = len(w)
        X = rng.standard_normal((N, d))
        cdf = gpu.inclusive_scan(T(w))
        guide = gpu.cdf_guide(cdf)
        kinds = T([-1, -1], dtype=torch.int32)
        params = T(np.zeros(8))
        L = T(np.eye(d) * 0.1)
        _, _, a0, _ = gpu.propose(T(X), cdf, L, kinds, params, 7, 1, 0, 20000, 1, d)
        _, _, a1, _ = gpu.propose(T(X), cdf, L, kinds, params, 7, 1, 0, 20000, 1, d,
                                  guide=guide)
        assert torch.equal(a0, a1), name
        g = guide.cpu().numpy()
        c = cdf.cpu().numpy()
        t = np.arange(N) * (c[-1] / N)
        np.testing.assert_array_equal(
            g, np.minimum(np.searchsorted(c, t, side="right"), N - 1), err_msg=name)


@pytest.mark.parametrize("d,k,jitter", [(3, 40, 1e-7), (4, 700, 1e-7), (5, 50, 3e-8),
                                         (8, 90, 1e-7), (12, 300, 1e-7), (5, 1500, 0.0)])
def test_local_fit_knn_keys_at_the_fp32_bound(dev, d, k, jitter):
    """The k-NN select sorts on fp32 MFMA keys and settles only the keys
    within its rigorous fp32/fp64 bound in fp64 (abc_local_knn.h kn_bound).
    A jittered integer grid puts thousands of distances within a few fp32
    ulps of one another -- and of the k-th distance -- so the cuts decide
    exactly at the bound's edge (jitter 0: exact ties, taken by index).
    N >= 2048 runs the MFMA select; d = 8 its in-kernel moments (list mode),
    d = 12 three feature blocks; k = 700, 1500 the bin mode."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(d * 1000 + k)
    N = 3000
    X = rng.integers(0, 4, size=(N, d)).astype(float) + jitter * rng.standard_normal((N, d))
    X += 250.0          # far from the origin: the keys are centred first
    w = np.exp(0.3 * rng.standard_normal(N))
    w /= w.sum()
    ref = oracle.local_fit(X, w, k=k, k_fraction=None)
    covs, inv, dets, chol, lnorm = gpu.local_fit(gpu.as_dev(X), gpu.as_dev(w), k, 1.0, 1e-3)
    np.testing.assert_allclose(covs.cpu().numpy(), ref["covs"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(dets.cpu().numpy(), ref["dets"], rtol=1e-8)


@pytest.mark.parametrize("N,d,k,grid", [(12000, 5, 3000, None), (6000, 3, 1500, 5),
                                         (4096, 2, 1024, None)])
def test_local_fit_deferred_collect(dev, N, d, k, grid):
    """Dense k at d <= 5 runs the deferred collect: the count sweep's bracket
    goes to the moments sweep, which queues the open pairs in an order set by
    atomics; the resolve kernel selects among them and sums the queued
    members in index order.  The fit must equal the oracle's and be
    bit-identical between runs (every rank of a multi-GPU run fits the same
    population itself).  The {0..4}^3 grid holds hundreds of exact ties at
    the k-th distance: the queue overflows and the fit falls back to the
    select's own collect sweep."""
    from pyabc_amd import gpu
    rng = np.random.default_rng(N + d + k)
    if grid is None:
        X = rng.normal(size=(N, d))
    else:
        X = rng.integers(0, grid, size=(N, d)).astype(float)
    w = np.exp(0.3 * rng.standard_normal(N))
    w /= w.sum()
    ref = oracle.local_fit(X, w, k=k, k_fraction=None)
    Xd, wd = gpu.as_dev(X), gpu.as_dev(w)
    covs = [gpu.local_fit(Xd, wd, k, 1.0, 1e-3)[0].cpu().numpy() for _ in range(3)]
    np.testing.assert_allclose(covs[0], ref["covs"], rtol=1e-9, atol=1e-12)
    for c in covs[1:]:
        np.testing.assert_array_equal(c, covs[0])
