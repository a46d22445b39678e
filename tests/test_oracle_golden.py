"""Pin the CPU oracle: reference known-answer tests + golden vectors.

The known answers are the ones pyABC's own tests hold:
test_weighted_statistics.py:10-39, test_epsilon.py:25-47,
test_distance_function.py:80-96 and :137-155.  The golden vectors were made
by importing the reference (tests/golden/make_golden.py).
"""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN


def load(name):
    return np.load(os.path.join(GOLDEN, name))


# ---- reference known-answer tests, restated -----------------------------

def test_kat_weighted_quantile():
    # test_weighted_statistics.py:10-39
    pts = np.array([1, 2, 3, 4.])
    w = np.array([.25, .25, .25, .25])
    assert oracle.weighted_quantile(pts, w, alpha=.5) == 2.5
    w = np.array([.1, .2, .3, .4])
    assert 3 <= oracle.weighted_quantile(pts, w, alpha=.5) <= 4
    assert oracle.weighted_quantile(pts, np.array([.1, .2, .3, .4]), 1) == 4
    assert oracle.weighted_quantile(pts, None, 0.2) == 1.3


def test_kat_quantile_epsilon():
    # test_epsilon.py:25-47: unweighted median of [1,2,3,4] * 1.1
    e = oracle.quantile_epsilon([1, 2, 3, 4], [1, 1, 1, 1], alpha=.5,
                                multiplier=1.1, weighted=False)
    assert e == pytest.approx(2.5 * 1.1)
    e = oracle.quantile_epsilon([1, 2, 3, 4], [.1, .2, .3, .4], alpha=.9)
    assert 3 <= e <= 4


def test_kat_pnorm():
    # test_distance_function.py:80-96: |(1,2)|_2 weighted -> sqrt(5)
    d = oracle.pnorm([[1, 2]], [0, 0], w=[1, 1], p=2)
    assert d[0] == pytest.approx(np.sqrt(5))
    # test_distance_function.py:137-155: initial weights (1, 2) -> sqrt(2^2+6^2)
    d = oracle.pnorm([[2, 3]], [0, 0], w=[1, 2], p=2)
    assert d[0] == pytest.approx(np.sqrt(2 ** 2 + 6 ** 2))


# ---- golden vectors from the imported reference --------------------------

MVN = ["d1_n1000", "d2_n500", "d10_n4096", "d3_unnorm_scaled", "singular",
       "n1"]


@pytest.mark.parametrize("tag", MVN)
def test_mvn_fit_and_pdf(tag):
    g = load(f"mvn_{tag}.npz")
    cov, wn = oracle.mvn_fit(g["X"], g["w"], scaling=float(g["scaling"]))
    np.testing.assert_allclose(cov, g["cov"], rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(wn, g["w_fit"], rtol=1e-13)
    pdf = oracle.mvn_pdf(g["x"], g["X"], wn, cov)
    np.testing.assert_allclose(pdf, g["pdf"], rtol=1e-9, atol=0)


@pytest.mark.parametrize("tag", ["k50", "default"])
def test_local_fit_and_pdf(tag):
    g = load(f"local_{tag}.npz")
    kw = dict(k=50, k_fraction=None) if tag == "k50" else {}
    fit = oracle.local_fit(g["X"], g["w"], **kw)
    assert fit["k"] == int(g["k"])
    np.testing.assert_allclose(fit["covs"], g["covs"], rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(fit["dets"], g["dets"], rtol=1e-8)
    pdf = oracle.local_pdf(g["x"], g["X"], fit)
    np.testing.assert_allclose(pdf, g["pdf"], rtol=1e-9)


@pytest.mark.parametrize("d", [3, 20, 80])
def test_local_fit_degenerate_weights(d):
    """Neighbourhoods whose weights make np.cov's 1 - sum a^2 exactly 0 (one
    neighbour carries all the weight) or whose weights are all 0: the
    reference's covariances (tests/golden/local_degenerate.npz, made by
    importing pyABC) are non-finite exactly there and its det loop exits on
    the NaN determinant; the oracle gives the same non-finite set and the
    finite covariances to 1e-9 relative."""
    g = load("local_degenerate.npz")
    with np.errstate(all="ignore"):
        fit = oracle.local_fit(g[f"X{d}"], g[f"w{d}"], k=int(g[f"k{d}"]), k_fraction=None)
    ref = g[f"covs{d}"]
    fin = np.isfinite(ref).all(axis=(1, 2))
    assert 0 < fin.sum() < len(fin)
    np.testing.assert_array_equal(np.isfinite(fit["covs"]).all(axis=(1, 2)), fin)
    np.testing.assert_allclose(fit["covs"][fin], ref[fin], rtol=1e-9, atol=1e-13)


def test_pnorm_golden():
    g = load("pnorm.npz")
    cases = sorted({k.split("__")[0] for k in g.files})
    assert len(cases) == 9
    for c in cases:
        d = oracle.pnorm(g[c + "__x"], g[c + "__x0"], g[c + "__w"],
                         g[c + "__f"], float(g[c + "__p"]))
        np.testing.assert_allclose(d, g[c + "__d"], rtol=1e-12, err_msg=c)


def test_adaptive_golden():
    g = load("adaptive.npz")
    tags = sorted({k.split("__")[0] for k in g.files})
    assert len(tags) == 8
    for t in tags:
        sf = "std" if "_std_" in t else "mad"
        ratio = float(g[t + "__ratio"])
        w = oracle.adaptive_weights(g[t + "__data"], sf,
                                    max_weight_ratio=None if np.isnan(ratio)
                                    else ratio)
        np.testing.assert_allclose(w, g[t + "__w"], rtol=1e-12, err_msg=t)


def test_quantile_golden():
    g = load("quantile.npz")
    for name in ("n10k", "ties", "zerow", "n1"):
        pts, w = g[f"{name}__points"], g[f"{name}__w"]
        for a in (0.2, 0.5, 0.9, 1.0):
            q = oracle.weighted_quantile(pts, w, a)
            assert q == pytest.approx(float(g[f"{name}__a{a}__q"]),
                                      rel=1e-13), (name, a)
        for weighted in (True, False):
            e = oracle.quantile_epsilon(pts, w * 2.0, 0.3, 1.1, weighted)
            assert e == pytest.approx(float(g[f"{name}__eps_w{int(weighted)}"]),
                                      rel=1e-13)


def test_step_golden():
    g = load("step.npz")
    cov, wn = oracle.mvn_fit(g["X"], g["w"])
    tp = oracle.mvn_pdf(g["theta"], g["X"], wn, cov)
    np.testing.assert_allclose(tp, g["trans_pd"], rtol=1e-10)
    d = oracle.pnorm(g["xsim"], g["x0"], p=2)
    np.testing.assert_allclose(d, g["d"], rtol=1e-13)
    acc = d <= float(g["eps"])
    np.testing.assert_array_equal(acc, g["accept"])
    from scipy.stats import norm
    prior = norm.pdf(g["theta"]).prod(1)
    np.testing.assert_allclose(prior, g["prior_pd"], rtol=1e-13)
    wt = np.where(acc, oracle.importance_weights(prior, tp), 0.0)
    np.testing.assert_allclose(wt, g["weight"], rtol=1e-10)


def test_philox_known_answer():
    # Random123 KAT: philox4x32_10(ctr=0, key=0)
    r = oracle.philox4x32_10(np.zeros(1, np.uint64), 0, 0, 0)[0]
    assert [int(v) for v in r] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c,
                                   0x9b00dbd8]


def test_box_muller_replay_accuracy_and_tail():
    """oracle.normal_pairs -- the bit-for-bit replay of the device transform
    (abc_common.h box_muller; tests/test_gpu_fused.py pins device == oracle)
    -- is within 4 fp32 ulp of R of a long-double R cos / R sin on 2M random
    words plus the edges (u1 = 2^-41, the 41-bit u1 below 2^-23 and the
    32-bit one above, u1 next to the series branch at 1 - 2^-8, u1 -> 1),
    and its largest radius is sqrt(-2 ln 2^-41) = 7.54: P(R > 7.54) =
    2^-41 (32 bits alone: 6.66, 2^-32)."""
    rng = np.random.default_rng(3)
    a = rng.integers(0, 2 ** 32, 1 << 21, dtype=np.uint64)
    b = rng.integers(0, 2 ** 32, 1 << 21, dtype=np.uint64)
    edge = np.array([0, 1, 2, 3, 511, 512, 513, 2 ** 24 - 1, 2 ** 32 - 2 ** 24 - 1,
                     2 ** 32 - 2 ** 24, 2 ** 32 - 2 ** 24 + 1, 2 ** 32 - 3, 2 ** 32 - 1],
                    dtype=np.uint64)
    a = np.concatenate([edge, a])
    eb = rng.integers(0, 2 ** 32, len(edge), dtype=np.uint64)
    eb[0] &= np.uint64(0xFFFFFE00)          # a = 0 with b's 9 low bits 0: u1 = 2^-41
    b = np.concatenate([eb, b])
    n0, n1 = oracle.normal_pairs(a.astype(np.uint32), b.astype(np.uint32))
    ld = np.longdouble
    ext = a < np.uint64(512)
    u1 = np.where(ext, ((a << np.uint64(9)) | (b & np.uint64(511)) | np.uint64(1)).astype(ld)
                  * ld(2.0) ** -41, (a | np.uint64(1)).astype(ld) * ld(2.0) ** -32)
    m2 = ((b >> np.uint64(9)) * 2 + 1).astype(ld)
    R = np.sqrt(-2 * np.log(u1))
    ang = ld("3.14159265358979323846264338327950288") * m2 * ld(2.0) ** -23
    for got, ex in ((n0, R * np.cos(ang)), (n1, R * np.sin(ang))):
        ulp = np.abs(got - ex.astype(np.float64)) / \
            np.spacing(R.astype(np.float32)).astype(np.float64)
        assert ulp.max() <= 4, ulp.max()
    r0 = float(np.hypot(n0[0], n1[0]))
    assert abs(r0 - np.sqrt(82 * np.log(2))) < 1e-5 and r0 > 7.53
    # the 32-bit branch above 2^-23 is unchanged: a = 512 is its smallest u1
    r512 = float(np.hypot(n0[5], n1[5]))
    assert abs(r512 - np.sqrt(-2 * np.log(513 * 2.0 ** -32))) < 1e-5


# ---- bootstrapped KDE CV (cv/bootstrap.py, golden from the reference) -----

def test_cv_fixed_samples_golden():
    g = load("cv.npz")
    dens = oracle.mvn_bootstrap_densities(g["samples"], g["X"])
    np.testing.assert_allclose(dens, g["dens"], rtol=1e-11)
    var, cv = oracle.bootstrap_variation(dens, g["w"])
    np.testing.assert_allclose(var, g["variation"], rtol=1e-9)
    assert cv == pytest.approx(float(g["cv_fixed"]), rel=1e-10)


def test_cv_statistics_match_reference():
    # the reference's calc_cv over 24 seeds at n = 100, 400 (numpy RNG);
    # the restatement with an independent RNG must agree in distribution
    g = load("cv.npz")
    rng = np.random.default_rng(5)
    for i, n in enumerate(g["stat_n"]):
        ref = g["cvs"][i]
        ours = np.array([oracle.mvn_calc_cv(int(n), g["X"], g["w"], 10, rng)
                         for _ in range(12)])
        se = np.hypot(ref.std() / np.sqrt(len(ref)),
                      ours.std() / np.sqrt(len(ours)))
        assert abs(ours.mean() - ref.mean()) < 4 * se, (n, ours.mean(), ref.mean())
