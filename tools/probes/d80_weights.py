"""Diagnose test_local_transition_d80_generations on a given build (probe):
the worst rows of err / first-order bound at each generation, and for the
worst row the particles carrying its density, with the device fit's and
the oracle's covariance determinant and regularisation for each.
    ABCGPU_LIB=... python tools/probes/d80_weights.py"""
import os
import sys

import numpy as np
import pandas as pd
from scipy import stats

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
from test_gpu_fallbacks import _local_weight_bound  # noqa: E402


def main():
    import pyabc_amd as pa
    d = 80
    names = [f"p{q:02d}" for q in range(d)]
    keys = [f"y{q:02d}" for q in range(d)]
    model = pa.LinearGaussianModel(names, keys, src=list(range(d)), sigma=[0.5] * d)
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    abc = pa.ABCSMC(model, prior, pa.PNormDistance(p=2), population_size=600,
                    transitions=pa.LocalTransition(k=100, k_fraction=None),
                    sampler=pa.BatchedGPUSampler(seed=13),
                    eps=pa.QuantileEpsilon(alpha=0.5))
    abc.new("sqlite://", {k: 0.3 for k in keys})
    h = abc.run(max_nr_populations=3)
    for t in range(1, h.max_t + 1):
        dfp, wp = h.get_distribution(0, t - 1)
        df, w = h.get_distribution(0, t)
        Xp, x = dfp[names].to_numpy(), df[names].to_numpy()
        fit = oracle.local_fit(Xp, wp, k=100, k_fraction=None)
        lw = stats.norm.logpdf(x).sum(1) - np.log(oracle.local_pdf(x, Xp, fit))
        ref = lw - lw.max()
        ref -= np.log(np.exp(ref).sum())
        bound = _local_weight_bound(x, Xp, fit, np.exp(ref))
        got = np.log(w)
        err = np.abs(got - ref)
        ratio = err / bound
        order = np.argsort(-ratio)[:3]
        print(f"t={t}: worst rows {order.tolist()} ratio {ratio[order].round(2).tolist()} "
              f"err {err[order].tolist()} bound {bound[order].tolist()}")
        # the device fit of the same population
        lt = pa.LocalTransition(k=100, k_fraction=None)
        lt.fit(pd.DataFrame(Xp, columns=names), wp)
        dcov = lt.covs
        ddet = lt._dev_dets.cpu().numpy() if hasattr(lt, "_dev_dets") else None
        cov_rel = np.abs(dcov - fit["covs"]).max(axis=(1, 2)) / np.abs(fit["covs"]).max(axis=(1, 2))
        odet = np.linalg.slogdet(fit["covs"])
        print(f"  fit: max cov rel diff {cov_rel.max():.2e} (particle {int(cov_rel.argmax())}); "
              f"oracle cond max {np.linalg.cond(fit['covs']).max():.2e}")
        i = int(order[0])
        dl = Xp - x[i]
        v = np.einsum("jab,jb->ja", fit["inv_covs"], dl)
        q = np.einsum("ja,ja->j", dl, v)
        lt_ = np.log(fit["w"]) - 0.5 * q - np.log(fit["normalization"])
        r = np.exp(lt_ - lt_.max())
        r /= r.sum()
        top = np.argsort(-r)[:5]
        for j in top:
            c = np.linalg.cond(fit["covs"][j])
            dd = ddet[j] if ddet is not None else float("nan")
            print(f"   row {i}: particle {int(j)} share {r[j]:.3e} cond {c:.2e} "
                  f"logdet oracle {odet[1][j]:.6f} sign {odet[0][j]:.0f} device det {dd!r} "
                  f"cov rel diff {cov_rel[j]:.2e}")


if __name__ == "__main__":
    main()
