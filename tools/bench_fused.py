"""Micro-benchmark of the fused candidate round (abc_candidates_round) on a
c3-shaped generation: population 1e6 x 10 ~ the conjugate posterior
N(0.8, 0.2 I), MVN kernel with the Silverman bandwidth at ESS 2e4,
LinearGaussian y = theta + 0.5 e, PNorm p = 2, x0 = 1; eps set for a target
acceptance rate.  Prints candidates/s for the plain and early-reject modes
(HIP events on the launch stream) and the staged pipeline for comparison.

    python tools/bench_fused.py [--rates 1e-2 1e-4] [--B 268435456]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", type=float, nargs="+", default=[1e-2, 1e-4])
    ap.add_argument("--B", type=int, default=1 << 28)
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=10)
    ap.add_argument("--S", type=int, default=None, help="statistics (default d)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--wsigma", type=float, default=0.0,
                    help="lognormal importance weights, ESS/N = exp(-wsigma^2) "
                         "(c3's last generations: ~1e-2)")
    ap.add_argument("--chain", type=int, default=1,
                    help="rounds queued back to back per timed repetition (the "
                         "per-round time is their mean: no host gap or clock "
                         "ramp between rounds)")
    ap.add_argument("--staged", action="store_true")
    ap.add_argument("--sort-weights", action="store_true",
                    help="population rows in descending weight order (probe of a "
                         "weight-sorted ancestor table: the heavy rows' records "
                         "and guide bins contiguous)")
    ap.add_argument("--modes", nargs="+", default=["plain", "filter"],
                    choices=["plain", "filter"])
    a = ap.parse_args()
    import torch
    from pyabc_amd import gpu
    dev = gpu.require_device()
    d, N = a.d, a.N
    S = a.S or a.d
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.8 + np.sqrt(0.2) * torch.randn(N, d, generator=g, dtype=torch.float64)).to(dev)
    w = torch.exp(a.wsigma * torch.randn(N, generator=g, dtype=torch.float64)).to(dev)
    w /= w.sum()
    if a.sort_weights:
        order = torch.argsort(w, descending=True, stable=True)
        X, w = X[order].contiguous(), w[order].contiguous()
    bw = (4 / (2e4 * (d + 2))) ** (1 / (d + 4))
    L = torch.eye(d, dtype=torch.float64, device=dev) * (bw * np.sqrt(0.2))
    cdf = gpu.inclusive_scan(w)
    guide = gpu.cdf_guide(cdf)
    kind = torch.zeros(d, dtype=torch.int32, device=dev)
    params = torch.tensor(np.tile([0.0, 1.0, 0, 0], d), dtype=torch.float64, device=dev)
    src = torch.arange(S, dtype=torch.int32, device=dev) % d
    one = torch.ones(S, dtype=torch.float64, device=dev)
    half = torch.full((S,), 0.5, dtype=torch.float64, device=dev)
    fr = gpu.CandidateRound(d, S, kind, params, src, one, half, one.clone(), one.clone(),
                            2.0, 7, 5, 10000, X=X, cdf=cdf, guide=guide, L=L)
    # distances of a probe batch -> eps per target rate
    probe = 1 << 22
    th, lp, anc, att = gpu.propose(X, cdf, L, kind, params, 7, 5, 0, probe, 10000, d,
                                   guide=guide)
    x = gpu.simulate_linear_gaussian(th, src, one, half, 7, 5, 0)
    dist = gpu.pnorm(x, one, one, 2.0).cpu().numpy()
    for rate in a.rates:
        eps = float(np.quantile(dist, rate))
        for filt in [m == "filter" for m in a.modes]:
            ts = []
            for r in range(a.reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for q in range(a.chain):
                    idx, cnt = fr.run((r * a.chain + q) * a.B, a.B, eps, cap=1 << 20,
                                      filter=filt)
                e1.record()
                e1.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1) / a.chain)
            c = int(cnt.cpu())
            ms = float(np.median(ts))
            print(f"rate {rate:g} eps {eps:.4f} filter={filt}: B={a.B} {ms:.2f} ms "
                  f"-> {a.B / ms * 1e3:.3e} candidates/s (accepted {c}, "
                  f"{c / a.B:.2e})", flush=True)
        if a.staged:
            B = 1 << 22
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for r in range(2):
                e0.record()
                th, lp, anc, att = gpu.propose(X, cdf, L, kind, params, 7, 5, 0, B, 10000, d,
                                               guide=guide)
                x = gpu.simulate_linear_gaussian(th, src, one, half, 7, 5, 0)
                dd = gpu.pnorm(x, one, one, 2.0)
                idx, cnt = gpu.accept_compact(dd, eps)
                e1.record()
                e1.synchronize()
            ms = e0.elapsed_time(e1)
            print(f"  staged 4-kernel pipeline: B={B} {ms:.2f} ms -> "
                  f"{B / ms * 1e3:.3e} candidates/s", flush=True)


if __name__ == "__main__":
    main()
