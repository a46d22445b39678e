"""How many x3 tile pairs could be skipped at c3?  Runs the c3 bench workload
(bench.build_abc) for G generations; on the last population it fits the MVN
transition, proposes M candidates (with their ancestors, the hint rows) and
measures, for 16 x 16 (candidate, population row) tiles, the fraction whose
largest log2 term  s_ij - o_i = lw_j - |z_i - y_j|^2 / 2 log2(e) - o_i  lies
below -T (T = 30, 40, 50): such a tile adds < 2^-T per pair to a density
that is >= ~1 at the hinted offset o_i.  Orders compared: as drawn (the
kernel's today) and kd-ordered (population rows by recursive median splits
of the whitened coordinates, candidates by their ancestor's position).
An estimate of tile-pair skipping, not part of the
library.  python tools/probes/x3_tile_skip_probe.py [--gens 22] [--M 65536]
"""
import argparse
import math
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
LOG2E = 1.4426950408889634


def kd_order(Y, leaf=16):
    """Row order of Y by recursive median splits on the widest coordinate."""
    order = np.empty(len(Y), dtype=np.int64)
    out = 0
    stack = [np.arange(len(Y))]
    while stack:
        idx = stack.pop()
        if len(idx) <= leaf:
            order[out:out + len(idx)] = idx
            out += len(idx)
            continue
        P = Y[idx]
        dim = int(np.argmax(P.max(0) - P.min(0)))
        half = len(idx) // 2
        part = np.argpartition(P[:, dim], half)
        stack.append(idx[part[half:]])
        stack.append(idx[part[:half]])
    return order


def tile_fractions(torch, Zc, Yc, lw, o, thresholds, chunk=2048):
    """Fraction of 16 x 16 tiles whose max (lw_j - |z_i - y_j|^2 / 2 log2 e
    - o_i) < -T for each T (rows and candidates in the given order)."""
    M, N = Zc.shape[0], Yc.shape[0]
    nt = N // 16
    Yc, lw = Yc[:nt * 16], lw[:nt * 16]
    yn = (Yc * Yc).sum(1)
    counts = np.zeros(len(thresholds), dtype=np.int64)
    total = 0
    for a in range(0, M - M % 16, chunk):
        z = Zc[a:a + chunk]
        zn = (z * z).sum(1)
        d2 = (zn[:, None] + yn[None, :] - 2.0 * (z @ Yc.T)).clamp_min_(0.0)
        s = lw[None, :] - 0.5 * LOG2E * d2 - o[a:a + chunk, None]
        tm = s.view(z.shape[0] // 16, 16, nt, 16).amax(dim=(1, 3))
        for q, T in enumerate(thresholds):
            counts[q] += int((tm < -T).sum())
        total += tm.numel()
    return counts / total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", type=int, default=22)
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--pop", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch
    import bench
    import pandas as pd
    from pyabc_amd.transition import MultivariateNormalTransition
    args = types.SimpleNamespace(dim=10, precision="x3", pop=a.pop, filter_below=None)
    abc, _ = bench.build_abc(args, 0, 1)
    abc.run(max_nr_populations=a.gens)
    t = abc.history.max_t
    cols = abc.history.get_population_device(t)
    X = cols.theta.double()
    w = cols.weights.double()
    w = w / w.sum()
    names = list(cols.param_names)
    tr = MultivariateNormalTransition()
    tr.fit(pd.DataFrame(X.cpu().numpy(), columns=names), w.cpu().numpy().copy())
    th, _, anc, _ = tr.propose_device(a.M)
    cov = np.asarray(tr.cov)
    ev, V = np.linalg.eigh(cov)
    U = V / np.sqrt(ev)                      # (x - mu) U: kernel-whitened
    Ut = torch.as_tensor(U, device=X.device)
    mu = X.mean(0)
    Y = ((X - mu) @ Ut).float()
    Z = ((th.double() - mu) @ Ut).float()
    lw = torch.log2(w).float()
    anc = anc.long()
    dz = Z - Y[anc]
    o = torch.ceil(lw[anc] - 0.5 * LOG2E * (dz * dz).sum(1))
    ths = [30, 40, 50]
    ess = 1.0 / float((w * w).sum())
    print(f"t={t} N={X.shape[0]} ESS={ess:.4g} M={a.M}", flush=True)
    f0 = tile_fractions(torch, Z, Y, lw, o, ths)
    print("as drawn   : " + ", ".join(f"<-{T}: {f:.4f}" for T, f in zip(ths, f0)), flush=True)
    perm = kd_order(Y.cpu().numpy().astype(np.float64))
    pos = np.empty_like(perm)
    pos[perm] = np.arange(len(perm))
    cperm = np.argsort(pos[anc.cpu().numpy()], kind="stable")
    P = torch.as_tensor(perm, device=X.device)
    C = torch.as_tensor(cperm, device=X.device)
    f1 = tile_fractions(torch, Z[C], Y[P], lw[P], o[C], ths)
    print("kd-ordered : " + ", ".join(f"<-{T}: {f:.4f}" for T, f in zip(ths, f1)), flush=True)


if __name__ == "__main__":
    main()
