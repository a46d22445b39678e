"""Diagnostic: hinted-offset statistics of the x3 density kernel on a real
ABC population (how many candidates the lg - o > 20 rule sends to fp64).

    python tools/diag_x3_hint.py [--pop 1000000] [--gens 3] [--M 200000]

Reads the kernel's workspace (offsets, per-chunk partial sums, rescue count)
after one hinted call; layout mirrors plan_x3_ws in abc_mvn_x3.hip.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cdiv(a, b):
    return -(-a // b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=1_000_000)
    ap.add_argument("--gens", type=int, default=3)
    ap.add_argument("--M", type=int, default=200_000)
    a = ap.parse_args()
    import torch
    import bench
    from pyabc_amd import gpu
    sys.argv = [sys.argv[0], "--pop", str(a.pop)]
    args = bench.parse()
    abc, tr = bench.build_abc(args, 0, 1)
    abc.run(max_nr_populations=a.gens)
    t = abc.transitions[0]
    N = t._dev_X.shape[0]
    M = a.M
    th, _, anc, _ = t.propose_device(M)
    out = t.logpdf_device(th, hint=anc)
    torch.cuda.synchronize()
    ws = gpu._ws[(torch.cuda.current_device(), "mvn")].cpu().numpy()
    KB, CT = 3, 8
    MT, NT = cdiv(M, 16), cdiv(N, 16)
    groups = cdiv(cdiv(MT, CT), 4)
    MTpad = groups * 4 * CT
    Mpad = MTpad * 16
    nc = min(max(cdiv(cdiv(NT, 128), 8) * 8, 8), 32)
    off = 0

    def take(n, sz):
        nonlocal off
        start = cdiv(off, 256) * 256
        off = start + n * sz
        return start
    take(MTpad * KB * 64 * 8, 2)
    fl = take(Mpad, 4)
    co = take(Mpad, 4)
    take(nc * Mpad, 8)
    pl = take(nc * Mpad, 8)
    take(Mpad, 8)
    nr = take(64, 4)
    flags = ws[fl:fl + 4 * M].view(np.int32)
    cand_o = ws[co:co + 4 * M].view(np.float32)
    nres = ws[nr:nr + 4].view(np.uint32)[0]
    # part_l was overwritten by the rescue partials for rescued rows; use the
    # combine rule on the surviving ones
    print(f"N={N} M={M} nchunk={nc} rescued={nres} ({nres / M:.2%}) flags={flags.sum()}")
    print("cand_o pct", np.percentile(cand_o, [0, 1, 50, 99, 100]))
    w = t._dev_w.cpu().numpy()
    print("ESS/N", 1 / (w ** 2).sum() / N / (w.sum() ** 2) * w.sum() ** 2)
    lo = out.cpu().numpy()
    print("logpdf pct", np.percentile(lo, [0, 1, 50, 99, 100]))


if __name__ == "__main__":
    main()
