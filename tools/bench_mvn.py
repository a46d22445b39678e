"""Micro-benchmark of the transition-density kernels at the c2 shape.

    python tools/bench_mvn.py [--N 100000] [--M 100000] [--d 10] [--reps 5]

Times the GEMM launch with libabcgpu's HIP-event profile hooks (same
numbers as bench.py's roofline) and checks x3 against the f64-MFMA kernel.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=100_000)
    ap.add_argument("--M", type=int, default=100_000)
    ap.add_argument("--d", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--prec", default="x3,x3+hint,f64")
    a = ap.parse_args()
    import pandas as pd
    import torch
    from pyabc_amd import gpu, _native as nat
    from pyabc_amd.transition import MultivariateNormalTransition
    rng = np.random.default_rng(5)
    X = 0.8 + np.sqrt(0.2) * rng.standard_normal((a.N, a.d))
    w = np.exp(0.5 * rng.standard_normal(a.N))
    w /= w.sum()
    cols = [f"p{k}" for k in range(a.d)]
    res = {}
    cand = None
    for prec in a.prec.split(","):
        hinted = prec.endswith("+hint")
        prec = prec.replace("+hint", "")
        t = MultivariateNormalTransition(precision=prec)
        t.fit(pd.DataFrame(X, columns=cols), w.copy())
        if cand is None:
            cand, _, anc, _ = t.propose_device(a.M)
        hint = anc if hinted else None
        if hinted:
            prec += "+hint"
        t.logpdf_device(cand, hint=hint)
        torch.cuda.synchronize()
        nat.call("abc_profile_begin")
        t0 = time.perf_counter()
        for _ in range(a.reps):
            out = t.logpdf_device(cand, hint=hint)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.reps
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        nat.call("abc_profile_end", ctypes.addressof(ms), ctypes.addressof(n))
        kms = ms.value / max(n.value, 1)
        pairs = a.M * a.N
        res[prec] = out.cpu().numpy()
        print(f"{prec}: kernel {kms:.3f} ms  call {1e3 * wall:.3f} ms  "
              f"{pairs / kms / 1e9:.3e} Gpairs/s  "
              f"{2 * a.d * pairs / kms / 1e9:.1f} TFLOP/s(2d/pair)", flush=True)
    for k in ("x3", "x3+hint"):
        if k in res and "f64" in res:
            err = np.abs(np.expm1(res[k] - res["f64"]))
            print(f"{k} vs f64: max rel {err.max():.3e}  mean {err.mean():.3e}")


if __name__ == "__main__":
    main()
