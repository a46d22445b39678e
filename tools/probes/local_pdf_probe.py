"""LocalTransition density at the c5 shape (1e5 candidates x 1e5 particles,
d = 5; the population of tools/bench_components.py's c5 line, k = 50), for
kernel traces, PMC passes and same-box A/Bs of local_mfma_kernel (library
from ABCGPU_LIB, default in-tree).

    python tools/probes/local_pdf_probe.py [--reps 5]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import pandas as pd
    import torch
    from pyabc_amd.transition import LocalTransition
    rng = np.random.default_rng(99)
    N, d = 100_000, 5
    comp = rng.integers(0, 2, N)
    A = rng.standard_normal((d, d)) * 0.3 + np.eye(d)
    X = rng.standard_normal((N, d)) @ A.T + np.where(comp[:, None] == 1, 2.0, -1.0)
    w = np.exp(0.5 * rng.standard_normal(N))
    w /= w.sum()
    t = LocalTransition(k=50, k_fraction=None)
    t.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(d)]), w.copy())
    x = t.propose_device(N)[0]
    out = t.logpdf_device(x)
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = t.logpdf_device(x)
        torch.cuda.synchronize()
        ms.append(1e3 * (time.perf_counter() - t0))
    v = out.cpu().numpy()
    print(f"local pdf ms {[round(m, 3) for m in ms]} min {min(ms):.3f}; "
          f"checksum {float(np.sum(v[np.isfinite(v)])):.9e} finite {int(np.isfinite(v).sum())}")


if __name__ == "__main__":
    main()
