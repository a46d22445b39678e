"""Per-block timeline of the LocalTransition density (local_mfma_kernel) at
c5's shape (probe; needs a library built from a block-stamped abc_local.hip
exporting abc_probe_trace / abc_probe_trace_reset, e.g.
ABCGPU_LIB=ab/liblocal_trace.so): busy blocks over the launch, per-XCC
block counts and ends, block durations.

    ABCGPU_LIB=ab/liblocal_trace.py python tools/probes/local_trace.py
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import pandas as pd
    import torch
    from pyabc_amd import _native
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
    lib = _native.load()
    nmax = 100000
    for _ in range(3):
        assert lib.abc_probe_trace_reset(nmax) == 0
        torch.cuda.synchronize()
        t.logpdf_device(x)
        torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (3 * nmax))()
    assert lib.abc_probe_trace(buf, nmax) == 0
    tr = np.frombuffer(buf, dtype=np.uint64).reshape(nmax, 3)
    tr = tr[tr[:, 1] > 0]
    st, en = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    xcc = (tr[:, 2] >> 32).astype(np.int64)
    t0 = st.min()
    st, en = (st - t0) / 1e2, (en - t0) / 1e2          # us (100 MHz clock)
    dur = en - st
    span = en.max()
    print(f"blocks={len(st)} span {span:.1f} us; block duration median {np.median(dur):.1f} "
          f"p10 {np.percentile(dur, 10):.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f} us")
    grid = np.linspace(0, span, 41)
    busy = [int(((st <= g) & (en > g)).sum()) for g in grid]
    print("busy blocks over the launch:", busy)
    for q in range(int(xcc.max()) + 1):
        m = xcc == q
        if m.any():
            print(f"  xcc {q}: blocks {int(m.sum())}, median {np.median(dur[m]):.1f} us, "
                  f"last end {en[m].max():.1f} us")
    order = np.argsort(st)
    print("start times of blocks by launch rank (every 256th):",
          [round(float(st[order[i]]), 1) for i in range(0, len(st), 256)])
    full = max(busy)
    work = dur.sum()
    print(f"work {work:.0f} block-us; at {full} busy blocks the ideal span {work / full:.1f} us")


if __name__ == "__main__":
    main()
