"""Per-block timeline of the hinted x3 density launch at c3's shape (probe;
needs a library built from a block-stamped abc_mvn_x3.hip variant exporting
abc_probe_trace / abc_probe_trace_reset, e.g. ABCGPU_LIB=ab/libx3_trace.so):
per-XCC block counts, median block times and last block ends.

    ABCGPU_LIB=ab/libx3_trace.so python tools/probes/x3_trace.py [--N 1000000]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--M", type=int, default=None)
    ap.add_argument("--d", type=int, default=10)
    a = ap.parse_args()
    import pandas as pd
    import torch
    from pyabc_amd import gpu, _native
    from pyabc_amd.transition import MultivariateNormalTransition
    gpu.require_device()
    M = a.M or a.N
    rng = np.random.default_rng(5)
    X = 0.8 + np.sqrt(0.2) * rng.standard_normal((a.N, a.d))
    w = np.exp(2.2 * rng.standard_normal(a.N))
    w /= w.sum()
    t = MultivariateNormalTransition()
    t.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(a.d)]), w)
    cand, _, anc, _ = t.propose_device(M)
    lib = _native.load()
    nmax = 100000
    for rep in range(3):
        assert lib.abc_probe_trace_reset(nmax) == 0
        torch.cuda.synchronize()
        t.logpdf_device(cand, hint=anc)
        torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (3 * nmax))()
    assert lib.abc_probe_trace(buf, nmax) == 0
    tr = np.frombuffer(buf, dtype=np.uint64).reshape(nmax, 3)
    used = tr[:, 1] > 0
    tr = tr[used]
    st, en = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    xcc = (tr[:, 2] >> 32).astype(np.int64)
    t0 = st.min()
    st, en = (st - t0) / 1e5, (en - t0) / 1e5          # ms (100 MHz clock)
    dur = en - st
    span = en.max()
    print(f"N={a.N} M={M} blocks={len(st)} span {span:.2f} ms; block median {np.median(dur) * 1e3:.1f} us "
          f"p10 {np.percentile(dur, 10) * 1e3:.1f} p90 {np.percentile(dur, 90) * 1e3:.1f}")
    ends = []
    for x in range(int(xcc.max()) + 1):
        m = xcc == x
        if m.any():
            ends.append(en[m].max())
            print(f"  xcc {x}: blocks {int(m.sum())}, median block {np.median(dur[m]) * 1e3:.1f} us, "
                  f"last end {en[m].max():.2f} ms")
    ends = np.array(ends)
    print(f"XCC last-end spread: {ends.min():.2f} .. {ends.max():.2f} ms "
          f"(mean {ends.mean():.2f}; the launch waits {span - ends.mean():.2f} ms for the slowest)")
    grid = np.linspace(0, span, 41)
    busy = [int(((st <= x) & (en > x)).sum()) for x in grid]
    print("busy blocks over the launch:", busy)


if __name__ == "__main__":
    main()
