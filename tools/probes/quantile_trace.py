"""Per-block stage timeline of the one-launch weighted quantile (probe; needs
a library built from a stamped abc_quantile.hip variant exporting
abc_probe_trace / abc_probe_trace_reset, e.g. ABCGPU_LIB=ab/libq_trace.so).
Stamps: 0 start, 1 loaded + reduced, 2 past hand-off 1, 3 level 1 flushed,
4 arrived (last: picked), 5 past hand-off 2, 6 level 2 flushed, 7 arrived,
8 past hand-off 3, 9 gathered, 10 last block in, 11 final done.

    ABCGPU_LIB=ab/libq_trace.so python tools/probes/quantile_trace.py [--N 1000000]
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
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from pyabc_amd import gpu, _native
    gpu.require_device()
    lib = _native.load()
    d = torch.rand(a.N, dtype=torch.float64, device="cuda") * 4 + 1
    w = torch.rand(a.N, dtype=torch.float64, device="cuda")
    nb = min(256, -(-a.N // 4096))
    for rep in range(a.reps):
        assert lib.abc_probe_trace_reset(nb) == 0
        torch.cuda.synchronize()
        gpu.weighted_quantile(d, w, 0.5)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (12 * nb))()
        assert lib.abc_probe_trace(buf, nb) == 0
        tr = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 12).astype(np.int64)
        t0 = tr[:, 0].min()
        rel = np.where(tr > 0, (tr - t0) / 100.0, np.nan)   # us (100 MHz)
        line = []
        for k in range(12):
            col = rel[:, k]
            col = col[~np.isnan(col)]
            if len(col):
                line.append(f"{k}:{col.min():.1f}/{np.median(col):.1f}/{col.max():.1f}")
        print(f"N={a.N} nb={nb} rep {rep}: stamp min/median/max us  " + "  ".join(line))


if __name__ == "__main__":
    main()
