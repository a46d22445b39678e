"""Per-block timeline of one fused candidate round (probe; needs a library
built from a traced abc_fused.hip variant exporting abc_probe_trace, e.g.
ABCGPU_LIB=ab/libfr_trace.so): block start / end wall clocks (100 MHz), CU
and XCC ids -> busy-block profile over the launch, per-XCC finish times,
ramp and tail.

    ABCGPU_LIB=ab/libfr_trace.so python tools/probes/round_trace.py --B 33554432
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1 << 25)
    ap.add_argument("--wsigma", type=float, default=2.2)
    a = ap.parse_args()
    import torch
    from pyabc_amd import gpu, _native
    dev = gpu.require_device()
    d = S = 10
    N = 1_000_000
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.8 + np.sqrt(0.2) * torch.randn(N, d, generator=g, dtype=torch.float64)).to(dev)
    w = torch.exp(a.wsigma * torch.randn(N, generator=g, dtype=torch.float64)).to(dev)
    w /= w.sum()
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
    eps = 0.6841
    for r in range(3):
        idx, cnt = fr.run(r * a.B, a.B, eps, cap=1 << 20, filter=False)
    torch.cuda.synchronize()
    nb = (a.B + 2047) // 2048
    n = min(nb, 200000)
    buf = (ctypes.c_ulonglong * (3 * n))()
    lib = _native.load()
    assert lib.abc_probe_trace(buf, n) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(n, 3)
    st, en = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    cu = (t[:, 2] & 0xFFFFFFFF).astype(np.int64)
    xcc = (t[:, 2] >> 32).astype(np.int64)
    t0 = st.min()
    st, en = (st - t0) * 10 / 1e3, (en - t0) * 10 / 1e3     # us
    span = en.max()
    dur = en - st
    print(f"B={a.B} blocks={n} span {span:.1f} us; block duration median {np.median(dur):.1f} "
          f"p10 {np.percentile(dur, 10):.1f} p90 {np.percentile(dur, 90):.1f} us")
    grid = np.linspace(0, span, 41)
    busy = [int(((st <= x) & (en > x)).sum()) for x in grid]
    print("busy blocks over the launch (41 samples):", busy)
    full = np.median(busy[5:-5]) if len(busy) > 10 else max(busy)
    work = dur.sum()
    print(f"steady busy {full:.0f}; ideal span at that occupancy {work / full:.1f} us "
          f"-> loss {span - work / full:.1f} us ({(span - work / full) / span * 100:.1f}%)")
    for x in range(int(xcc.max()) + 1):
        m = xcc == x
        if m.any():
            print(f"  xcc {x}: blocks {int(m.sum())}, last end {en[m].max():.1f} us, "
                  f"median duration {np.median(dur[m]):.1f} us, CUs {len(np.unique(cu[m]))}")
    last = np.argsort(en)[-5:]
    print("last blocks (id, start, end, xcc, cu):",
          [(int(i), round(float(st[i]), 1), round(float(en[i]), 1), int(xcc[i]), int(cu[i]))
           for i in last])
    first_end = np.sort(en)[: int(full)].max() if full else 0
    print(f"first start spread: {np.percentile(st[: int(full)], 99):.1f} us for the first {int(full)} blocks")


if __name__ == "__main__":
    main()
