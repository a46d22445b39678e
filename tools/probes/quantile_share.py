"""Two processes sharing the GPU, each calling the one-launch weighted
quantile at N = 1e6 in a loop (probe): do both grids always complete, and
does any call end on the bounded wait (NaN, then the workspace on the sorted
path)?   python tools/probes/quantile_share.py [--procs 2] [--calls 300]"""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(calls):
    sys.path.insert(0, ROOT)
    import torch
    from pyabc_amd import gpu
    gpu.require_device()
    N = 1_000_000
    g = torch.Generator(device="cuda").manual_seed(os.getpid())
    d = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) * 4 + 1
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g)
    ref = float(gpu.weighted_quantile(d, w, 0.5, sorted_path=True).cpu()[0])
    nan = bad = 0
    worst = 0.0
    vals = set()
    t0 = time.time()
    for _ in range(calls):
        q = float(gpu.weighted_quantile(d, w, 0.5).cpu()[0])
        if q != q:
            nan += 1
            continue
        vals.add(q)
        rel = abs(q - ref) / abs(ref)
        worst = max(worst, rel)
        bad += rel > 1e-12
    # (the select and the sort-based path sum the weights in different
    # orders: equal to 1e-12, not necessarily bit for bit)
    print(f"pid {os.getpid()}: {calls} calls in {time.time() - t0:.2f} s, NaN {nan}, "
          f"beyond 1e-12 {bad}, max rel diff vs sorted {worst:.2e}, distinct values {len(vals)}",
          flush=True)
    return 1 if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        sys.exit(child(a.calls))
    ps = [subprocess.Popen([sys.executable, __file__, "--child", "--calls", str(a.calls)])
          for _ in range(a.procs)]
    rc = [p.wait() for p in ps]
    sys.exit(max(rc))


if __name__ == "__main__":
    main()
