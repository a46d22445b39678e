"""Host-side (Python) profile of c2 generations on the GPU box.

    python tools/profile_host.py [--pop 100000] [--gens 3] [--top 40]

Runs the bench workload (warm-up run, then a timed run) under cProfile and
prints the top functions by cumulative and by own time, plus the per-generation
wall times, to find the host gaps between kernel launches.
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=100_000)
    ap.add_argument("--gens", type=int, default=3)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import torch
    import bench
    sys.argv = [sys.argv[0], "--pop", str(a.pop)]
    args = bench.parse()
    abc, tr = bench.build_abc(args, 0, 1)
    abc.run(max_nr_populations=2)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    abc.run(max_nr_populations=a.gens)
    torch.cuda.synchronize()
    pr.disable()
    print(f"timed run: {1e3 * (time.perf_counter() - t0):.2f} ms for {a.gens} gens; "
          f"per gen {[round(1e3 * g['seconds'], 2) for g in abc.generation_log[-a.gens:]]}")
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(a.top)
    # microseconds per generation (pstats prints milliseconds at best)
    rows = sorted(st.stats.items(), key=lambda kv: -kv[1][2])[:a.top]
    print(f"{'own us/gen':>10} {'cum us/gen':>10} {'calls/gen':>9}  function")
    for (f, line, name), (cc, nc, tt, ct, _) in rows:
        print(f"{1e6 * tt / a.gens:10.1f} {1e6 * ct / a.gens:10.1f} {nc / a.gens:9.1f}  "
              f"{os.path.basename(f)}:{line}({name})")


if __name__ == "__main__":
    main()
