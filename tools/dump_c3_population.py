"""Run the c3 bench workload (bench.py build_abc) for G generations and save
the populations' weights (float32) of the last few generations, for the
ancestor-draw access analysis (tools/ancestor_access.py).

    python tools/dump_c3_population.py --gens 25 --keep 5 --out gpurun_out/pop
"""
import argparse
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", type=int, default=25)
    ap.add_argument("--keep", type=int, default=5)
    ap.add_argument("--pop", type=int, default=1_000_000)
    ap.add_argument("--out", default="gpurun_out/pop")
    a = ap.parse_args()
    import bench
    os.makedirs(a.out, exist_ok=True)
    args = types.SimpleNamespace(dim=10, precision="x3", pop=a.pop, filter_below=None)
    abc, tr = bench.build_abc(args, 0, 1)

    def on_generation(t):
        if t >= a.gens - a.keep:
            cols = abc.history.get_population_device(t)
            w = cols.weights.double()
            w = (w / w.sum()).float().cpu().numpy()
            np.save(os.path.join(a.out, f"w_t{t}.npy"), w)
            print(f"t={t} saved, ESS={1.0 / float((w.astype(np.float64) ** 2).sum()):.4g}",
                  flush=True)
    abc.generation_callback = on_generation
    abc.run(max_nr_populations=a.gens)


if __name__ == "__main__":
    main()
