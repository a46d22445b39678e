"""One c4 run (S = 256, N = 2e5, AdaptivePNormDistance with the MAD scale,
record_rejected) for rocprofv3 kernel traces of a whole generation; the same
model as tools/bench_components.py's e2e c4 line."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import pyabc_amd as pa
    rng = np.random.default_rng(1234)
    S, d = 256, 4
    names = [f"p{k}" for k in range(d)]
    keys = [f"s{k:03d}" for k in range(S)]
    a = rng.uniform(0.5, 2.0, S)
    sig = 10 ** rng.uniform(-2, 2, S)
    model = pa.LinearGaussianModel(names, keys, src=[k % d for k in range(S)], a=a, sigma=sig)
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    x0 = {k: float(a[i] * 0.5) for i, k in enumerate(keys)}
    abc = pa.ABCSMC(model, prior,
                    pa.AdaptivePNormDistance(scale_function=pa.distance.median_absolute_deviation),
                    population_size=200_000, sampler=pa.BatchedGPUSampler(seed=2))
    abc.new("sqlite://", x0)
    abc.run(max_nr_populations=5)
    torch.cuda.synchronize()
    print([round(1e3 * g["seconds"], 2) for g in abc.generation_log])


if __name__ == "__main__":
    main()
