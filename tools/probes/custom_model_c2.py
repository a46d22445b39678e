"""c2-shaped ABC-SMC (N = 1e5, d = S = 10) with a user VectorizedModel (a
torch closure, no fused simulator) against the built-in LinearGaussianModel:
per-generation wall times of the batched sampler's two paths."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "/root/repo")
import pyabc_amd as pa  # noqa: E402

GENS = int(sys.argv[1]) if len(sys.argv) > 1 else 12
N, d = 100_000, 10
names = [f"p{k}" for k in range(d)]
keys = [f"y{k}" for k in range(d)]


def user_sim(theta, seed, gen, idx0):
    g = torch.Generator(device=theta.device)
    g.manual_seed((seed * 1000003 + gen * 7919 + idx0) % (2 ** 63))
    return theta + 0.5 * torch.randn(theta.shape, generator=g, dtype=theta.dtype,
                                      device=theta.device)


def run(model, tag):
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    abc = pa.ABCSMC(model, prior, pa.PNormDistance(p=2), population_size=N,
                    eps=pa.QuantileEpsilon(alpha=0.5),
                    sampler=pa.BatchedGPUSampler(seed=5))
    abc.new("sqlite://", {k: 1.0 for k in keys})
    times = []
    last = [time.perf_counter()]

    def cb(t):
        torch.cuda.synchronize()
        now = time.perf_counter()
        times.append(round(1e3 * (now - last[0]), 2))
        last[0] = now
    abc.generation_callback = cb
    abc.run(max_nr_populations=GENS)
    st = abc.sampler.last_stats
    print(json.dumps({"model": tag, "generation_ms": times,
                      "median_ms_gen2+": float(np.median(times[2:])),
                      "last_stats": {k: st[k] for k in st if k in ("rounds", "evaluations", "fused")}}),
          flush=True)


which = sys.argv[2] if len(sys.argv) > 2 else "both"
if which in ("both", "builtin"):
    run(pa.LinearGaussianModel(names, keys, src=list(range(d)), sigma=[0.5] * d), "builtin")
if which in ("both", "user"):
    run(pa.VectorizedModel(user_sim, keys), "user")
