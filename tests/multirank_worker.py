"""Worker for tests/test_gpu_multirank.py (not a test module).

Runs a small c2-shaped ABC-SMC (d = 4, QuantileEpsilon, PNorm, MVN x3; or
with MODE=stochastic the StochasticAcceptor / Temperature stack) with
the batched GPU sampler and writes rank 0's final population, weights,
epsilons and evaluation counts to ``$OUT``.  Started either as a single
process or under torch.distributed.run (gloo backend, every rank on cuda:0:
the functional multi-rank path on a one-GPU box).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    if ws > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    import pyabc_amd as pa
    d = 4
    names = [f"p{k}" for k in range(d)]
    keys = [f"y{k}" for k in range(d)]
    model = pa.LinearGaussianModel(names, keys, src=list(range(d)),
                                   sigma=[0.5] * d)
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    if os.environ.get("MODE") == "stochastic":
        # noise-model ABC: kernel values, stochastic accept, records of all
        # candidates with both transition densities, temperature bisection
        dist = pa.IndependentNormalKernel(var=[0.3] * d)
        eps = pa.Temperature()
        acceptor = pa.StochasticAcceptor()
    else:
        dist, eps, acceptor = (pa.PNormDistance(p=2),
                               pa.QuantileEpsilon(alpha=0.5), None)
    pop = int(os.environ.get("POP", "20000"))
    if os.environ.get("MODE") == "adaptive_popsize":
        # every rank fits the same bootstraps from its own numpy stream;
        # rank 0's size must be the one every rank samples
        np.random.seed(1000 + rank)
        pop = pa.AdaptivePopulationSize(pop, mean_cv=0.2, n_bootstrap=3,
                                        max_population_size=3 * pop)
    abc = pa.ABCSMC(model, prior, dist,
                    population_size=pop,
                    transitions=pa.MultivariateNormalTransition(),
                    eps=eps, acceptor=acceptor,
                    sampler=pa.BatchedGPUSampler(seed=77, batch_size=None))
    abc.new("sqlite://", {k: 1.0 for k in keys})
    h = abc.run(max_nr_populations=int(os.environ.get("GENS", "4")))
    if rank == 0:
        df, w = h.get_distribution(0, h.max_t)
        pops = h.get_all_populations()
        np.savez(os.environ["OUT"], theta=df.values, w=w,
                 eps=pops["epsilon"].values[1:],
                 samples=pops["samples"].values[1:],
                 sizes=pops["particles"].values[1:])
    if ws > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
