"""Benchmark: accepted particles / s per ABC-SMC generation on MI355X.

Workload (BASELINE.json configs[1], "c2"): 10-D Gaussian model with the
vectorised simulator y_k = theta_k + 0.5 eps_k, prior N(0, 1)^10, x_0 = 1,
MultivariateNormalTransition (f64-MFMA transition density), PNormDistance
p = 2, QuantileEpsilon(alpha = 0.5), population 1e5 per GPU.  A "step" is one
full generation: batched candidate generation until N_pop are accepted,
importance weights (the N_acc x N_pop transition density), fit of the next
transition, epsilon quantile.  Inputs are synthetic and generated on the
device; nothing is read from the host inside the timed region except the
per-round accept counts.

Multi-GPU (torch.distributed.run, one rank per GPU, nccl = RCCL): candidates
are sharded by global index, the population (1e5 x n_gpus particles) is
replicated by all-gather each generation ("scaling": "weak": per-GPU accepted
particles fixed; the transition density per GPU grows with the population).

The JSON line also carries the roofline of the dominant kernel (the fused
cross-term GEMM + log-sum-exp, mvn_lse_kernel) timed with HIP events on the
launch stream, and a CPU baseline: the numpy oracle (oracle/) timed on a
bounded sample of the same generation on this host.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

F64_MFMA_PEAK_TFLOPS = 78.6    # MI355X FP64 matrix (spec)
F32_MFMA_PEAK_TFLOPS = 157.3   # MI355X FP32 matrix (spec; MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pop", type=int, default=100_000, help="per GPU")
    ap.add_argument("--dim", type=int, default=10)
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def setup_dist():
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if ws > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, ws


class KernelTimer:
    """HIP-event timing of every transition-density launch on its stream."""

    def __init__(self, transition):
        import torch
        self.torch = torch
        self.events = []
        self.shapes = []
        self.active = False
        orig = transition.logpdf_device

        def timed(xd, out=None):
            if not self.active:
                return orig(xd, out=out)
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            r = orig(xd, out=out)
            e.record()
            self.events.append((s, e))
            self.shapes.append((xd.shape[0], transition._dev_X.shape[0],
                                xd.shape[1]))
            return r
        transition.logpdf_device = timed

    def summary(self):
        self.torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e in self.events]
        flops = [2.0 * d * M * N for (M, N, d) in self.shapes]
        pairs = [M * N for (M, N, d) in self.shapes]
        return ms, flops, pairs


def build_abc(args, rank, ws):
    import pyabc_amd as pa
    d = args.dim
    names = [f"p{k}" for k in range(d)]
    keys = [f"y{k}" for k in range(d)]
    model = pa.LinearGaussianModel(names, keys, src=list(range(d)),
                                   sigma=[0.5] * d)
    prior = pa.Distribution(**{n: pa.RV("norm", 0, 1) for n in names})
    tr = pa.MultivariateNormalTransition(precision=args.precision)
    abc = pa.ABCSMC(model, prior, pa.PNormDistance(p=2),
                    population_size=args.pop * ws,
                    transitions=tr, eps=pa.QuantileEpsilon(alpha=0.5),
                    sampler=pa.BatchedGPUSampler(seed=20251016))
    abc.new("sqlite://", {k: 1.0 for k in keys})
    return abc, tr


def cpu_baseline(args, population, cov, budget_s):
    """Oracle (numpy fp64) on a bounded sample of one generation: per
    accepted particle it pays the transition density against the full
    population plus (1/acceptance rate) candidates of rvs + prior + simulate
    + distance.  Returns accepted particles/s on this host, 1 core."""
    import oracle
    import oracle.sampler as osamp
    X, w = population
    N, d = X.shape
    L = np.linalg.cholesky(cov)
    t0 = time.perf_counter()
    n_c = 0
    # candidate stage (vectorised numpy, like a tuned CPU port)
    while time.perf_counter() - t0 < 0.25 * budget_s:
        th, lp, _, _ = osamp.propose_mvn(X, w, L, 1, 1, n_c, 4096,
                                         ["norm"] * d, np.tile([0, 1, 0, 0], (d, 1)))
        x = osamp.simulate_linear_gaussian(th, np.arange(d), np.ones(d),
                                           np.full(d, .5), 1, 1, n_c)
        oracle.pnorm(x, np.ones(d))
        n_c += 4096
    t_cand = (time.perf_counter() - t0) / n_c
    t1 = time.perf_counter()
    n_p = 0
    while time.perf_counter() - t1 < 0.75 * budget_s:
        oracle.mvn_logpdf(th[:64], X, w, cov, block=64)
        n_p += 64
    t_pdf = (time.perf_counter() - t1) / n_p
    return t_cand, t_pdf, n_c, n_p


def main():
    args = parse()
    import torch
    rank, ws = setup_dist()
    if ws != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {ws}", file=sys.stderr)
    import pyabc_amd as pa  # noqa: F401  (loads libabcgpu.so, fails loudly)
    abc, tr = build_abc(args, rank, ws)
    timer = KernelTimer(tr)

    def barrier():
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    # warmup: calibration + W generations
    abc.run(max_nr_populations=max(args.warmup, 1))
    barrier()
    n_before = len(abc.generation_log)
    timer.active = True
    t0 = time.perf_counter()
    abc.run(max_nr_populations=args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    timer.active = False
    gens = abc.generation_log[n_before:]
    steps = len(gens)
    t_local = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if ws > 1:
        torch.distributed.all_reduce(t_local, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t_local.item())
    n_pop = args.pop * ws
    value = steps * n_pop / elapsed
    pair_evals = steps * n_pop * n_pop / elapsed
    ms, flops, pairs = timer.summary()
    # dominant kernel: the transition density launches of the timed region
    avg_ms = float(np.mean(ms)) if ms else float("nan")
    avg_flop = float(np.mean(flops)) if flops else float("nan")
    achieved = avg_flop / (avg_ms * 1e-3) / 1e12
    peak = F64_MFMA_PEAK_TFLOPS if args.precision == "f64" else F32_MFMA_PEAK_TFLOPS
    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and ws == 1:
            hist = abc.history
            df, w = hist.get_distribution(0, hist.max_t)
            acc_rate = n_pop / gens[-1]["n_sim"]
            t_cand, t_pdf, n_c, n_p = cpu_baseline(
                args, (df.values, w), tr.cov, args.cpu_baseline_seconds)
            per_acc = t_pdf + t_cand / acc_rate
            cpu = {"value": 1.0 / per_acc, "unit": "accepted particles/s",
                   "cores": 1, "kind": "port",
                   "sample": (f"oracle (numpy fp64) on this host: {n_p} transition "
                              f"densities vs the full N={n_pop} population + {n_c} "
                              f"candidates (rvs, prior, simulate, distance), "
                              f"extrapolated at the measured acceptance rate "
                              f"{acc_rate:.3f}")}
        out = {
            "metric": "accepted particles/sec/generation",
            "value": value,
            "unit": "accepted particles/s",
            "n_gpus": ws,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / max(steps, 1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (device-generated, counter-based RNG)",
            "config": {"workload": "c2: 10-D Gaussian, vectorised simulator, "
                                   "MVN transition, PNorm p=2, QuantileEpsilon(0.5)",
                       "population": n_pop, "population_per_gpu": args.pop,
                       "d": args.dim, "parallelism": f"candidate-sharded x{ws}"},
            "pair_evals_per_s": pair_evals,
            "acceptance_rate_last": n_pop / gens[-1]["n_sim"] if gens else None,
            "generation_ms": [round(1e3 * g["seconds"], 3) for g in gens],
            "roofline": {"bound": "mfma", "kernel": "mvn_lse_kernel "
                         f"({args.precision} MFMA cross term + exp2 + LSE)",
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak,
                         "frac_of_f32_mfma_peak": achieved / F32_MFMA_PEAK_TFLOPS,
                         "flop_per_pair": 2 * args.dim,
                         "launches": len(ms), "avg_launch_ms": avg_ms,
                         "traffic": None},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if ws > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
