"""Benchmark: accepted particles / s per ABC-SMC generation on MI355X.

Workload (BASELINE.json configs[2], "c3"): 10-D Gaussian model with the
vectorised simulator y_k = theta_k + 0.5 eps_k, prior N(0, 1)^10, x_0 = 1,
MultivariateNormalTransition (x3 limb-split f16-MFMA transition density),
PNormDistance p = 2, QuantileEpsilon(alpha = 0.5), population 1e6 in total.
A "step" is one full generation: batched candidate generation until N_pop
are accepted, importance weights (the N_acc x N_pop transition density), fit
of the next transition, epsilon quantile.  Inputs are synthetic and generated
on the device; nothing is read from the host inside the timed region except
the per-round accept counts.  `--pop 100000` runs configs[1] ("c2", the
one-GPU config); both are reported in DESIGN.md.

Multi-GPU (one rank per GPU, nccl = RCCL): `python bench.py --gpus N` starts
its N rank processes itself (`spawn_ranks`, the parent never touches the
GPU); under `torch.distributed.run` (WORLD_SIZE set) each process is one
rank.  Candidates
are sharded by global index, each rank weights its own accepted rows against
the replicated population, the accepted rows are all-gathered ("scaling":
"strong": the population -- total work -- is fixed as N grows).  The c3
population is the one the north star's 8-GPU target is stated on; at c2 size
one generation is ~3 ms and too small to split over 8 GPUs.

The JSON line also carries the roofline of the dominant kernel (the fused
cross-term GEMM + exp2 + sum, mvn_x3_kernel) timed with HIP events recorded
by libabcgpu on the launch stream around each launch, and a CPU baseline: the
numpy oracle (oracle/) timed on a bounded sample of the same generation on
this host.
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
F16_MFMA_PEAK_TFLOPS = 2516.6  # MI355X FP16 dense matrix (spec, no sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pop", type=int, default=1_000_000,
                    help="total population (all GPUs)")
    ap.add_argument("--dim", type=int, default=10)
    ap.add_argument("--precision", default="x3", choices=["x3", "f64", "f32"])
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-cores", type=int, default=16,
                    help="worker processes of the CPU baseline (the box's CPU "
                         "share per GPU is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--collectives", default="torch", choices=["torch", "abc"],
                    help="abc: the sampler's all-gathers through libabcgpu's RCCL "
                         "wrappers (abc_comm_*) instead of torch.distributed")
    ap.add_argument("--filter-below", type=float, default=None,
                    help="BatchedGPUSampler.filter_below (default: the sampler's)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: functional multi-rank runs on one GPU (tests)")
    ap.add_argument("--launcher-check", action="store_true",
                    help="rendezvous over gloo on the CPU, exchange one value per "
                         "rank and print the rank count; no GPU (tests the launcher)")
    return ap.parse_args()


def launcher_check():
    import torch
    import torch.distributed as dist
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("BENCH_LAUNCHER_FAIL_RANK") == str(rank):
        sys.exit(3)     # the launcher test's failing rank
    if ws > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank), 1.0], dtype=torch.float64)
    if ws > 1:
        dist.all_reduce(t)
    got = [None] * ws
    if ws > 1:
        dist.all_gather_object(got, (rank, int(os.environ.get("LOCAL_RANK", "0")), os.getpid()))
        dist.destroy_process_group()
    else:
        got = [(0, 0, os.getpid())]
    if rank == 0:
        print(json.dumps({"launcher_check": True, "n_gpus": ws,
                          "rank_sum": t[0].item(), "ranks": t[1].item(),
                          "local_ranks": [g[1] for g in got],
                          "distinct_pids": len({g[2] for g in got})}), flush=True)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv=None):
    """`python bench.py --gpus N` with no WORLD_SIZE in the environment: start
    N rank processes of this script (RANK = LOCAL_RANK = i, WORLD_SIZE = N,
    MASTER_ADDR 127.0.0.1, a free MASTER_PORT) and wait for all of them -- the
    process fan-out of the reference's MulticoreEvalParallelSampler
    (multicore_evaluation_parallel.py:92-150), one process per GPU.  This
    parent never touches the GPU (no torch import); the children are started
    as new processes, never exec'd over it.  Returns the first non-zero child
    exit code (a failed rank kills the others), else 0."""
    import signal
    import subprocess
    argv = list(sys.argv[1:] if argv is None else argv)
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)]
                                      + argv, env=env, start_new_session=True))
    rc = 0
    live = set(range(n))
    try:
        while live:
            for r in sorted(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench: rank {r} exited with {code}; stopping the others",
                          file=sys.stderr, flush=True)
                    for q in live:
                        try:
                            os.killpg(procs[q].pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        raise
    for p in procs:
        p.wait()
    return rc


def setup_dist(backend="nccl"):
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    if ws > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    return rank, ws


class KernelTimer:
    """Dominant-kernel timing: libabcgpu records HIP events on the launch
    stream directly around every transition-density GEMM launch
    (abc_profile_begin/end); the wrapper below only logs the (M, N, d) shape
    of each call for the algorithmic FLOP count."""

    def __init__(self, transition):
        self.shapes = []
        self.active = False
        orig = transition.logpdf_device

        def logged(xd, out=None, hint=None):
            if self.active and getattr(transition, "_mfma", False):
                self.shapes.append((xd.shape[0], transition._dev_X.shape[0],
                                    xd.shape[1]))
            return orig(xd, out=out, hint=hint)
        transition.logpdf_device = logged

    def begin(self):
        from pyabc_amd import _native as nat
        self.shapes = []
        self.active = True
        nat.call("abc_profile_begin")

    def end(self):
        import ctypes
        from pyabc_amd import _native as nat
        self.active = False
        ms = ctypes.c_double(0.0)
        n = ctypes.c_int64(0)
        nat.call("abc_profile_end", ctypes.addressof(ms), ctypes.addressof(n))
        flops = sum(2.0 * d * M * N for (M, N, d) in self.shapes)
        pairs = sum(M * N for (M, N, d) in self.shapes)
        self.channels = {}
        for name, ch in (("candidates", nat.ABC_PROF_CANDIDATES),
                         ("regen", nat.ABC_PROF_REGEN),
                         ("rescue", nat.ABC_PROF_RESCUE)):
            cm, cn = ctypes.c_double(0.0), ctypes.c_int64(0)
            nat.call("abc_profile_channel", ch, ctypes.addressof(cm), ctypes.addressof(cn))
            self.channels[name] = (cm.value, int(cn.value))
        return ms.value, int(n.value), flops, pairs


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
                    population_size=args.pop,
                    transitions=tr, eps=pa.QuantileEpsilon(alpha=0.5),
                    sampler=pa.BatchedGPUSampler(seed=20251016, **(
                        {} if args.filter_below is None
                        else {"filter_below": args.filter_below})))
    abc.new("sqlite://", {k: 1.0 for k in keys})
    return abc, tr


def _cpu_worker(job):
    """One MulticoreEval-style worker (multicore_evaluation_parallel.py:14-50
    evaluates candidates until the shared count is reached): here the
    oracle's vectorised restatement of the same per-candidate closure in
    chunks of 4096 for cand_s seconds, then transition densities of
    candidates against the full population for pdf_s seconds."""
    import oracle
    import oracle.sampler as osamp
    from multiprocessing import shared_memory
    name, shape, wname, L, cov, cand_s, pdf_s, wid = job
    shm, shw = shared_memory.SharedMemory(name=name), shared_memory.SharedMemory(name=wname)
    try:
        X = np.ndarray(shape, dtype=np.float64, buffer=shm.buf)
        w = np.ndarray((shape[0],), dtype=np.float64, buffer=shw.buf)
        d = shape[1]
        t0 = time.perf_counter()
        n_c = 0
        idx0 = wid << 40
        while time.perf_counter() - t0 < cand_s:
            th, lp, _, _ = osamp.propose_mvn(X, w, L, 1, 1, idx0 + n_c, 4096,
                                             ["norm"] * d, np.tile([0, 1, 0, 0], (d, 1)))
            x = osamp.simulate_linear_gaussian(th, np.arange(d), np.ones(d),
                                               np.full(d, .5), 1, 1, idx0 + n_c)
            oracle.pnorm(x, np.ones(d))
            n_c += 4096
        t_c = time.perf_counter() - t0
        t1 = time.perf_counter()
        n_p = 0
        while time.perf_counter() - t1 < pdf_s:
            oracle.mvn_logpdf(th[n_p % 4096:n_p % 4096 + 4], X, w, cov, block=4)
            n_p += 4
        return n_c, t_c, n_p, time.perf_counter() - t1
    finally:
        shm.close()
        shw.close()


def cpu_baseline(args, population, cov, budget_s, cores):
    """The oracle (numpy fp64 restatement of the per-candidate closure and of
    the transition density) on `cores` worker processes of this host, shaped
    like MulticoreEvalParallelSampler: every worker evaluates candidates and
    densities on the shared population for a bounded time.  Returns the
    host's aggregate rates (candidates/s, densities/s)."""
    import multiprocessing as mp
    from multiprocessing import shared_memory
    X, w = population
    X = np.ascontiguousarray(X, dtype=np.float64)
    w = np.ascontiguousarray(w, dtype=np.float64)
    L = np.linalg.cholesky(cov)
    shm = shared_memory.SharedMemory(create=True, size=X.nbytes)
    shw = shared_memory.SharedMemory(create=True, size=w.nbytes)
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS",
                                            "MKL_NUM_THREADS")}
    try:
        np.ndarray(X.shape, dtype=np.float64, buffer=shm.buf)[:] = X
        np.ndarray(w.shape, dtype=np.float64, buffer=shw.buf)[:] = w
        for k in saved:     # one BLAS thread per worker process
            os.environ[k] = "1"
        jobs = [(shm.name, X.shape, shw.name, L, cov, 0.25 * budget_s, 0.75 * budget_s, i)
                for i in range(cores)]
        with mp.get_context("spawn").Pool(cores) as pool:
            res = pool.map(_cpu_worker, jobs)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        shm.close()
        shm.unlink()
        shw.close()
        shw.unlink()
    n_c = sum(r[0] for r in res)
    n_p = sum(r[2] for r in res)
    cand_rate = sum(r[0] / r[1] for r in res)
    pdf_rate = sum(r[2] / r[3] for r in res)
    return cand_rate, pdf_rate, n_c, n_p


def measured_traffic(args, n_pop, kernel):
    """HBM bytes per launch of the dominant kernel from the committed
    rocprofv3 --pmc passes (profiles/*_x3_traffic_*.json, written by
    tools/traffic_from_pmc.py) when they were taken on this workload and on
    the kernel the library runs now (`kernel`: its mangled-name stem)."""
    import glob
    if args.precision != "x3":
        return None, None
    # newest round first (profiles/rNN_...): the kernel that runs is HEAD's
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_x3_traffic_*.json")),
                    reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (t.get("population") == n_pop and t.get("d") == args.dim
                and kernel in t.get("kernel_name", "")):
            return t["traffic_bytes"], os.path.relpath(f, ROOT)
    return None, None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.launcher_check:
        return launcher_check()
    import torch
    rank, ws = setup_dist(args.dist_backend)
    if ws != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {ws}", file=sys.stderr)
    import pyabc_amd as pa  # noqa: F401  (loads libabcgpu.so, fails loudly)
    if ws > 1 and args.collectives == "abc":
        from pyabc_amd.sampler import distributed as dd
        from pyabc_amd.sampler.comm import RcclComm
        dd.use_comm(RcclComm.from_process_group())
    abc, tr = build_abc(args, rank, ws)
    timer = KernelTimer(tr)

    def barrier():
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    # one run of W + K generations: calibration + W untimed warm-up
    # generations, then EXACTLY K timed ones (each: sample until N accepted,
    # importance weights, fit of the next transition, epsilon update),
    # bracketed by barrier + synchronize, started/stopped from the
    # per-generation hook so every timed generation is a genuine continuation
    warm = max(args.warmup, 1)
    clock = {}

    cand_per_gen = []

    def on_generation(t):
        done = len(abc.generation_log)
        cand_per_gen.append(int(abc.sampler.last_stats.get("candidates", 0)))
        if done == warm:
            barrier()
            timer.begin()
            clock["n0"] = done
            clock["t0"] = time.perf_counter()
        elif done == warm + args.steps:
            barrier()
            clock["t1"] = time.perf_counter()
            clock["kernel"] = timer.end()
    abc.generation_callback = on_generation
    abc.run(max_nr_populations=warm + args.steps)
    if "t1" not in clock:
        raise RuntimeError("run stopped before the timed generations finished")
    elapsed = clock["t1"] - clock["t0"]
    elapsed_local = elapsed
    k_ms, k_n, k_flops, k_pairs = clock["kernel"]
    n_before = clock["n0"]
    gens = abc.generation_log[n_before:n_before + args.steps]
    steps = len(gens)
    t_local = torch.tensor([elapsed], dtype=torch.float64,
                           device="cuda" if args.dist_backend == "nccl" else "cpu")
    if ws > 1:
        torch.distributed.all_reduce(t_local, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t_local.item())
    n_pop = args.pop
    value = steps * n_pop / elapsed
    pair_evals = steps * n_pop * n_pop / elapsed
    # dominant kernel: the transition-density GEMM launches of the timed region
    avg_ms = k_ms / k_n if k_n else float("nan")
    achieved = k_flops / (k_ms * 1e-3) / 1e12 if k_n else float("nan")
    peak = F64_MFMA_PEAK_TFLOPS if args.precision == "f64" else F32_MFMA_PEAK_TFLOPS
    # executed K per pair and the kernel, as the library reports them
    from pyabc_amd import gpu
    _, x3_k, x3_ct = gpu.mvn_x3_layout(args.dim) if args.precision == "x3" else (0, 0, 0)
    kpad = {"x3": x3_k,
            "f64": 4 * math.ceil((args.dim + 1) / 4),
            "f32": 4 * math.ceil((args.dim + 1) / 4)}[args.precision]
    executed = 2.0 * kpad * k_pairs / (k_ms * 1e-3) / 1e12 if k_n else float("nan")
    exec_peak = {"x3": F16_MFMA_PEAK_TFLOPS, "f64": F64_MFMA_PEAK_TFLOPS,
                 "f32": F32_MFMA_PEAK_TFLOPS}[args.precision]
    kname = {"x3": (f"mvn_x3_kernel (f16 MFMA, K = {x3_k} per pair; 3-limb split "
                    "operands, exact-grid f32 accumulation + exp2 + sum)"),
             "f64": "mvn_lse_kernel<double> (f64 MFMA cross term + exp2 + LSE)",
             "f32": "mvn_lse_kernel<float> (f32 MFMA cross term + exp2 + LSE)"}
    # the main (hinted) instantiation, mvn_x3_kernel<KB, CT, false>
    traffic, traffic_src = measured_traffic(
        args, n_pop, f"mvn_x3_kernelILi{x3_k // 16}ELi{x3_ct}ELb0E")
    # per-stage split of the timed region (HIP events on the launch streams)
    c_ms, c_n = timer.channels["candidates"]
    r_ms, r_n = timer.channels["regen"]
    x_ms, x_n = timer.channels["rescue"]
    timed_cands = cand_per_gen[n_before:n_before + steps]
    n_cand = int(sum(timed_cands))
    stages = {"density_gemm_ms": k_ms, "candidate_rounds_ms": c_ms,
              "regen_ms": r_ms, "density_rescue_ms": x_ms,
              "other_ms": 1e3 * elapsed - k_ms - c_ms - r_ms - x_ms,
              "note": ("other = fit (moments, eigh, guide, x3 pack), epsilon "
                       "quantile, weights, compaction, host gaps")}
    cand = {"kernel": "fused_round_kernel (proposal + prior re-draw + "
                      "LinearGaussian simulation + p-norm + accept bit)",
            "candidates": n_cand, "launches": c_n,
            "candidates_per_s": n_cand / (c_ms * 1e-3) if c_ms else None,
            "bytes_per_candidate": {"written": 0.125,
                                    "read_cached": 8 * (args.dim + 3) + 8},
            "bound": ("random accesses + VALU issue, not HBM: per candidate "
                      "1.67 L2 misses + 0.88 L2 hits (ancestor guide entry + "
                      "record) at c3's skewed weights and ~1380 VALU lane-"
                      "instructions (Philox4x32-10 and the fp32 Box-Muller "
                      "transform); PMC in profiles/r03_fused_pmc_skewed_w.txt"),
            "candidates_per_generation": timed_cands}
    # unique bytes one launch must move: the population and candidate
    # operand images (kpad f16 per row) + the fp64 result
    avg_m = k_pairs / max(k_n, 1) / n_pop if k_n else 0
    algo_bytes = ((n_pop + avg_m) * kpad * 2 + avg_m * 8) if args.precision == "x3" else None
    out = None
    stages_per_rank = None
    if ws > 1:
        # each rank's own stage split (its density launches, candidate
        # rounds, ...) so a scaling line can be read from its own output
        mine = {k: (round(v, 3) if isinstance(v, float) else v)
                for k, v in stages.items() if k != "note"}
        mine["other_ms"] = round(1e3 * elapsed_local - k_ms - c_ms - r_ms - x_ms, 3)
        mine.update(rank=rank, elapsed_ms=round(1e3 * elapsed_local, 3),
                    density_launches=k_n, candidate_launches=c_n)
        box = [None] * ws
        torch.distributed.all_gather_object(box, mine)
        stages_per_rank = box
        # every rank is done with the GPU; rank 0 alone times the host leg
        torch.distributed.destroy_process_group()
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:
            hist = abc.history
            df, w = hist.get_distribution(0, hist.max_t)
            cores = max(1, min(args.cpu_cores, os.cpu_count() or 1))
            cand_rate, pdf_rate, n_c, n_p = cpu_baseline(
                args, (df.values, w), tr.cov, args.cpu_baseline_seconds, cores)
            # the same generations as the GPU value: per timed generation its
            # evaluated candidates (n_sim, at that generation's acceptance)
            # and one transition density per accepted particle; value = all
            # accepted particles / the summed CPU time
            cpu_s = sum(g["n_sim"] / cand_rate + n_pop / pdf_rate for g in gens)
            acc_last = n_pop / gens[-1]["n_sim"]
            last = 1.0 / (1.0 / (cand_rate * acc_last) + 1.0 / pdf_rate)
            cpu = {"value": steps * n_pop / cpu_s, "unit": "accepted particles/s",
                   "cores": cores, "kind": "port",
                   "sample": (f"oracle (numpy fp64 restatement) on {cores} worker "
                              f"processes of this host, MulticoreEval-shaped: "
                              f"{n_c} candidates (rvs, prior, simulate, distance) "
                              f"at {cand_rate:.3e}/s and {n_p} transition densities "
                              f"vs the full N={n_pop} population at {pdf_rate:.3e}/s; "
                              f"value = the timed generations' accepted particles "
                              f"over the CPU time of their own candidate counts "
                              f"(n_sim, acceptance {n_pop / gens[0]['n_sim']:.2e} .. "
                              f"{acc_last:.2e}) and densities; the reference's own "
                              f"samplers are slower than this port by the ratio in "
                              f"BASELINE.md §3"),
                   "value_last_generation": last,
                   "candidates_per_s": cand_rate, "densities_per_s": pdf_rate}
        out = {
            "metric": "accepted particles/sec/generation",
            "value": value,
            "unit": "accepted particles/s",
            "n_gpus": ws,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / max(steps, 1),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": {"x3": "f32 (f16x3-limb MFMA, f32-grade)", "f64": "f64",
                      "f32": "f32"}[args.precision],
            "data": "synthetic (device-generated, counter-based RNG)",
            "config": {"workload": ("c3" if n_pop == 1_000_000 else
                                    ("c2" if n_pop == 100_000 else "custom"))
                                   + ": 10-D Gaussian, vectorised simulator, "
                                   "MVN transition, PNorm p=2, QuantileEpsilon(0.5)",
                       "population": n_pop, "accepted_per_gpu": n_pop // ws,
                       "d": args.dim, "parallelism": f"candidate-sharded x{ws}",
                       "dist_backend": args.dist_backend if ws > 1 else None},
            "pair_evals_per_s": pair_evals,
            "acceptance_rate_last": n_pop / gens[-1]["n_sim"] if gens else None,
            "generation_ms": [round(1e3 * g["seconds"], 3) for g in gens],
            "stages": stages,
            "stages_per_rank": stages_per_rank,
            "candidate_kernel": cand,
            "roofline": {"bound": "mfma", "kernel": kname[args.precision],
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak,
                         "flop_per_pair": 2 * args.dim,
                         "note": ("achieved = algorithmic 2*d FLOP per (candidate, "
                                  "population) pair / HIP-event time of the GEMM "
                                  "launch; peak = fp32 MFMA (x3/f32) or fp64 MFMA. "
                                  "x3 runs f16 MFMA on 3-limb operands, so frac can "
                                  "exceed 1 (fp32-grade results above the fp32 MFMA "
                                  "roofline); its own bound is the MFMA + exp2 + add "
                                  "issue rate per 32x32 tile pair, and executed_frac is "
                                  "the f16 MFMA pipe's share"),
                         "pairs_per_s": k_pairs / (k_ms * 1e-3) if k_n else None,
                         "executed_mfma_tflops": executed,
                         "executed_mfma_peak": exec_peak,
                         "executed_frac": executed / exec_peak,
                         "launches": k_n, "avg_launch_ms": avg_ms,
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes": algo_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
