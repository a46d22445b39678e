"""Multi-rank parity on one GPU: the candidate-sharded sampler run on 2 and
3 ranks (torch.distributed.run, gloo backend, every rank on cuda:0) gives
BIT-IDENTICAL populations, weights, epsilons and evaluation counts to the
single-rank run (draws keyed by the global candidate index,
first-n-accepted cutoff in global order, x3 density summation order
independent of the sharding).  The RCCL (nccl) path runs the same code: a
plain `python bench.py --gpus N` starts N ranks itself (bench.spawn_ranks),
so the driver's scaling run measures it; here bench.py's self-launched
multi-rank path runs with gloo on the one GPU (test_bench_spawned_ranks).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "multirank_worker.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, nproc, mode="uniform", pop=20000, gens=4):
    out = str(tmp_path / f"pop_{mode}_{nproc}_{pop}.npz")
    env = dict(os.environ, OUT=out, POP=str(pop), GENS=str(gens), MODE=mode)
    if nproc == 1:
        cmd = [sys.executable, WORKER]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
               f"--master-port={_port()}", WORKER]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return dict(np.load(out))


def test_sharded_generations_bit_identical(tmp_path):
    """1 vs 2, 3, 4 and 8 ranks (1/2/4/8-rank runs produce an
    identical accepted set)."""
    ref = _run(tmp_path, 1)
    for nproc in (2, 3, 4, 8):
        got = _run(tmp_path, nproc)
        for k in ("theta", "w", "eps", "samples"):
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{k} @ {nproc} ranks")


def test_sharded_tiny_population_bit_identical(tmp_path):
    """A population of 7 on 8 ranks: every round is at least 4096 candidates
    per rank, so rank 0 alone completes each generation and ranks 1..7 keep
    no rows (empty shards in the packed gather, the cutoff on rank 0)."""
    ref = _run(tmp_path, 1, pop=7, gens=3)
    got = _run(tmp_path, 8, pop=7, gens=3)
    for k in ("theta", "w", "eps", "samples"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_sharded_stochastic_generations_bit_identical(tmp_path):
    """The StochasticAcceptor path on 1 vs 2 ranks: accept uniforms keyed by
    the global index, records all-gathered back into global order, the
    temperature objective reduced over identical records."""
    ref = _run(tmp_path, 1, "stochastic")
    got = _run(tmp_path, 2, "stochastic")
    for k in ("theta", "w", "eps", "samples"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{k} @ 2 ranks")


def test_sharded_adaptive_population_size(tmp_path):
    """AdaptivePopulationSize with 1 vs 2 ranks whose numpy streams differ
    (rank-dependent seeds): the broadcast size keeps the ranks in step, and
    rank 0's run equals the single-rank run."""
    ref = _run(tmp_path, 1, "adaptive_popsize")
    got = _run(tmp_path, 2, "adaptive_popsize")
    assert len(set(ref["sizes"])) > 1          # the size did adapt
    for k in ("theta", "w", "eps", "samples", "sizes"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_bench_spawned_ranks():
    """`python bench.py --gpus 2` with no WORLD_SIZE: bench.py starts its two
    rank processes itself; rank 0 prints one line with n_gpus = 2 and a CPU
    baseline (timed after the ranks left the GPU)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--pop", "20000", "--steps", "2",
                        "--warmup", "1", "--cpu-baseline-seconds", "2",
                        "--cpu-cores", "2"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2
    assert out["config"]["dist_backend"] == "gloo"
    assert out["value"] > 0
    assert out["cpu_baseline"] is not None and out["cpu_baseline"]["value"] > 0
