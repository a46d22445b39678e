"""`python bench.py --gpus N` starts its own N rank processes (CPU, no GPU).

The driver's scaling command is a plain `python bench.py --gpus N`; bench.py
must then fan out one process per GPU by itself (the reference's process
fan-out: multicore_evaluation_parallel.py:92-150).  `--launcher-check` runs
the rendezvous and one gloo all-reduce / all-gather per rank without touching
a GPU, so the launcher is covered here.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"),
                           "--gpus", str(n), "--launcher-check"],
                          env=env, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_ranks(n):
    p = _run(n)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1          # rank 0 alone prints the line
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["ranks"] == n
    assert out["rank_sum"] == n * (n - 1) / 2
    assert out["local_ranks"] == list(range(n))
    assert out["distinct_pids"] == n


def test_bench_launcher_propagates_failure():
    p = _run(2, {"BENCH_LAUNCHER_FAIL_RANK": "1"})
    assert p.returncode == 3
    assert "rank 1 exited with 3" in p.stderr


def test_bench_single_rank_no_spawn():
    p = _run(1)
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 1
