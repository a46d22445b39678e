"""World-size-2 gloo tests of the candidate-sharded sampler (CPU, no GPU).

The real ``BatchedGPUSampler.sample_until_n_accepted`` loop and the
``sampler/distributed.py`` collectives run on two gloo ranks.  The per-stage
device calls (propose, simulate, distance, compaction, gather, weights) are
replaced -- in this test only -- by the oracle's replay of the same
counter-based streams (``oracle/sampler.py``), so the sharded run must give
exactly the population of the single-rank run: the first n accepted in global
candidate-index order, with the same ``nr_evaluations_`` and the
same recorded sum stats.  The product path never routes through these doubles
(``gpu.require_device`` raises without a GPU).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import oracle.sampler as osamp

D = 3
SEED = 4242
GEN = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Population:
    def __init__(self):
        rng = np.random.default_rng(3)
        self.X = rng.normal(0.2, 1.0, (500, D))
        w = np.exp(0.3 * rng.standard_normal(500))
        self.w = w / w.sum()
        self.L = np.linalg.cholesky(0.3 * np.eye(D) + 0.05)


class _Transition:
    """propose_device / logpdf_device doubles: oracle replay on CPU."""

    def __init__(self, pop):
        self.pop = pop
        self.cov = pop.L @ pop.L.T

    def propose_device(self, B, kind, params, seed, generation, idx0,
                       max_attempts):
        th, lp, _, _ = osamp.propose_mvn(self.pop.X, self.pop.w, self.pop.L,
                                         seed, generation, idx0, B,
                                         ["norm"] * D, np.tile([0, 1, 0, 0], (D, 1)))
        return torch.from_numpy(th), torch.from_numpy(lp), None, None

    def logpdf_device(self, theta, hint=None):
        return torch.from_numpy(oracle.mvn_logpdf(theta.numpy(), self.pop.X,
                                                  self.pop.w, self.cov))


class _Model:
    def simulate_batch(self, theta, seed, gen, lo):
        return torch.from_numpy(osamp.simulate_linear_gaussian(
            theta.numpy(), np.arange(D), np.ones(D), np.full(D, 0.5), seed,
            gen, lo))


class _Distance:
    def device_call(self, x, x0, t, keys):
        return torch.from_numpy(oracle.pnorm(x.numpy(), x0.numpy()))


class _TailDistance(_Distance):
    """A p-norm distance with the fused form: the staged loop then decides
    acceptance in the accept tail (gpu.pnorm_accept)."""

    def fused_pnorm(self, t, keys, device):
        return torch.ones(D, dtype=torch.float64), 2.0


class _Fut:
    def __init__(self, v):
        self.v = v

    def get(self):
        return np.array([self.v])


class _Spec:
    batched_capable = True

    def __init__(self, eps, tail=False, nan_first=False):
        pop = _Population()
        self.t = GEN
        self.param_names = [f"p{k}" for k in range(D)]
        self.sum_stat_keys = [f"y{k}" for k in range(D)]
        self.transition = _Transition(pop)
        self.model = _Model()
        self.distance = _TailDistance() if tail else _Distance()
        self.x0vec = torch.ones(D, dtype=torch.float64)
        self.eps = eps
        self.weight_scale = 1.0
        if nan_first:
            # QuantileEpsilon's device threshold when its select left the
            # quantile undecided (a knot in a > 2048-key tie run): NaN
            nan = float("nan")
            self.eps_device = (torch.tensor([nan], dtype=torch.float64), 1.0, _Fut(nan))
        self.prior_kind = None
        self.prior_params = None


def _install_cpu_doubles(monkeypatch_like):
    from pyabc_amd.sampler import batched
    g = batched.gpu

    def accept_compact(d, eps):
        idx = torch.nonzero(d <= eps).flatten().to(torch.int64)
        return idx, torch.tensor(idx.numel())

    def gather_rows(x, idx, n=None):
        return x.index_select(0, idx)

    def gather_rows_batch(arrays, idx, n=None):
        return [a.index_select(0, idx) for a in arrays]

    def importance_weights(lp, lt, scale=1.0, acc_w=None):
        w = torch.exp(lp - lt) * scale
        return w if acc_w is None else w * acc_w

    def pnorm(x, x0, wf, pv):
        return torch.from_numpy(oracle.pnorm(x.numpy(), x0.numpy()))

    def pnorm_accept(x, x0, wf, pv, eps, cap, att=None, max_attempts=0):
        acc = np.nonzero(oracle.pnorm(x.numpy(), x0.numpy()) <= eps)[0]
        idx = torch.zeros(max(int(cap), 1), dtype=torch.int64)
        k = min(int(cap), len(acc))
        idx[:k] = torch.from_numpy(acc[:k])
        return idx, torch.tensor([len(acc)])

    def round_keep(counts, need, rank):
        # abc_round_keep on the host (its kernel is tested on the GPU)
        from pyabc_amd.sampler import distributed as dd
        return torch.tensor([int(dd.cutoff(counts.numpy(), need)[rank])])

    monkeypatch_like(g, "round_keep", round_keep)
    monkeypatch_like(g, "pnorm", pnorm)
    monkeypatch_like(g, "pnorm_accept", pnorm_accept)
    monkeypatch_like(g, "require_device", lambda: torch.device("cpu"))
    monkeypatch_like(g, "accept_compact", accept_compact)
    monkeypatch_like(g, "gather_rows", gather_rows)
    monkeypatch_like(g, "gather_rows_batch", gather_rows_batch)
    monkeypatch_like(g, "importance_weights", importance_weights)


class _FusedRound:
    """abc_candidates_round / _regen doubles (oracle replay of the same
    streams): accept positions of a round, and the rows of kept ones."""

    def __init__(self, spec):
        self.pop = spec.transition.pop
        self.d = D

    def _rows(self, lo, B):
        pop = self.pop
        th, lp, anc, _ = osamp.propose_mvn(pop.X, pop.w, pop.L, SEED, GEN, lo, B,
                                           ["norm"] * D, np.tile([0, 1, 0, 0], (D, 1)))
        x = osamp.simulate_linear_gaussian(th, np.arange(D), np.ones(D),
                                           np.full(D, 0.5), SEED, GEN, lo)
        return th, lp, anc, x, oracle.pnorm(x, np.ones(D))

    def run(self, lo, B, eps, cap, filter=True, rec_x=None, eps_dev=None, eps_scale=1.0):
        if eps_dev is not None:
            eps = float(eps_dev[0]) * eps_scale
        *_, x, d = self._rows(lo, B)
        acc = np.nonzero(d <= eps)[0]
        idx = torch.zeros(max(int(cap), 1), dtype=torch.int64)
        k = min(int(cap), len(acc))
        idx[:k] = torch.from_numpy(acc[:k])
        if rec_x is not None:
            rec_x.copy_(torch.from_numpy(x))
        return idx, torch.tensor([len(acc)])

    def regen(self, lo, idx, out=None):
        i = idx.numpy()
        B = int(i.max()) + 1 if len(i) else 0
        th, lp, anc, x, d = self._rows(lo, B)
        rows = tuple(torch.from_numpy(np.ascontiguousarray(a[i]))
                     for a in (th, lp, anc, x, d))
        if out is None:
            return rows
        for o, r in zip(out, rows):   # the sampler's preallocated views
            o.copy_(r.reshape(o.shape))
        return tuple(out)

    def regen_into(self, lo, idx_ptr, n, ptrs, n_dev=None):
        """The sampler's raw-address path (host tensors here): the rows are
        written at the addresses it computed, so its offsets are checked;
        n_dev: the round's count (rows = min(n, count), as on the device)."""
        import ctypes
        if n_dev is not None:
            n = min(int(n), int(n_dev.reshape(-1)[0]))
        if not n:
            return
        i = np.ctypeslib.as_array((ctypes.c_int64 * n).from_address(idx_ptr)).copy()
        th, lp, anc, x, d = self._rows(lo, int(i.max()) + 1)
        for ptr, a, dt in zip(ptrs, (th, lp, anc, x, d),
                              (np.float64, np.float64, np.int64, np.float64, np.float64)):
            r = np.ascontiguousarray(a[i], dtype=dt)
            ctypes.memmove(ptr, r.ctypes.data, r.nbytes)


def _run(n, eps, batch, record, fused=False, nan_first=False):
    """fused: False (staged distance + compaction), True (fused rounds) or
    "tail" (staged rounds with the accept tail); nan_first: the first fused
    round gets an undecided (NaN) device threshold."""
    from pyabc_amd.sampler import BatchedGPUSampler
    s = BatchedGPUSampler(batch_size=batch, seed=SEED, fused=fused is True)
    if fused is True:
        s._fused_round = lambda spec, seed, gen, dev: _FusedRound(spec)
    s.sample_factory.record_rejected = record
    sample = s.sample_until_n_accepted(n, _Spec(eps, tail=fused == "tail",
                                                nan_first=nan_first))
    c = sample._cols
    rec = sample._recorded
    return dict(theta=c.theta.numpy(), w=c.weights.numpy(),
                d=c.distances.numpy(), x=c.sum_stats.numpy(),
                n_eval=np.array(s.nr_evaluations_),
                rounds=np.array(s.last_stats["rounds"]),
                reruns=np.array(s.last_stats.get("quantile_reruns", 0)),
                rec=(rec.numpy() if rec is not None else np.zeros(0)))


def _count_collectives():
    """Wrap the all-gathers the sampler may call; returns the call counter."""
    calls = {"n": 0}
    for name in ("all_gather", "all_gather_into_tensor"):
        f = getattr(dist, name)

        def wrapped(*a, _f=f, **k):
            calls["n"] += 1
            return _f(*a, **k)
        setattr(dist, name, wrapped)
    return calls


def _worker(rank, ws, port, out_dir, n, eps, batch, record, fused=False, nan_first=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        _install_cpu_doubles(setattr)
        calls = _count_collectives()
        res = _run(n, eps, batch, record, fused, nan_first)
        res["collectives"] = np.array(calls["n"])
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fused", [False, True, "tail"])
@pytest.mark.parametrize("n,batch,record,ws", [(300, 256, True, 2), (37, 64, False, 2),
                                               (1, 128, True, 2), (300, 128, True, 4),
                                               (5, 64, True, 4)])
def test_sharded_sampler_matches_single_rank(monkeypatch, n, batch, record, ws, fused):
    """Staged and fused sampler loops: 2 and 4 gloo ranks == 1 rank, and the
    fused loop == the staged loop (same streams, same cutoff).  n = 1 and 5
    leave the later ranks with no kept rows.  Collectives: one count gather
    per round, then ONE packed row gather that also carries the cutoff
    position (+ one for the recorded rows)."""
    eps = 1.6
    _install_cpu_doubles(monkeypatch.setattr)
    ref = _run(n, eps, batch * ws, record, fused)  # 1 rank, same global round size
    if fused:
        staged = _run(n, eps, batch * ws, record, False)   # fused / tail == staged
        for k in ("theta", "w", "d", "x", "n_eval", "rec"):
            np.testing.assert_array_equal(ref[k], staged[k], err_msg=k)
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(ws, _free_port(), tmp, n, eps, batch,
                                          record, fused),
                           nprocs=ws, join=True, start_method="spawn")
        for rank in range(ws):
            got = dict(np.load(os.path.join(tmp, f"r{rank}.npz")))
            assert int(got["n_eval"]) == int(ref["n_eval"])
            assert int(got["collectives"]) == int(got["rounds"]) + 1 + int(record)
            for k in ("theta", "w", "d", "x"):
                assert got[k].shape[0] == n
                np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
            if record:
                np.testing.assert_array_equal(got["rec"], ref["rec"])
    # the cutoff keeps exactly the first n accepted in global index order
    assert np.all(ref["d"] <= eps)


@pytest.mark.parametrize("n,batch,record", [(300, 256, True), (37, 64, False)])
def test_sharded_fused_quantile_rerun(monkeypatch, n, batch, record):
    """The fused loop's first round at an undecided (NaN) device quantile
    (batched.py: the round accepts nothing and the same candidates run again
    at the host value): 1 and 2 ranks equal the staged loop -- population,
    evaluations, recorded rows -- with one re-run counted
    (last_stats["quantile_reruns"]) and its count gather the only extra
    collective."""
    eps, ws = 1.6, 2
    _install_cpu_doubles(monkeypatch.setattr)
    ref = _run(n, eps, batch * ws, record, True, nan_first=True)
    staged = _run(n, eps, batch * ws, record, False)
    assert int(ref["reruns"]) == 1
    for k in ("theta", "w", "d", "x", "n_eval", "rec"):
        np.testing.assert_array_equal(ref[k], staged[k], err_msg=k)
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(ws, _free_port(), tmp, n, eps, batch,
                                          record, True, True),
                           nprocs=ws, join=True, start_method="spawn")
        for rank in range(ws):
            got = dict(np.load(os.path.join(tmp, f"r{rank}.npz")))
            assert int(got["reruns"]) == 1
            assert int(got["n_eval"]) == int(ref["n_eval"])
            assert int(got["collectives"]) == int(got["rounds"]) + 2 + int(record)
            for k in ("theta", "w", "d", "x"):
                np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
            if record:
                np.testing.assert_array_equal(got["rec"], ref["rec"])


def _collective_worker(rank, ws, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from pyabc_amd.sampler import distributed as dd
        dev = torch.device("cpu")
        assert dd.world() == (rank, ws)
        counts = dd.allgather_counts(10 * rank + 3, dev)
        rows = torch.full((rank + 1, 2), float(rank), dtype=torch.float64)
        gathered = dd.allgather_rows(rows, dev)
        empty = dd.allgather_rows(torch.zeros((0, 2), dtype=torch.float64), dev)
        b = dd.broadcast_int(99 if rank == 0 else -1, dev)
        # packed ordered gather: 3 rounds, rank 1 keeps nothing in round 1,
        # rank 0 nothing in round 2; rows carry their global order number
        keeps = np.array([[2, 1], [3, 0], [0, 2]])
        order = np.arange(keeps.sum()).reshape(-1)
        mine, o = [], 0
        for r in range(keeps.shape[0]):
            for q in range(ws):
                if q == rank:
                    mine.extend(order[o:o + keeps[r, q]])
                o += keeps[r, q]
        g = torch.tensor(mine, dtype=torch.float64)
        th = torch.stack([g, -g], 1)
        t2, w2, x2 = dd.allgather_rows_ordered(
            [th, g + 0.5, torch.stack([g, g, g], 1).reshape(-1, 3, 1)], keeps, dev)
        e1, e2 = dd.allgather_rows_ordered(
            [torch.zeros((0, 2), dtype=torch.float64),
             torch.zeros(0, dtype=torch.float64)], np.zeros((1, ws)), dev)
        np.savez(os.path.join(out_dir, f"c{rank}.npz"), counts=counts,
                 gathered=gathered.numpy(), empty=np.array(empty.shape),
                 b=np.array(b), t2=t2.numpy(), w2=w2.numpy(), x2=x2.numpy(),
                 e=np.array(list(e1.shape) + list(e2.shape)))
    finally:
        dist.destroy_process_group()


def test_collectives_two_ranks():
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_collective_worker, args=(2, _free_port(), tmp),
                           nprocs=2, join=True, start_method="spawn")
        for rank in range(2):
            r = np.load(os.path.join(tmp, f"c{rank}.npz"))
            np.testing.assert_array_equal(r["counts"], [3, 13])
            np.testing.assert_array_equal(r["gathered"],
                                          [[0, 0], [1, 1], [1, 1]])
            np.testing.assert_array_equal(r["empty"], [0, 2])
            assert int(r["b"]) == 99
            g = np.arange(8, dtype=np.float64)
            np.testing.assert_array_equal(r["t2"], np.stack([g, -g], 1))
            np.testing.assert_array_equal(r["w2"], g + 0.5)
            assert r["x2"].shape == (8, 3, 1)
            np.testing.assert_array_equal(r["x2"][:, :, 0], np.stack([g] * 3, 1))
            np.testing.assert_array_equal(r["e"], [0, 2, 0])


def test_allgather_rows_ordered_single_rank():
    """Without a process group the packed gather is the identity (ws = 1)."""
    from pyabc_amd.sampler import distributed as dd
    a = torch.arange(6, dtype=torch.float64).reshape(3, 2)
    b = torch.arange(3, dtype=torch.float64)
    out = dd.allgather_rows_ordered([a, b], np.array([[2], [1]]), torch.device("cpu"))
    assert out[0] is a and out[1] is b
    t = dd.allgather_counts(torch.tensor([7]), torch.device("cpu"))
    np.testing.assert_array_equal(t, [7])


def test_cutoff_prefix():
    from pyabc_amd.sampler.distributed import cutoff, rank_range
    np.testing.assert_array_equal(cutoff([5, 7, 2], 9), [5, 4, 0])
    np.testing.assert_array_equal(cutoff([0, 0], 3), [0, 0])
    np.testing.assert_array_equal(cutoff([4, 4], 8), [4, 4])
    assert rank_range(100, 10, 3) == (130, 140)


def _nccl_branch_worker(rank, ws, port, out_dir):
    """The sampler's collectives with dist.get_backend() reporting "nccl",
    so all_gather_flat takes its RCCL branch (no host staging: the tensors
    go to all_gather_into_tensor as given); a gloo stand-in underneath
    checks every call the way RCCL would take it -- contiguous buffers of
    one dtype on one device, out = world_size x the input along dim 0 --
    then performs it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    calls = []
    real_into, real_list = dist.all_gather_into_tensor, dist.all_gather
    try:
        from pyabc_amd.sampler import distributed as dd

        def into(out, t, *a, **k):
            assert out.is_contiguous() and t.is_contiguous()
            assert out.dtype == t.dtype and out.device == t.device
            assert out.shape[0] == ws * t.shape[0] and out.shape[1:] == t.shape[1:]
            calls.append(("into", tuple(t.shape), str(t.dtype)))
            return real_into(out, t, *a, **k)

        def lst(outs, t, *a, **k):
            assert len(outs) == ws and t.is_contiguous()
            assert all(o.shape == t.shape and o.dtype == t.dtype for o in outs)
            calls.append(("list", tuple(t.shape), str(t.dtype)))
            return real_list(outs, t, *a, **k)
        dist.all_gather_into_tensor, dist.all_gather = into, lst
        dist.get_backend = lambda *a, **k: "nccl"
        dev = torch.device("cpu")
        # ragged keeps over 3 rounds: ranks with nothing in a round, one rank
        # with nothing at all; rows carry their global order number
        rng = np.random.default_rng(ws)
        keeps = rng.integers(0, 4, (3, ws))
        keeps[:, ws - 1] = 0
        keeps[1, 0] = 0
        order = np.arange(keeps.sum())
        mine, o = [], 0
        for r in range(keeps.shape[0]):
            for q in range(ws):
                if q == rank:
                    mine.extend(order[o:o + keeps[r, q]])
                o += keeps[r, q]
        g = torch.tensor(mine, dtype=torch.float64).reshape(-1)
        cols = [torch.stack([g, -g], 1), g + 0.5, torch.stack([g] * 4, 1)]
        (th, w, x), ex = dd.allgather_rows_ordered(
            cols, keeps, dev, extra=torch.tensor([float(100 + rank)], dtype=torch.float64))
        counts = dd.allgather_counts(torch.tensor([5 * rank + 1]), dev)
        np.savez(os.path.join(out_dir, f"n{rank}.npz"), th=th.numpy(), w=w.numpy(),
                 x=x.numpy(), ex=ex, counts=counts, n=np.array(len(order)),
                 calls=np.array([f"{a}:{b}:{c}" for a, b, c in calls]))
    finally:
        dist.all_gather_into_tensor, dist.all_gather = real_into, real_list
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 8])
def test_nccl_branch_collectives(ws):
    """The RCCL code path of the packed row gather and the count gather
    (sampler/distributed.py all_gather_flat with backend "nccl") at world
    size 2 and 8, through a gloo stand-in that asserts RCCL's buffer
    contract on every call: one all_gather_into_tensor of the packed
    [rows x (2 + 1 + 4)] f64 buffer (+ the cutoff row), one list all_gather
    of the int64 counts; every rank gets the rows in global order and the
    extras in rank order."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_nccl_branch_worker, args=(ws, _free_port(), tmp),
                           nprocs=ws, join=True, start_method="spawn")
        for rank in range(ws):
            r = np.load(os.path.join(tmp, f"n{rank}.npz"))
            g = np.arange(int(r["n"]), dtype=np.float64)
            np.testing.assert_array_equal(r["th"], np.stack([g, -g], 1))
            np.testing.assert_array_equal(r["w"], g + 0.5)
            np.testing.assert_array_equal(r["x"], np.stack([g] * 4, 1))
            np.testing.assert_array_equal(r["ex"], 100.0 + np.arange(ws))
            np.testing.assert_array_equal(r["counts"], 5 * np.arange(ws) + 1)
            calls = list(r["calls"])
            assert [c.split(":")[0] for c in calls] == ["into", "list"], calls
            assert calls[0].endswith("torch.float64") and calls[1].endswith("torch.int64")
