"""Rank bookkeeping for the multi-GPU batched sampler.

One process per GPU, ``torch.distributed`` with the nccl (= RCCL) backend on
MI355X; the same code runs on gloo for CPU tests.  Candidates are sharded by
global index: round r covers [base, base + R*B) and rank k evaluates
[base + k*B, base + (k+1)*B).  Because every random draw is keyed by the
global index, the first-n-accepted cutoff -- and so the whole population --
is identical for 1, 2, 4 or 8 ranks.

Collectives per generation (all RCCL over xGMI on the GPU box):
  * all_gather of per-round accept counts (R int64) -> global cutoff
    (computed on the device before the host reads the counts),
  * ONE all_gather of the accepted rows (theta, weight, distance, sum stats
    packed column-wise) -> the next population, replicated on every rank;
    row counts come from the cutoff every rank already holds,
  * one all_gather of the recorded rows when the distance adapts (or the
    temperature needs every record).
"""
import numpy as np

try:
    import torch
    import torch.distributed as dist
except ImportError:  # pragma: no cover
    torch = None
    dist = None


def world():
    """(rank, world_size) of the default group, (0, 1) when not initialised."""
    if dist is not None and dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def rank_range(base, B, rank):
    """Global index range [lo, hi) of ``rank`` in the round starting at base."""
    return base + rank * B, base + (rank + 1) * B


def allgather_counts(count, device):
    """int count (or a 1-element device tensor, read by no one but the
    collective) per rank -> numpy array [world] (rank order)."""
    rank, ws = world()
    if isinstance(count, torch.Tensor):
        t = count.reshape(1).to(torch.int64)
        if ws == 1:
            return t.cpu().numpy()
    else:
        if ws == 1:
            return np.array([int(count)])
        t = torch.tensor([int(count)], dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    return torch.cat(out).cpu().numpy()      # one host read


def allgather_counts_device(count):
    """A 1-element device count per rank -> device int64 tensor [world] in
    rank order, with no host read (RCCL gathers on the stream; gloo stages
    through the host inside the collective).  The multi-rank fused round
    computes its cutoff from it on the device (gpu.round_keep) and reads it
    on the host only afterwards."""
    rank, ws = world()
    t = count.reshape(1).to(torch.int64)
    if ws == 1:
        return t
    out = torch.empty(ws, dtype=torch.int64, device=t.device)
    all_gather_flat(out, t)
    return out


def cutoff(counts, needed):
    """Given per-rank accepted counts of one round (rank order = global
    index order) and the number still needed, return how many accepted
    candidates each rank keeps (prefix in rank order)."""
    keep = np.zeros(len(counts), dtype=np.int64)
    left = int(needed)
    for k, c in enumerate(counts):
        take = min(int(c), left)
        keep[k] = take
        left -= take
    return keep


def allgather_rows(t, device):
    """Concatenate a per-rank tensor [n_k, ...] over ranks in rank order
    (variable n_k: padded to the max, then trimmed)."""
    rank, ws = world()
    if ws == 1:
        return t
    n = allgather_counts(t.shape[0], device)
    nmax = int(n.max())
    shape = (nmax,) + tuple(t.shape[1:])
    pad = torch.zeros(shape, dtype=t.dtype, device=t.device)
    if t.shape[0]:
        pad[: t.shape[0]] = t
    out = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(out, pad)
    return torch.cat([o[: int(k)] for o, k in zip(out, n)], dim=0)


def allgather_rows_ordered(tensors, keeps, device, extra=None):
    """All-gather several per-rank row blocks in ONE collective and return
    them in global candidate-index order.

    ``extra``: an optional 1-element f64 tensor per rank (the sampler's
    cutoff position of the generation's last round) carried in one more row
    of the same collective; the call then returns (rows, extras[ws]).

    tensors: list of same-dtype tensors [n_mine, c_i] or [n_mine] with the
    same leading size (this rank's rows, round after round); keeps: [rounds x
    ranks] rows each rank contributed per round -- known identically on every
    rank from the cutoff, so no count exchange (and no host read) is needed.
    The columns are packed into one [nmax x sum(c_i)] buffer (padded to the
    largest rank), gathered with one all_gather, and the pieces (round-major,
    then rank) are cut straight from the padded result: one collective and
    one concatenation instead of a count gather + row gather + trim + reorder
    per tensor.
    """
    rank, ws = world()
    k = np.asarray(keeps, dtype=np.int64).reshape(len(keeps), -1)
    if ws == 1:
        if extra is not None:
            return list(tensors), extra.reshape(1).to(torch.float64).cpu().numpy()
        return list(tensors)
    per_rank = k.sum(0)
    nmax = int(per_rank.max()) if per_rank.size else 0
    if len({t.dtype for t in tensors}) != 1:
        raise TypeError("allgather_rows_ordered packs one dtype per call")
    cols = [t.reshape(t.shape[0], int(np.prod(t.shape[1:], dtype=np.int64)))
            for t in tensors]
    widths = [c.shape[1] for c in cols]
    C = int(sum(widths))
    n_mine = cols[0].shape[0]
    if n_mine != int(per_rank[rank]):
        raise AssertionError(
            f"rank {rank}: {n_mine} rows, cutoff says {int(per_rank[rank])}")
    rows = max(nmax, 1) + (1 if extra is not None else 0)
    pad = torch.zeros((rows, C), dtype=cols[0].dtype, device=cols[0].device)
    c0 = 0
    for c, wdt in zip(cols, widths):
        if n_mine:
            pad[:n_mine, c0:c0 + wdt] = c
        c0 += wdt
    if extra is not None:
        pad[rows - 1, :1] = extra.reshape(1).to(pad.dtype)
    out = torch.empty((ws * pad.shape[0], C), dtype=pad.dtype, device=pad.device)
    all_gather_flat(out, pad)
    # piece (round r, rank q) starts at q * nmax + rows q kept in rounds < r
    round_off = np.cumsum(k, axis=0) - k
    pieces = [(int(q * pad.shape[0] + round_off[r, q]), int(k[r, q]))
              for r in range(k.shape[0]) for q in range(ws) if k[r, q] > 0]
    if not pieces:
        full = out[:0]
    else:
        full = torch.cat([out[a:a + n] for a, n in pieces], 0)
    res, c0 = [], 0
    for t, wdt in zip(tensors, widths):
        piece = full[:, c0:c0 + wdt]
        res.append(piece.reshape((full.shape[0],) + tuple(t.shape[1:])).contiguous())
        c0 += wdt
    if extra is not None:
        ex = out.view(ws, rows, C)[:, rows - 1, 0].cpu().numpy()
        return res, ex
    return res


_comm = None


def use_comm(comm):
    """Route the flat all-gathers of device tensors through `comm` (an
    RcclComm over the C ABI's abc_comm_*) instead of torch.distributed;
    None restores torch.distributed."""
    global _comm
    _comm = comm


def all_gather_flat(out, t):
    """dist.all_gather_into_tensor(out, t) on every backend: RCCL (nccl)
    gathers device tensors directly; gloo, whose flat all-gather takes host
    tensors only, gets host copies (multi-rank runs on one GPU, CPU tests).
    The caller's packing and cutting are the same code either way.  With
    use_comm(RcclComm) device tensors go through libabcgpu's RCCL wrappers."""
    if _comm is not None and t.is_cuda:
        return _comm.all_gather_into(out, t.contiguous())
    # one collective call for every backend; only gloo with device tensors
    # stages through host buffers
    staged = t.is_cuda and dist.get_backend() == "gloo"
    src = t.cpu() if staged else t
    dst = torch.empty(out.shape, dtype=out.dtype) if staged else out
    dist.all_gather_into_tensor(dst, src)
    if staged:
        out.copy_(dst)
    return out


def broadcast_object(obj):
    """Rank 0's picklable object on every rank (the per-candidate fallback
    of BatchedGPUSampler runs on rank 0 only)."""
    rank, ws = world()
    if ws == 1:
        return obj
    box = [obj if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def broadcast_int(v, device):
    rank, ws = world()
    if ws == 1:
        return int(v)
    t = torch.tensor([int(v)], dtype=torch.int64, device=device)
    dist.broadcast(t, 0)
    return int(t.item())
