"""Rank bookkeeping for the multi-GPU batched sampler.

One process per GPU, ``torch.distributed`` with the nccl (= RCCL) backend on
MI355X; the same code runs on gloo for CPU tests.  Candidates are sharded by
global index: round r covers [base, base + R*B) and rank k evaluates
[base + k*B, base + (k+1)*B).  Because every random draw is keyed by the
global index, the first-n-accepted cutoff -- and so the whole population --
is identical for 1, 2, 4 or 8 ranks.

Collectives per generation (all RCCL over xGMI on the GPU box):
  * all_gather of per-round accept counts (R int64) -> global cutoff,
  * all_gather of the accepted rows (theta, weight, distance, sum stats) ->
    the next population, replicated on every rank,
  * all_gather of the recorded sum stats when the distance adapts.
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
    """int count per rank -> numpy array [world] (rank order)."""
    rank, ws = world()
    if ws == 1:
        return np.array([int(count)])
    t = torch.tensor([int(count)], dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    return torch.cat(out).cpu().numpy()      # one host read


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


def broadcast_int(v, device):
    rank, ws = world()
    if ws == 1:
        return int(v)
    t = torch.tensor([int(v)], dtype=torch.int64, device=device)
    dist.broadcast(t, 0)
    return int(t.item())
