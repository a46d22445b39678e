"""RCCL communicator over the C ABI (abc_comm_*, include/abcgpu.h).

The multi-GPU sampler's collectives (pyabc_amd/sampler/distributed.py) go
through torch.distributed by default (backend "nccl" is RCCL on ROCm).  This
class is the same transport without torch.distributed's process-group layer:
one RCCL communicator per process, device buffers handed over as pointers on
the current stream.  `distributed.use_comm(RcclComm.from_process_group())`
routes the sampler's flat all-gathers through it.

The reference has no counterpart: MulticoreEvalParallelSampler
(multicore_evaluation_parallel.py:92-150) shares one evaluation counter
between forked workers on one host.
"""
import ctypes as C

from .. import _native as nat
from .. import gpu


class RcclComm:
    """One RCCL communicator: `nranks` processes, this one `rank`, all
    initialised from the same 128-byte unique id (rank 0's
    `RcclComm.unique_id()`, moved to the others by any channel)."""

    def __init__(self, rank, nranks, uid):
        if len(uid) != nat.ABC_COMM_ID_BYTES:
            raise ValueError("RcclComm: unique id must be 128 bytes")
        self.rank, self.nranks = int(rank), int(nranks)
        h = C.c_void_p()
        nat.call("abc_comm_init", C.addressof(h), self.nranks, self.rank,
                 C.create_string_buffer(bytes(uid), nat.ABC_COMM_ID_BYTES))
        self._h = h

    @staticmethod
    def unique_id():
        buf = C.create_string_buffer(nat.ABC_COMM_ID_BYTES)
        nat.call("abc_comm_unique_id", buf)
        return buf.raw

    @classmethod
    def from_process_group(cls):
        """Rank 0 draws the id; torch.distributed's default group (gloo or
        nccl) broadcasts it."""
        import torch.distributed as dist
        rank, ws = dist.get_rank(), dist.get_world_size()
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return cls(rank, ws, box[0])

    def _live(self):
        if self._h is None:
            raise RuntimeError("RcclComm: communicator closed")
        return self._h

    def all_gather_into(self, out, t):
        """out [nranks * n, ...] = the ranks' t [n, ...] in rank order (device
        tensors, contiguous, same dtype)."""
        if not (t.is_cuda and out.is_cuda and t.is_contiguous() and out.is_contiguous()):
            raise ValueError("RcclComm.all_gather_into: contiguous device tensors")
        if out.dtype != t.dtype or out.numel() != t.numel() * self.nranks:
            raise ValueError("RcclComm.all_gather_into: out must hold nranks x t")
        nbytes = t.numel() * t.element_size()
        nat.call("abc_comm_allgather", self._live(), gpu.p(t), gpu.p(out), nbytes,
                 gpu.stream_ptr())
        return out

    def all_reduce(self, t, op="sum"):
        """In place; float64 or int64 device tensors."""
        torch = gpu.torch
        dt = {torch.float64: nat.ABC_COMM_F64, torch.int64: nat.ABC_COMM_I64}.get(t.dtype)
        if dt is None or not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm.all_reduce: contiguous float64 / int64 device tensor")
        o = {"sum": nat.ABC_COMM_SUM, "max": nat.ABC_COMM_MAX, "min": nat.ABC_COMM_MIN}[op]
        nat.call("abc_comm_allreduce", self._live(), gpu.p(t), gpu.p(t), t.numel(), dt, o,
                 gpu.stream_ptr())
        return t

    def broadcast(self, t, root=0):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm.broadcast: contiguous device tensor")
        nat.call("abc_comm_broadcast", self._live(), gpu.p(t), t.numel() * t.element_size(),
                 int(root), gpu.stream_ptr())
        return t

    def close(self):
        if self._h is not None:
            nat.call("abc_comm_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
