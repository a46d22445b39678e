"""RCCL collectives over the C ABI (abc_comm_*, pyabc_amd/sampler/comm.py).

One GPU per process and one GPU per box here, so the communicator runs with
one rank: the collectives' data paths are identities (all-gather = copy,
all-reduce = the input, broadcast = the input) and check the binding, the
pointer/stream plumbing and the sampler's transport switch.  Multi-rank RCCL
rejects two ranks on one device; the multi-rank packing and cutting logic is
covered by the gloo tests (tests/test_distributed_gloo.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def comm():
    from pyabc_amd import gpu
    from pyabc_amd.sampler.comm import RcclComm
    gpu.require_device()
    c = RcclComm(0, 1, RcclComm.unique_id())
    yield c
    c.close()


def test_single_rank_collectives(comm):
    dev = torch.device("cuda")
    x = torch.arange(1000, dtype=torch.float64, device=dev) * 0.5
    out = torch.empty_like(x)
    comm.all_gather_into(out, x)
    assert torch.equal(out, x)
    y = x.clone()
    for op in ("sum", "max", "min"):
        comm.all_reduce(y, op)
    assert torch.equal(y, x)
    k = torch.arange(7, dtype=torch.int64, device=dev)
    comm.all_reduce(k)
    assert torch.equal(k, torch.arange(7, dtype=torch.int64, device=dev))
    b = x.clone()
    comm.broadcast(b, 0)
    assert torch.equal(b, x)
    with pytest.raises(ValueError):
        comm.all_gather_into(torch.empty(3, dtype=torch.float64, device=dev), x)


def test_sampler_transport_switch(comm):
    """distributed.all_gather_flat routes device tensors through the
    communicator once use_comm is set."""
    from pyabc_amd.sampler import distributed as dd
    dev = torch.device("cuda")
    t = torch.randn(33, 5, dtype=torch.float64, device=dev)
    out = torch.empty_like(t)
    dd.use_comm(comm)
    try:
        dd.all_gather_flat(out, t)
    finally:
        dd.use_comm(None)
    assert torch.equal(out, t)
