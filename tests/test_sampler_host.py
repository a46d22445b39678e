"""Host-side decisions of the batched sampler (no GPU): when a fused round
may take the lazy early reject (BatchedGPUSampler._lazy_capable mirrors the
device-side lazy_filter_ok preconditions of abc_candidate.h; the kernel
re-checks the support bound exactly), and the round sizing."""
import math
import types

import pytest

from pyabc_amd._native import PRIOR_KINDS
from pyabc_amd.sampler.batched import BatchedGPUSampler


def _fr(d=10, S=10, p=2.0, X=1, ppl=0, src=None):
    spec = types.SimpleNamespace(X=X, per_particle_L=ppl, d=d, S=S, p=p)
    return types.SimpleNamespace(spec=spec, src_host=list(range(S)) if src is None else src)


def _gen(kinds=("norm",) * 10):
    return types.SimpleNamespace(prior_kind_host=tuple(PRIOR_KINDS[k] for k in kinds))


@pytest.mark.parametrize("case,ok", [
    (dict(), True),
    (dict(p=1.0), True),
    (dict(p=math.inf), True),
    (dict(p=3.0), False),                 # partial p-norm not monotone-exact
    (dict(X=None), False),                # t = 0: prior proposals
    (dict(ppl=1), False),                 # LocalTransition factors
    (dict(d=4, S=10), False),             # the head is the whole theta
    (dict(S=4), False),                   # the 4 statistics are all of them
    (dict(src=[7, 1, 2, 3, 4, 5, 6, 8, 9, 0]), False),   # stat 0 reads theta_7
])
def test_lazy_capable(case, ok):
    s = BatchedGPUSampler(seed=1, filter_min_stats=5)
    assert s._lazy_capable(_gen(), _fr(**case)) is ok


def test_lazy_capable_priors_and_min_stats():
    s = BatchedGPUSampler(seed=1, filter_min_stats=5)
    assert s._lazy_capable(_gen(("laplace",) * 10), _fr())
    assert not s._lazy_capable(_gen(("uniform",) + ("norm",) * 9), _fr())
    assert not s._lazy_capable(types.SimpleNamespace(), _fr())   # no host kinds
    assert not BatchedGPUSampler(seed=1, filter_min_stats=16)._lazy_capable(_gen(), _fr())
    assert BatchedGPUSampler(seed=1).filter_below == 0.0        # off by default


def test_fused_round_sizing():
    s = BatchedGPUSampler(seed=1)
    # need / rate (+6% once measured) / ranks + 4096, capped by the launch budget;
    # a first round: rate x the last drop, spare min(10%, 4e6 candidates per rank)
    assert s._fused_size(1000, 1, 0.01, False, 10, False) == int(1000 * 100 * 1.1 + 4096)
    s._acc_trend = 0.8
    n, r = 10 ** 7, 0.01
    assert s._fused_size(n, 2, r, False, 10, False) == \
        int(n / (r * 0.8) * (1 + 4e6 * 2 * r * 0.8 / n) / 2 + 4096)
    s._acc_trend = 1.0
    assert s._fused_size(1000, 2, 0.01, True, 10, False) == int(1000 * 100 * 1.06 / 2 + 4096)
    assert s._fused_size(10 ** 9, 1, 1e-6, True, 10, False) == s.max_fused_batch_size
    # record_rejected: rows of S doubles within record_budget_bytes
    assert s._fused_size(10 ** 6, 1, 1e-3, True, 256, True) == s.record_budget_bytes // (8 * 256)


def test_join_rows_view_or_copy():
    """Recorded rows of consecutive fused rounds sit back to back in one
    arena: joined as a view (no copy); anything else is concatenated."""
    torch = pytest.importorskip("torch")
    arena = torch.arange(60, dtype=torch.float64).reshape(20, 3)
    a, b, c = arena[0:5], arena[5:12], arena[12:13]
    j = BatchedGPUSampler._join_rows([a, b, c])
    assert j.data_ptr() == arena.data_ptr() and torch.equal(j, arena[:13])
    gap = BatchedGPUSampler._join_rows([arena[0:5], arena[6:8]])
    assert gap.data_ptr() != arena.data_ptr()
    assert torch.equal(gap, torch.cat([arena[0:5], arena[6:8]]))
    other = torch.zeros(2, 3, dtype=torch.float64)
    assert torch.equal(BatchedGPUSampler._join_rows([a, other]), torch.cat([a, other]))
