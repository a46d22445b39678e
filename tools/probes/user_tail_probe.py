"""The staged path of a user VectorizedModel at c2's shape (d = S = 10):
abc_candidates_propose (theta rows for the user's simulator) and
abc_pnorm_accept (p-norm + accept bits + compaction) on B = 4M candidates,
HIP-event times, candidates/s and the HBM rate of their algorithmic bytes.
tools/probes, not part of the library."""
import numpy as np
import torch

from pyabc_amd import gpu

dev = gpu.require_device()
d = S = 10
N, B = 100_000, 1 << 22
g = torch.Generator(device="cpu").manual_seed(0)
X = (0.8 + np.sqrt(0.2) * torch.randn(N, d, generator=g, dtype=torch.float64)).to(dev)
w = torch.exp(2.2 * torch.randn(N, generator=g, dtype=torch.float64)).to(dev)
w /= w.sum()
L = torch.eye(d, dtype=torch.float64, device=dev) * 0.1
cdf = gpu.inclusive_scan(w)
guide = gpu.cdf_guide(cdf)
kind = torch.zeros(d, dtype=torch.int32, device=dev)
params = torch.tensor(np.tile([0.0, 1.0, 0, 0], d), dtype=torch.float64, device=dev)
src = torch.arange(S, dtype=torch.int32, device=dev) % d
one = torch.ones(S, dtype=torch.float64, device=dev)
half = torch.full((S,), 0.5, dtype=torch.float64, device=dev)
fr = gpu.CandidateRound(d, S, kind, params, src, one, half, one.clone(), one.clone(),
                        2.0, 7, 5, 10000, X=X, cdf=cdf, guide=guide, L=L)


def timed(fn, reps=5):
    ts = []
    for r in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        e1.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), out


ms, (th, lp, anc, att) = timed(lambda: fr.propose(0, B))
print(f"propose  B={B}: {ms:.3f} ms -> {B / ms * 1e3:.3e} cand/s, "
      f"{B * (8 * d + 8 + 8 + 4) / ms / 1e9:.2f} TB/s written", flush=True)
try:
    ms, _ = timed(lambda: fr.propose(0, B, with_lp=False))
    print(f"propose (no lp) B={B}: {ms:.3f} ms -> {B / ms * 1e3:.3e} cand/s, "
          f"{B * (8 * d + 8 + 4) / ms / 1e9:.2f} TB/s written", flush=True)
except ValueError as e:          # a library without the optional output
    print("propose (no lp): unsupported:", e)
x = th + 0.5 * torch.randn_like(th)
dist = gpu.pnorm(x, one, one, 2.0)
eps = float(torch.quantile(dist[:1 << 20], 1e-3))
ms, _ = timed(lambda: gpu.pnorm_accept(x, one, one, 2.0, eps, 1 << 16, att=att,
                                       max_attempts=10000))
print(f"pnorm_accept B={B}: {ms:.3f} ms -> {B / ms * 1e3:.3e} cand/s, "
      f"{B * 8 * S / ms / 1e9:.2f} TB/s read", flush=True)
