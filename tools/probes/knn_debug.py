"""Diagnostics of knn_select_kernel (build with -DABC_KNN_DEBUG): per
particle [fail, nest, bincount, listcount, below2, tlo, thi, chi, clo, R2,
lor, sh, listmode, rr, B0, 0] for c5-shaped data."""
import sys
import numpy as np
import torch
sys.path.insert(0, "/root/repo")
from pyabc_amd import gpu  # noqa: E402
rng = np.random.default_rng(99)
N, d = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000, 5
X = rng.standard_normal((N, d))
w = np.full(N, 1.0 / N)
k = int(sys.argv[1]) if len(sys.argv) > 1 else 50
covs = gpu.local_fit(gpu.as_dev(X), gpu.as_dev(w), k, 1.0, 1e-3)[0]
dg = covs.reshape(-1)[: 16 * N].reshape(N, 16).cpu().numpy()
np.set_printoptions(linewidth=200, precision=5, suppress=False)
print("fail frac", dg[:, 0].mean(), "listmode frac", dg[:, 12].mean())
bad = (dg[:, 0] > 0) | (dg[:, 3] > 256) | (dg[:, 13] < 0) | (dg[:, 13] >= np.minimum(dg[:, 3], 256))
print("bad frac", bad.mean())
for i in list(range(3)) + list(np.nonzero(bad)[0][:3]):
    print(i, dg[i])
# keys of particles 0..15 (debug kernel, written into the inverse-covariance
# output): the sweeps' MFMA keys against numpy's fp32 expanded form
inv = gpu.local_fit(gpu.as_dev(X), gpu.as_dev(w), k, 1.0, 1e-3)[1]
keys = inv.reshape(-1)[: 16 * N].reshape(2, 8, N).cpu().numpy()
c = 0.5 * X.min(0) + 0.5 * X.max(0)
y = (X - c).astype(np.float32)
s64 = ((X[None, :8] - X[:, None]) ** 2).sum(-1).T      # [8, N]
rows0 = np.nonzero(((np.arange(N) // 16) % 4) == 0)[0]
rows0 = rows0[rows0 < (N // 128) * 128]
for v, name in ((0, "2-tile"), (1, "1-tile")):
    sel = rows0 if v == 0 else np.arange(N)
    err = np.abs(keys[v][:, sel] - s64[:, sel])
    print(name, "max |s^ - s64|", err.max(), "at", np.unravel_index(err.argmax(), err.shape))
    print("  sample keys", keys[v][0, :8], "s64", s64[0, :8])

for i in range(8):
    h = dg[i, 6] - dg[i, 14]
    print(i, "nest", dg[i, 1], "#{s^ < h}", int((keys[1][i] < h).sum()), "#{s64 < thi}", int((s64[i] < dg[i, 6]).sum()), "list", dg[i, 3])
