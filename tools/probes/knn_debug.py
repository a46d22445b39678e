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
lm = dg[:, 12]
print("listmode frac", lm.mean(), "fail frac", dg[:, 0].mean())
nl = np.nonzero(lm == 0)[0]
print("non-list particles", len(nl), "first", nl[:20])
blk = nl // 16
for b in np.unique(blk)[:5]:
    print("block", b); print(dg[16 * b: 16 * b + 16, [0, 1, 2, 3, 4, 10, 11, 13]])
