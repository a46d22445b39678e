"""Per-phase clock64 cycles of knn_select_kernel (build with
-DABC_KNN_TIMING): sample+sort, count sweep, bin scan, collect sweep,
select; mean over blocks (wave 0, thread 0)."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
from pyabc_amd import gpu  # noqa: E402
rng = np.random.default_rng(99)
N, d = 100_000, 5
X = rng.standard_normal((N, d))
w = np.full(N, 1.0 / N)
for k in (50, 25000):
    for _ in range(2):
        covs = gpu.local_fit(gpu.as_dev(X), gpu.as_dev(w), k, 1.0, 1e-3)[0]
    nb = (N + 15) // 16
    t = covs.reshape(-1)[: 8 * nb].reshape(nb, 8).cpu().numpy()[:, 1:6]
    print(f"k={k}: cycles per phase (mean over blocks):",
          dict(zip(["sample+sort", "count", "binscan", "collect", "select"],
                   np.round(t.mean(0)).astype(int))))
