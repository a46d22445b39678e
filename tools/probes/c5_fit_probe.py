"""c5 LocalTransition fit (N = 1e5, d = 5) repeated, for rocprofv3 kernel
traces: k = 50 (argv[1] = "50", default) or the default k = N/4 ("quarter")."""
import sys

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, "/root/repo")
from pyabc_amd.transition import LocalTransition  # noqa: E402

rng = np.random.default_rng(99)
N, d = 100_000, 5
X = rng.standard_normal((N, d))
w = np.full(N, 1.0 / N)
quarter = len(sys.argv) > 1 and sys.argv[1] == "quarter"
t = LocalTransition() if quarter else LocalTransition(k=50, k_fraction=None)
for _ in range(3):
    t.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(d)]), w.copy())
torch.cuda.synchronize()
print("ok")
