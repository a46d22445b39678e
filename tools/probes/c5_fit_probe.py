import sys, numpy as np, pandas as pd, torch
sys.path.insert(0, "/root/repo")
from pyabc_amd.transition import LocalTransition
rng = np.random.default_rng(99)
N, d = 100_000, 5
X = rng.standard_normal((N, d))
w = np.full(N, 1.0 / N)
t = LocalTransition(k=50, k_fraction=None)
for _ in range(3):
    t.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(d)]), w.copy())
torch.cuda.synchronize()
