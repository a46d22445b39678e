"""Dump the dense-k bracket [T_lo, T_hi) of the c5 fit (k = N/4) from the
fit workspace (sel_v, sel_jcut: its first two carved arrays) to an npz, to
compare two builds (probe):  ABCGPU_LIB=... python tools/probes/c5_bracket_dump.py OUT.npz"""
import sys

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, "/root/repo")
from pyabc_amd import gpu  # noqa: E402
from pyabc_amd.transition import LocalTransition  # noqa: E402

rng = np.random.default_rng(99)
N, d = 100_000, 5
X = rng.standard_normal((N, d))
w = np.full(N, 1.0 / N)
t = LocalTransition()
t.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(d)]), w.copy())
torch.cuda.synchronize()
ws = gpu._ws[(torch.cuda.current_device(), "local")]
off2 = ((N * 8 + 255) // 256) * 256
v = ws[:N * 8].view(torch.float64).cpu().numpy()
j = ws[off2:off2 + N * 8].view(torch.float64).cpu().numpy()
np.savez(sys.argv[1], tlo=v, thi=j)
fin = np.isfinite(v)
print(sys.argv[1], "finite brackets", fin.sum(), "median width", np.median((j - v)[fin & np.isfinite(j)]))
