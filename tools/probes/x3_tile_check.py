"""Which candidate tiles does the x3 density get wrong?  x3 vs the f64-MFMA mode
(2e-6) on random populations; prints the wrong candidate tiles per shape.
ABCGPU_LIB selects the library.  tools/probes, not part of the library."""
import sys

import numpy as np
import pandas as pd

from pyabc_amd import gpu
from pyabc_amd.transition import MultivariateNormalTransition

gpu.require_device()
bad_total = 0
for d, N, M in [(1, 1000, 256), (1, 1000, 1000), (2, 500, 256), (5, 4096, 512),
                (10, 4096, 512), (11, 2000, 300), (12, 2000, 300)]:
    rng = np.random.default_rng(d * 1000 + N)
    cols = [f"p{k}" for k in range(d)]
    X = pd.DataFrame(rng.normal(size=(N, d)), columns=cols)
    w = rng.random(N)
    x = pd.DataFrame(rng.normal(size=(M, d)) * 1.3, columns=cols)
    res = {}
    for prec in ("x3", "f64"):
        t = MultivariateNormalTransition(precision=prec)
        t.fit(X, w.copy())
        res[prec] = np.asarray(t.pdf(x))
        if prec == "x3":
            # hinted pass (the sampler's path): nearest population row
            import torch
            dx = x.to_numpy()[:, None, :] - X.to_numpy()[None, :, :]
            near = np.argmin((dx ** 2).sum(-1), axis=1)
            xd = torch.as_tensor(x.to_numpy(), device="cuda")
            hd = torch.as_tensor(near, dtype=torch.int64, device="cuda")
            res["x3h"] = np.exp(t.logpdf_device(xd, hint=hd).cpu().numpy())
    relh = np.abs(res["x3h"] / res["f64"] - 1)
    wh = np.nonzero(relh > 1e-5)[0]
    bad_total += len(wh)
    print(f"  hinted: {len(wh)} wrong, tiles {sorted(set((wh // 16).tolist()))[:20]}")
    rel = np.abs(res["x3"] / res["f64"] - 1)
    wrong = np.nonzero(rel > 1e-5)[0]
    bad_total += len(wrong)
    tiles = sorted(set((wrong // 16).tolist()))
    print(f"d={d} N={N} M={M}: {len(wrong)} wrong, tiles {tiles[:20]}, "
          f"max rel {rel.max():.3g}, ratio@first "
          f"{(res['x3'][wrong[0]] / res['f64'][wrong[0]]) if len(wrong) else 1:.4g}",
          flush=True)
print("TOTAL WRONG", bad_total)
