"""Debug: LocalTransition bootstrap CV with 2 particles (test_gpu_cv)."""
import numpy as np
import pandas as pd
import pyabc_amd as pa
from pyabc_amd.cv import bootstrap as bs

np.random.seed(1236)
df = pd.DataFrame({"a": np.random.rand(2), "b": np.random.rand(2)})
w = np.ones(2) / 2
tr = pa.LocalTransition()
tr.fit(df, w)
orig = bs._model_cv_device


def dbg(trans, test_trans, n, X, w, N_BOOTSTR, scale):
    from pyabc_amd import gpu
    torch = gpu.torch
    Xt = bs._test_points_device(trans, X)
    cols = list(trans.X.columns)
    unif = torch.full((int(n),), 1.0 / n, dtype=torch.float64, device=Xt.device)
    lds = []
    for b in range(N_BOOTSTR):
        bx = trans.propose_device(int(n))[0]
        test_trans.fit_device(bx, unif, cols)
        ld = test_trans.logpdf_device(Xt).cpu().numpy()
        lds.append(ld)
        if not np.isfinite(ld).all() or ld.max() > 5:
            Xn = bx.cpu().numpy()
            print("n", n, "b", b, "X", Xn.tolist(), "test", Xt.cpu().numpy().tolist(),
                  "dets", test_trans._dev_dets.cpu().numpy().tolist(),
                  "invs", test_trans._dev_inv.cpu().numpy().tolist() if hasattr(test_trans, "_dev_inv") else None,
                  "logdens", ld.tolist())
    print("n", n, "logdens per bootstrap", np.array(lds).round(3).tolist())
    var, cv = gpu.bootstrap_cv(torch.tensor(np.array(lds), device=Xt.device), 
                               bs._test_weights_device(trans, w, Xt.device, Xt.shape[0]), scale=scale)
    print("var", var.cpu().numpy().tolist(), "cv", float(cv))
    return var, cv


bs._model_cv_device = dbg
print(tr.required_nr_samples(.1))
