"""Where the quantile's gather + final kernel spends its time: a variant
library (wall_clock64 stamps in the last block, tools/build_src_variant.sh)
run on N = 1e6 / 1e5 points.

    ABCGPU_LIB=ab/libq_stamp.so python tools/probes/quantile_stamps.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pyabc_amd import gpu, _native  # noqa: E402

lib = ctypes.CDLL(os.environ["ABCGPU_LIB"])
buf = (ctypes.c_ulonglong * 10)()
for N in (1_000_000, 100_000):
    g = torch.Generator(device="cuda").manual_seed(1)
    d = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) * 4 + 1
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g)
    for _ in range(5):
        gpu.weighted_quantile(d, w, 0.5)
        lib.abc_wq_stamps(buf)
        b = list(buf)
        t = lambda i: (b[i] - b[7]) * 10 / 1000.0   # 100 MHz -> us from launch
        print(N, "m", b[6], "block0 start", t(8), "loop", t(9), "reduced", t(0), "last block", t(1), "sums", t(2),
              "loaded", t(3), "sorted", t(4), "end", t(5))
