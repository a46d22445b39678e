"""c4-shaped column MAD ([6.7e5 x 256] recorded sum stats, heterogeneous
scales) repeated, for rocprofv3 kernel traces of the select kernels."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from pyabc_amd import gpu
    dev = gpu.require_device()
    R, S = 670_000, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    scale = torch.tensor(10 ** np.random.default_rng(1).uniform(-2, 2, S))
    X = (torch.randn(R, S, generator=g, dtype=torch.float64) * scale).to(dev)
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
        gpu.column_mad(X)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
