"""Philox4x32-10 counter-based RNG (Salmon et al., SC'11) in numpy.

Test infrastructure only -- see ``oracle/__init__.py``.  The reference draws
from numpy's global MT19937 (pyabc/transition/multivariatenormal.py:85-97),
which no GPU reproduces; the batched sampler instead keys every draw by
(seed, generation, global candidate index, slot).  This module restates the
device generator bit for bit so the oracle can replay the GPU's draws.

Counter layout (shared with pyabc_amd/csrc/abc_rng.h):
  key = (seed & 0xffffffff, seed >> 32)
  ctr = (index & 0xffffffff, index >> 32, slot, generation)
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(index, slot, generation, seed):
    """Return uint32 array [..., 4] for counters built from ``index``."""
    index = np.asarray(index, dtype=np.uint64)
    c0 = (index & MASK).astype(np.uint64)
    c1 = (index >> np.uint64(32)).astype(np.uint64)
    c2 = np.broadcast_to(np.uint64(np.uint32(slot)), index.shape).astype(np.uint64)
    c3 = np.broadcast_to(np.uint64(np.uint32(generation)), index.shape).astype(np.uint64)
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK, lo1, (hi0 ^ c3 ^ k1) & MASK, lo0
        k0 = (k0 + np.uint64(W0)) & MASK
        k1 = (k1 + np.uint64(W1)) & MASK
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def uniform01(x):
    """u32 -> float in (0, 1): ((x >> 9) + 0.5) * 2^-23 (exact in fp32)."""
    return ((np.asarray(x, dtype=np.uint32) >> np.uint32(9)).astype(np.float64)
            + 0.5) * 2.0 ** -23


def uniform53(x0, x1):
    """Two u32 -> double in [0, 1) (numpy's random_double formula)."""
    a = (np.asarray(x0, dtype=np.uint32) >> np.uint32(5)).astype(np.float64)
    b = (np.asarray(x1, dtype=np.uint32) >> np.uint32(6)).astype(np.float64)
    return (a * 67108864.0 + b) / 9007199254740992.0


def normal_pairs(x0, x1):
    """Box-Muller on two u32 streams -> two standard normals (float64).
    The device evaluates the same formula with a table-driven fp64 transform
    (abc_common.h box_muller) that agrees to a few ulp."""
    u1 = uniform01(x0)
    u2 = uniform01(x1)
    r = np.sqrt(-2.0 * np.log(u1))
    return r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)
