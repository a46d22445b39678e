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


_BM = None


def _bm_tables():
    global _BM
    if _BM is None:
        import os
        t = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bm_tables.npz"))
        _BM = {k: t[k] for k in t.files}
    return _BM


def normal_pairs(x0, x1):
    """Box-Muller on two u32 streams -> two standard normals, R cos / R sin of
    2 pi u2 with R = sqrt(-2 ln u1), u = uniform01.  Restates the device
    transform (pyabc_amd/csrc/abc_common.h box_muller) operation for
    operation in float32 -- table-driven log and sin/cos, every operation
    correctly rounded (the device's sqrt_rn is the correctly rounded fp32
    sqrt, here float64 sqrt rounded once) -- so the normals replay the
    device BIT FOR BIT (tests/test_gpu_kernels.py).  Tables:
    oracle/bm_tables.npz (tools/gen_bm_tables.py)."""
    T = _bm_tables()
    f32 = np.float32
    a = np.asarray(x0, dtype=np.uint32).astype(np.uint64)
    b = np.asarray(x1, dtype=np.uint32).astype(np.uint64)
    m1 = a | np.uint64(1)                 # u1 = m1 2^-32 (32 bits; 41 below 2^-23)
    yi = np.uint64(1 << 32) - m1
    # series branch: u1 > 1 - 2^-8
    y = yi.astype(np.float32) * f32(2.0 ** -32)
    z = y * f32(0.2) + f32(0.25)
    z = z * y + f32(1 / 3)
    z = z * y + f32(0.5)
    z = z * y + f32(1.0)
    v_series = z * y
    # table branch; u1 < 2^-23 (a < 2^9): 41 bits, b's 9 low bits below a's
    ext = a < np.uint64(512)
    mt = np.where(ext, (a << np.uint64(9)) | (b & np.uint64(511)) | np.uint64(1), m1)
    e = (np.frexp(mt.astype(np.float64))[1] - 1).astype(np.uint64)
    t = (mt << (np.uint64(31) - e)) & np.uint64(0xFFFFFFFF)
    i = ((t >> np.uint64(24)) & np.uint64(127)).astype(np.int64)
    delta = (t & np.uint64(0xFFFFFF)).astype(np.float32) * f32(2.0 ** -31)
    r = delta * T["inv"][i]
    p = r * f32(-0.25) + f32(1 / 3)
    p = p * r - f32(0.5)
    p = p * r + f32(1.0)
    p = p * r
    k = (np.where(ext, np.uint64(41), np.uint64(32)) - e).astype(np.float32)
    LN2_HI, LN2_LO = f32(float.fromhex("0x1.62e4p-1")), f32(float.fromhex("0x1.7f7d1cp-20"))
    v_table = (k * LN2_HI - T["hi"][i]) + ((k * LN2_LO - T["lo"][i]) - p)
    v = np.where(yi < np.uint64(1 << 24), v_series, v_table).astype(np.float32)
    R = np.sqrt((f32(2.0) * v).astype(np.float64)).astype(np.float32)
    m2 = ((b >> np.uint64(9)) << np.uint64(1)) | np.uint64(1)
    ia = (m2 >> np.uint64(16)).astype(np.int64)
    bb = (m2 & np.uint64(0xFFFF)).astype(np.float32) * f32(float.fromhex("0x1.921fb6p-22"))
    b2 = bb * bb
    sb = bb - (bb * b2) * f32(1 / 6)
    cb = f32(1.0) - b2 * (f32(0.5) - b2 * f32(1 / 24))
    sa, ca = T["sc"][ia, 0], T["sc"][ia, 1]
    sn = sa * cb + ca * sb
    cs = ca * cb - sa * sb
    return (R * cs).astype(np.float64), (R * sn).astype(np.float64)
