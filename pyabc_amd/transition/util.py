import numpy as np


def smart_cov(X_arr, w):
    """pyabc/transition/util.py:4-16 (host helper; the device fits use the
    weighted-moments kernel and the same formula)."""
    if X_arr.shape[0] == 1:
        return np.diag(np.absolute(X_arr[0]))
    cov = np.cov(X_arr, aweights=w, rowvar=False)
    return np.atleast_2d(cov)
