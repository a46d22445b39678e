"""Per-generation arithmetic restated from pyabc/smc.py and population.py.

Test infrastructure only -- see ``oracle/__init__.py``.
"""
import numpy as np


def effective_sample_size(w):
    """pyabc/weighted_statistics.py:73-83: (sum w)^2 / sum w^2."""
    w = np.asarray(w, dtype=np.float64)
    return float(w.sum() ** 2 / (w ** 2).sum())


def normalize_weights(w):
    """pyabc/population.py:123-145 for a single model: w_i / sum w."""
    w = np.asarray(w, dtype=np.float64)
    return w / w.sum()


def importance_weights(prior_pd, transition_pd, n_acc=1, n_per_param=1):
    """pyabc/smc.py:793-809 (single model: model factor 1):
    w = prior_pd * prod(acc_w)(=1) * (n_acc / n_per_param) / transition_pd."""
    return (np.asarray(prior_pd, dtype=np.float64) * (n_acc / n_per_param)
            / np.asarray(transition_pd, dtype=np.float64))
