"""Discrete random-walk transition for parameters on the integer grid
(pyabc/transition/randomwalk.py:9-83).

Each coordinate of a proposal is its ancestor's plus the sum of ``n_steps``
independent steps in {-1, 0, +1} with probabilities (p_l, p_c, p_r).  It is
the transition to pair with discrete priors (poisson, binom, ...), which have
no batched form: such runs take the per-candidate loop, so this class is
host code (numpy), not a device kernel.

The density is the mixture over the population of the product over
coordinates of the one-coordinate walk law P(s), s = x_k - X_jk.  P is a
table over s in [-n_steps, n_steps] (the trinomial sum of
randomwalk.py:99-118, formed once per parameter set), so a density is one
gather + product + weighted sum instead of one multinomial pmf per
(candidate, particle, coordinate, step count).
"""
from math import comb
from typing import Union

import numpy as np
import pandas as pd

from .base import DiscreteTransition


def walk_step_law(n_steps: int, p_l: float, p_r: float, p_c: float) -> np.ndarray:
    """P(net displacement = s) for s = -n .. n after n steps, as an array of
    2n + 1 entries (index s + n).  n_r right steps and n_l = n_r - s left steps
    leave n_c = n - n_r - n_l in place: multinomial(n; n_l, n_r, n_c)."""
    n = int(n_steps)
    law = np.zeros(2 * n + 1)
    for s in range(-n, n + 1):
        total = 0.0
        for n_r in range(max(s, 0), n + 1):
            n_l = n_r - s
            n_c = n - n_r - n_l
            if n_l < 0 or n_c < 0:
                continue
            total += (comb(n, n_r) * comb(n - n_r, n_l)
                      * p_r ** n_r * p_l ** n_l * p_c ** n_c)
        law[s + n] = total
    return law


class DiscreteRandomWalkTransition(DiscreteTransition):
    """Random walk of ``n_steps`` steps per coordinate from a weighted draw of
    the population (randomwalk.py:9-83).  Like the reference, it does not
    adapt to the population and is not a proper importance distribution
    (its support does not cover the prior's)."""

    def __init__(self, n_steps: int = 1, p_l: float = 1. / 3,
                 p_r: float = 1. / 3, p_c: float = 1. / 3):
        self.n_steps = n_steps
        self.p_l = p_l
        self.p_r = p_r
        self.p_c = p_c

    def fit(self, X: pd.DataFrame, w: np.ndarray):
        # nothing to fit: TransitionMeta keeps X and the normalised w
        pass

    def _law(self):
        key = (self.n_steps, self.p_l, self.p_r, self.p_c)
        if getattr(self, "_law_key", None) != key:
            self._law_table = walk_step_law(*key)
            self._law_key = key
        return self._law_table

    def _walk(self, size):
        """[size, dim] net displacements: n_steps steps per coordinate."""
        dim = len(self.X.columns)
        steps = np.random.choice([-1, 0, 1], p=[self.p_l, self.p_c, self.p_r],
                                 size=(self.n_steps, size, dim))
        return steps.sum(axis=0).astype(float)

    def rvs_single(self) -> pd.Series:
        start = self.X.sample(weights=self.w).iloc[0]
        return start + self._walk(1)[0]

    def rvs(self, size=None):
        if size is None:
            return self.rvs_single()
        idx = np.random.choice(len(self.X), size=size, p=np.asarray(self.w, float))
        vals = self.X.values[idx] + self._walk(size)
        return pd.DataFrame(vals, columns=self.X.columns)

    def pdf(self, x: Union[pd.Series, pd.DataFrame]) -> Union[float, np.ndarray]:
        """Probability mass at x; raises ValueError for non-integer x
        (randomwalk.py:55-70)."""
        if not np.all(np.isclose(x, x.astype(int))):
            raise ValueError(f"Transition can only handle integer values, not "
                             f"fulfilled by x={x}.")
        x = np.asarray(x[self.X.columns], dtype=float)
        single = x.ndim == 1
        xs = np.atleast_2d(x)
        law = self._law()
        n = self.n_steps
        X = self.X.values.astype(float)
        w = np.asarray(self.w, dtype=float)
        out = np.empty(xs.shape[0])
        for i, row in enumerate(xs):
            s = np.rint(row[None, :] - X).astype(np.int64)          # [N, dim]
            inside = np.abs(s) <= n
            p = np.where(inside, law[np.clip(s + n, 0, 2 * n)], 0.0).prod(axis=1)
            out[i] = float(p @ w)
        return out[0] if single else out
