"""Coefficient-of-variation estimation of the KDE (pyabc/cv)."""
from .bootstrap import calc_cv, weights
from .powerlaw import fitpowerlaw, power_law, finverse

__all__ = ["calc_cv", "weights", "fitpowerlaw", "power_law", "finverse"]
