"""Power-law fit of CV against population size (pyabc/cv/powerlaw.py:1-17).
A handful of (n, cv) points: host scipy, off the device path."""
import numpy as np
from scipy.optimize import curve_fit


def power_law(x, a, b):
    return a * x ** (-b)


def finverse(y, a, b):
    return (a / y) ** (1 / b)


def fitpowerlaw(x, y):
    """Least-squares a x^-b from the reference's start point (0.5, 0.2);
    curve_fit's RuntimeError on non-convergence propagates (the caller,
    predict_population_size, falls back on it)."""
    x = np.array(x)
    y = np.array(y)
    popt, _ = curve_fit(power_law, x, y, p0=[.5, 1 / 5])
    return popt, lambda x: power_law(x, *popt), lambda y: finverse(y, *popt)
