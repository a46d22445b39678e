"""Bootstrapped coefficient of variation of the transition KDE.

Reference: pyabc/cv/bootstrap.py:6-110 (``weights``, ``calc_cv``), used by
``Transition.mean_cv`` (transition/base.py:121-169) and
``AdaptivePopulationSize.update`` (populationstrategy.py:203-227), SURVEY.md
§8f row 3.

Each of the N_BOOTSTR rounds draws n_m points from transition m (rvs), fits a
copy of it to them with uniform weights and evaluates the copy's density at
the test points.  For device transitions (MultivariateNormalTransition,
LocalTransition) every step stays in HBM: ``propose_device`` (the a2 rvs
kernel), ``fit_device`` (a1/a4 fit), ``logpdf_device`` (the a3 density kernel,
N_test x n pairs) into one row of a [N_BOOTSTR, N_test] log-density buffer,
then ``abc_bootstrap_cv`` computes scipy.stats.variation over the bootstrap
axis and the weighted sum in one pass.  One host read per model: the CV.
Transitions without device entry points take the reference's host route.
"""
import copy

import numpy as np


def _is_device(tr):
    return (all(hasattr(tr, a) for a in ("propose_device", "fit_device",
                                         "logpdf_device"))
            and getattr(tr, "_dev_X", None) is not None
            and not getattr(tr, "no_parameters", False))


def weights(n_per_model, transitions, test_transitions, test_X):
    """bootstrap.py:6-41: sample n_m points from transitions[m], fit
    test_transitions[m] to them (uniform weights), densities at test_X[m]."""
    out = []
    for trans, test_trans, n, X in zip(transitions, test_transitions,
                                       n_per_model, test_X):
        bootstr_X = trans.rvs(size=n)
        test_trans.fit(bootstr_X, np.ones(len(bootstr_X)) / len(bootstr_X))
        out.append(test_trans.pdf(X))
    return out


def _test_points_device(trans, X):
    """Device [N_test, d] matrix of test points in the fit's column order."""
    from .. import gpu
    if X is trans.X and trans._dev_X is not None:
        return trans._dev_X
    cols = list(trans.X.columns)
    arr = np.asarray(X[cols] if hasattr(X, "columns") else X, dtype=np.float64)
    return gpu.as_dev(np.atleast_2d(arr), device=trans._dev_X.device)


def _test_weights_device(trans, w, device, n_test):
    from .. import gpu
    if hasattr(w, "_wd"):          # _LazyArray view of device weights
        return w._wd
    if np.ndim(w) == 0:            # a scalar weight for every test point
        return gpu.torch.full((n_test,), float(w), dtype=gpu.torch.float64,
                              device=device)
    return gpu.as_dev(np.asarray(w, dtype=np.float64), device=device)


def _model_cv_device(trans, test_trans, n, X, w, N_BOOTSTR, scale):
    """One model's bootstraps entirely in HBM; returns device (var, cv)."""
    from .. import gpu
    torch = gpu.torch
    Xt = _test_points_device(trans, X)
    wt = _test_weights_device(trans, w, Xt.device, Xt.shape[0])
    cols = list(trans.X.columns)
    logdens = torch.empty((N_BOOTSTR, Xt.shape[0]), dtype=torch.float64,
                          device=Xt.device)
    n = int(n)
    unif = torch.full((n,), 1.0 / max(n, 1), dtype=torch.float64,
                      device=Xt.device)
    for b in range(N_BOOTSTR):
        bootstr_X = trans.propose_device(n)[0]
        test_trans.fit_device(bootstr_X, unif, cols)
        test_trans.logpdf_device(Xt, out=logdens[b])
    return gpu.bootstrap_cv(logdens, wt, scale=scale)


def _model_cv_host(trans, test_trans, n, X, w, N_BOOTSTR, scale):
    """The reference's route for transitions without device entry points."""
    import scipy.stats as st
    dens = np.array([weights([n], [trans], [test_trans], [X])[0]
                     for _ in range(N_BOOTSTR)])
    var = st.variation(dens, axis=0)
    return var, float((var * scale * np.asarray(w)).sum())


def calc_cv(nr_particles, model_weights, N_BOOTSTR, test_w, transitions,
            test_X):
    """bootstrap.py:44-110.  Returns (cv, variations_at_X).

    Per model m: N_BOOTSTR x (draw n_m from transitions[m], fit a copy with
    uniform weights, densities at test_X[m]); variation over the bootstrap
    axis, scaled by n_m / sum n, weighted by test_w[m], summed."""
    test_transitions = copy.deepcopy(transitions)
    n_per_model = np.random.multinomial(nr_particles, model_weights)
    n_sum = n_per_model.sum()
    cvs, variations = [], []
    for trans, test_trans, n, X, w in zip(transitions, test_transitions,
                                          n_per_model, test_X, test_w):
        if _is_device(trans):
            var, cv = _model_cv_device(trans, test_trans, n, X, w, N_BOOTSTR,
                                       n / n_sum)
        else:
            var, cv = _model_cv_host(trans, test_trans, n, X, w, N_BOOTSTR,
                                     n / n_sum)
        cvs.append(cv)
        variations.append(var)
    cv = sum(float(c.item()) if hasattr(c, "cpu") else float(c) for c in cvs)
    return cv, [v.cpu().numpy() if hasattr(v, "cpu") else v
                for v in variations]
