"""Shared test utilities: synthetic data and oracle fits."""

import numpy as np

from mpitree_amd.core.binning import fit_bin_mapper
from mpitree_amd.core.criterion import Criterion
from mpitree_amd.core.reference import fit_reference


def random_problem(rng, n, F, C, levels, regression=False):
    X = rng.integers(0, levels, size=(n, F)).astype(np.float64) / 4.0
    if regression:
        y = rng.normal(size=n).round(3)
    else:
        w = rng.normal(size=F)
        score = X @ w + rng.normal(scale=0.5, size=n)
        y = np.digitize(score, np.quantile(score, np.linspace(0, 1, C + 1)[1:-1])).astype(np.int64)
    return X, y


def oracle(X, y, crit, max_depth=None, mss=2, msl=1, regression=False, max_bins=256):
    """Fit the plain-numpy oracle on exactly what the estimators would see."""
    from mpitree_amd.core.fit import _encode_targets, _finalize

    mapper = fit_bin_mapper(X, max_bins)
    codes = mapper.transform(X)
    if regression:
        yf, e = _encode_targets(y, len(y))
        ta = fit_reference(codes, yf, n_classes=0, n_bins=mapper.max_n_bins,
                           criterion=Criterion.SQUARED_ERROR, max_depth=max_depth,
                           min_samples_split=mss, min_samples_leaf=msl)
        return _finalize(ta, mapper, True, e)
    classes, enc = np.unique(y, return_inverse=True)
    ta = fit_reference(codes, enc, n_classes=len(classes), n_bins=mapper.max_n_bins,
                       criterion=crit, max_depth=max_depth, min_samples_split=mss,
                       min_samples_leaf=msl)
    return _finalize(ta, mapper, False, 0)
