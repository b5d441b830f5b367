"""Split criteria in integer form, mirrored bit-for-bit from ``ops/csrc/criterion.h``.

The reference scores candidate thresholds with probability-space entropy
(``mpitree/tree/decision_tree.py:37-51`` and ``:76-91``). We score with the
count-space equivalents documented in ``criterion.h``; numpy evaluates every
operation as one correctly rounded IEEE op without contraction, so the arrays
below equal the C++/HIP values exactly (checked in ``tests/test_criterion.py``).
"""

from __future__ import annotations

import enum

import numpy as np

__all__ = [
    "Criterion",
    "xlog2x",
    "tie_round",
    "entropy_term",
    "gini_term",
    "mse_term",
    "node_term",
    "impurity_from_term",
    "parse_criterion",
]


class Criterion(enum.IntEnum):
    ENTROPY = 0
    GINI = 1
    SQUARED_ERROR = 2


_ALIASES = {
    "entropy": Criterion.ENTROPY,
    "log_loss": Criterion.ENTROPY,
    "gini": Criterion.GINI,
    "squared_error": Criterion.SQUARED_ERROR,
    "mse": Criterion.SQUARED_ERROR,
}

_P = (
    0.047619047619047616,
    0.05263157894736842,
    0.058823529411764705,
    0.06666666666666667,
    0.07692307692307693,
    0.09090909090909091,
    0.1111111111111111,
    0.14285714285714285,
    0.2,
    0.3333333333333333,
    1.0,
)


def parse_criterion(name, *, regression: bool) -> Criterion:
    """Map a user criterion name to the enum, validating the task."""
    if isinstance(name, Criterion):
        crit = name
    else:
        try:
            crit = _ALIASES[str(name)]
        except KeyError:
            raise ValueError(f"unknown criterion {name!r}") from None
    if regression and crit != Criterion.SQUARED_ERROR:
        raise ValueError("regression trees support criterion='squared_error' only")
    if not regression and crit == Criterion.SQUARED_ERROR:
        raise ValueError("classification trees support 'entropy' or 'gini'")
    return crit


def xlog2x(x) -> np.ndarray:
    """Return ``x*log2(x)`` for non-negative integer counts (0 for x <= 1)."""
    x = np.asarray(x, dtype=np.int64)
    d = x.astype(np.float64)
    frac, e = np.frexp(d)  # d = frac * 2**e, frac in [0.5, 1)
    m = frac * 2.0
    e = e.astype(np.int64) - 1
    big = m > 1.4142135623730951
    m = np.where(big, m * 0.5, m)
    e = np.where(big, e + 1, e)
    f = m - 1.0
    s = f / (2.0 + f)
    z = s * s
    p = np.full_like(z, _P[0])
    for c in _P[1:]:
        p = p * z + c
    lnm = (2.0 * s) * p
    l2 = e.astype(np.float64) + lnm * 1.4426950408889634
    out = d * l2
    return np.where(x <= 1, 0.0, out)


def entropy_term(counts: np.ndarray, axis: int = -1) -> np.ndarray:
    """``T(m) - sum_c T(c)`` with the class sum taken sequentially in class order."""
    counts = np.asarray(counts, dtype=np.int64)
    m = counts.sum(axis=axis)
    t = xlog2x(counts)
    t = np.moveaxis(t, axis, -1)
    acc = np.zeros(t.shape[:-1], dtype=np.float64)
    for c in range(t.shape[-1]):  # sequential, as in the C++/HIP loops
        acc = acc + t[..., c]
    return xlog2x(m) - acc


def gini_term(counts: np.ndarray, axis: int = -1) -> np.ndarray:
    counts = np.asarray(counts, dtype=np.int64)
    m = counts.sum(axis=axis)
    sq = (counts * counts).sum(axis=axis)
    num = (m * m - sq).astype(np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = num / m.astype(np.float64)
    return np.where(m > 0, out, 0.0)


def tie_round(cost, m) -> np.ndarray:
    """Canonical ties (``criterion.h`` ``tie_unit``/``tie_round``): a node's
    candidate costs on a grid of ``2^-32 * (T(m) + m)``, so mathematically equal
    costs compare equal and the first candidate (lowest threshold, then lowest
    feature -- the reference's rule, ``decision_tree.py:88-90, 140``) wins."""
    unit = (xlog2x(np.asarray(m, dtype=np.int64)) + np.asarray(m, dtype=np.float64)) \
        * 2.3283064365386963e-10
    inv = 1.0 / unit
    with np.errstate(invalid="ignore"):
        return np.rint(np.asarray(cost, dtype=np.float64) * inv) * unit


def mse_term(m, s_fixed) -> np.ndarray:
    m = np.asarray(m, dtype=np.int64)
    s = np.asarray(s_fixed, dtype=np.int64).astype(np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = -((s * s) / m.astype(np.float64))
    return np.where(m > 0, out, 0.0)


def node_term(crit: Criterion, counts=None, m=None, s_fixed=None) -> np.ndarray:
    if crit == Criterion.ENTROPY:
        return entropy_term(counts)
    if crit == Criterion.GINI:
        return gini_term(counts)
    return mse_term(m, s_fixed)


def impurity_from_term(crit: Criterion, term, m, s2=None, scale=1.0):
    """Convert a node term back to the node impurity for reporting."""
    m = np.asarray(m, dtype=np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        if crit in (Criterion.ENTROPY, Criterion.GINI):
            return np.where(m > 0, np.asarray(term) / m, 0.0)
        # term = -S^2/m in fixed units; impurity = (S2 - S^2/m)/m
        return np.where(m > 0, (np.asarray(s2) + np.asarray(term) / (scale * scale)) / m, 0.0)
