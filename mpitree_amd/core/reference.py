"""Plain-numpy exact tree builder: the test oracle for every other builder.

Semantics follow the reference recursion (``mpitree/tree/decision_tree.py:93-166``):

* a node becomes a leaf when it is pure, when ``depth == max_depth``, when it
  has fewer than ``min_samples_split`` rows, or when its rows are identical
  (no feature has two distinct codes);
* candidates are every threshold present in the node (``x <= t`` goes left);
  per feature the cheapest candidate wins with ties to the smallest threshold,
  across features the largest gain wins with ties to the lowest index;
* the leaf label is the lowest class among tied maxima.

Deliberate fixes: a split that would leave a child empty is
never a candidate, so the reference's infinite recursion on a constant
feature cannot happen; ``min_samples_leaf`` (default 1) is an extra sklearn
style constraint.
"""

from __future__ import annotations

import numpy as np

from .criterion import Criterion, entropy_term, gini_term, mse_term, tie_round
from ..models.tree_arrays import TreeArrays

__all__ = ["best_split_dense", "fit_reference"]


def _terms(crit, cnt, s=None, m=None):
    if crit == Criterion.ENTROPY:
        return entropy_term(cnt)
    if crit == Criterion.GINI:
        return gini_term(cnt)
    return mse_term(m, s)


def best_split_dense(hist, crit, parent_term, m_total, min_samples_leaf=1, hist_sum=None):
    """Best split from a dense node histogram.

    ``hist`` is ``[F, B, C]`` class counts (classification) or ``[F, B]``
    counts with ``hist_sum`` ``[F, B]`` fixed-point target sums (regression).
    Returns ``(feature, bin, gain, left_count)`` or ``(-1, -1, -inf, 0)``.
    """
    if crit == Criterion.SQUARED_ERROR:
        cnt = hist.astype(np.int64)
        L = np.cumsum(cnt, axis=1)
        SL = np.cumsum(hist_sum.astype(np.int64), axis=1)
        mL = L
        mR = m_total - mL
        S_tot = SL[:, -1:]
        cost = _terms(crit, None, SL, mL) + _terms(crit, None, S_tot - SL, mR)
        nonempty = cnt > 0
    else:
        cnt = hist.astype(np.int64)
        L = np.cumsum(cnt, axis=1)
        tot = L[:, -1:, :]
        R = tot - L
        mL = L.sum(-1)
        mR = m_total - mL
        cost = tie_round(_terms(crit, L) + _terms(crit, R), m_total)
        nonempty = cnt.sum(-1) > 0
    valid = nonempty & (mL >= max(1, min_samples_leaf)) & (mR >= max(1, min_samples_leaf))
    cost = np.where(valid, cost, np.inf)
    b = np.argmin(cost, axis=1)
    F = hist.shape[0]
    best_cost = cost[np.arange(F), b]
    ok = np.isfinite(best_cost)
    if not ok.any():
        return -1, -1, -np.inf, 0
    gain = np.where(ok, parent_term - best_cost, -np.inf)
    f = int(np.argmax(gain))
    return f, int(b[f]), float(gain[f]), int(mL[f, b[f]])


def fit_reference(
    codes: np.ndarray,
    y: np.ndarray,
    *,
    n_classes: int,
    n_bins: int,
    criterion: Criterion = Criterion.ENTROPY,
    max_depth=None,
    min_samples_split: int = 2,
    min_samples_leaf: int = 1,
) -> TreeArrays:
    """Depth-first exact fit on pre-binned ``codes`` ``[n, F]``.

    ``y`` holds class indices ``0..n_classes-1`` (classification) or
    fixed-point int64 targets (regression, ``n_classes`` ignored).
    """
    codes = np.asarray(codes)
    n, F = codes.shape
    reg = criterion == Criterion.SQUARED_ERROR
    feats, tbin, left, right, nsamp, imp, cnts, sums = [], [], [], [], [], [], [], []
    fidx = np.broadcast_to(np.arange(F), (1, F))
    stack = [(np.arange(n), 0, -1, 0)]
    while stack:
        rows, depth, parent, side = stack.pop()
        i = len(feats)
        if parent >= 0:
            (left if side == 0 else right)[parent] = i
        m = rows.shape[0]
        yn = y[rows]
        if reg:
            s = int(yn.sum())
            pt = float(mse_term(m, s))
            pure = m == 0 or yn.min() == yn.max()
            cnts.append(None)
            sums.append(s)
        else:
            c = np.bincount(yn, minlength=n_classes).astype(np.int64)
            pt = float(_terms(criterion, c))
            pure = (c > 0).sum() <= 1
            cnts.append(c)
            sums.append(0)
        nsamp.append(m)
        imp.append(pt)
        feats.append(-1)
        tbin.append(-1)
        left.append(-1)
        right.append(-1)
        if pure or (max_depth is not None and depth >= max_depth) or m < min_samples_split:
            continue
        cn = codes[rows]
        fi = np.broadcast_to(fidx, cn.shape)
        if reg:
            h = np.zeros((F, n_bins), dtype=np.int64)
            hs = np.zeros((F, n_bins), dtype=np.int64)
            np.add.at(h, (fi, cn), 1)
            np.add.at(hs, (fi, cn), np.broadcast_to(yn[:, None], cn.shape))
            f, b, gain, ml = best_split_dense(h, criterion, pt, m, min_samples_leaf, hs)
        else:
            h = np.zeros((F, n_bins, n_classes), dtype=np.int64)
            np.add.at(h, (fi, cn, np.broadcast_to(yn[:, None], cn.shape)), 1)
            f, b, gain, ml = best_split_dense(h, criterion, pt, m, min_samples_leaf)
        if f < 0:
            continue
        feats[i] = f
        tbin[i] = b
        go_left = cn[:, f] <= b
        stack.append((rows[~go_left], depth + 1, i, 1))
        stack.append((rows[go_left], depth + 1, i, 0))
    N = len(feats)
    ta = TreeArrays(
        feature=np.asarray(feats, dtype=np.int32),
        threshold=np.full(N, np.nan),
        threshold_bin=np.asarray(tbin, dtype=np.int32),
        left=np.asarray(left, dtype=np.int32),
        right=np.asarray(right, dtype=np.int32),
        depth=np.zeros(N, dtype=np.int32),
        n_samples=np.asarray(nsamp, dtype=np.int64),
        impurity=np.asarray(imp, dtype=np.float64),
        count=None if reg else np.stack(cnts) if N else np.zeros((0, n_classes), np.int64),
        value=np.asarray(sums, dtype=np.float64) if reg else None,
    )
    # depth from the pre-order structure
    for k in range(N):
        if ta.feature[k] >= 0:
            ta.depth[ta.left[k]] = ta.depth[k] + 1
            ta.depth[ta.right[k]] = ta.depth[k] + 1
    if reg:
        ta.meta["sum_fixed"] = np.asarray(sums, dtype=np.int64)
    return ta
