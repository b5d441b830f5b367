"""Parity against the reference implementation's own source (an independent oracle).

The reference (``/root/reference/mpitree/tree/decision_tree.py``) is loaded
from source with a single-rank ``mpi4py`` stub (``tests/reference_oracle.py``)
and fitted on several hundred random small problems -- discrete features
(ties everywhere) and continuous ones -- next to this framework's default
estimator. ``export_text(precision=17)`` and ``predict`` must agree.

Where they do not, the first node at which the two trees diverge is
re-scored in exact decimal arithmetic (50 digits): the test then requires
that the two chosen splits have *mathematically equal* cost (a tie), and
that this framework's choice is the reference's stated tie rule -- lowest
feature among the minimum-cost splits (``np.argmax``, :140), smallest
threshold within it (``np.argmin``, :88-90) -- so the divergence is the
reference's floating-point rounding breaking its own rule. Problems on which
the reference recurses forever (zero-gain split onto an empty child,
SURVEY §2.7.5, a reference bug this framework fixes) are excluded and
counted. The summary is printed with ``-s``.
"""

from __future__ import annotations

import decimal
import re
import sys

import numpy as np
import pytest

from mpitree_amd import DecisionTreeClassifier

from .reference_oracle import load_reference

REF = load_reference()
pytestmark = pytest.mark.skipif(REF is None, reason="reference checkout absent")

_D = decimal.Context(prec=50)
_LN2 = _D.ln(decimal.Decimal(2))


def _entropy_exact(y):
    n = len(y)
    if n == 0:
        return decimal.Decimal(0)
    h = decimal.Decimal(0)
    for c in np.unique(y, return_counts=True)[1]:
        p = _D.divide(decimal.Decimal(int(c)), decimal.Decimal(n))
        h -= _D.multiply(p, _D.divide(_D.ln(p), _LN2))
    return h


def _cost_exact(X, y, f, t):
    left = X[:, f] <= t
    n = len(y)
    c = decimal.Decimal(0)
    for side in (left, ~left):
        m = int(side.sum())
        if m:
            c += _D.multiply(_D.divide(decimal.Decimal(m), decimal.Decimal(n)),
                             _entropy_exact(y[side]))
    return c


def _canon(txt: str) -> str:
    """-0.0 and 0.0 are one threshold value; which sign np.unique keeps depends
    on its (unstable) sort, so the rendering is compared sign-free for zero."""
    return re.sub(r"-(0\.0+)\]", r"\1]", txt)


def _problems(count, seed0):
    for s in range(seed0, seed0 + count):
        rng = np.random.default_rng(s)
        kind = "discrete" if s % 2 == 0 else "continuous"
        n = int(rng.integers(6, 36))
        F = int(rng.integers(1, 4))
        C = int(rng.integers(2, 4))
        if kind == "discrete":
            X = rng.integers(0, 5, size=(n, F)).astype(np.float64)
        else:
            X = np.round(rng.normal(size=(n, F)), 3)
        y = rng.integers(0, C, size=n)
        y = np.searchsorted(np.unique(y), y)  # labels 0..K-1 (the reference's contract)
        md = None if s % 3 else int(rng.integers(1, 4))
        yield s, kind, X, y, md


def _walk(tree, X, rows):
    """Pre-order (node, rows) pairs of a reference Node tree."""
    out = [(tree, rows)]
    if tree.threshold is not None and tree.left is not None:
        go = X[rows, tree.value] <= tree.threshold
        out += _walk(tree.left, X, rows[go])
        out += _walk(tree.right, X, rows[~go])
    return out


def _divergence(ref_tree, our_tree, X, y):
    """First pre-order node where the two trees choose different splits."""
    a = _walk(ref_tree, X, np.arange(len(y)))
    b = _walk(our_tree, X, np.arange(len(y)))
    for (na, ra), (nb, rb) in zip(a, b):
        sa = None if na.threshold is None else (int(na.value), float(na.threshold))
        sb = None if nb.threshold is None else (int(nb.value), float(nb.threshold))
        if sa != sb:
            return ra, sa, sb
    return None


def _canonical_best(X, y):
    """Exact minimum cost and the stated tie rule's choice (lowest feature, smallest t)."""
    best, choice = None, None
    for f in range(X.shape[1]):
        for t in np.unique(X[:, f]):
            c = _cost_exact(X, y, f, t)
            if best is None or c < best - decimal.Decimal("1e-40"):
                best, choice = c, (f, float(t))
    return best, choice


def test_reference_parity_random_problems():
    stats = dict(total=0, equal=0, ref_recursion=0, tie_breaks=0)
    ties = []
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(400)
    try:
        for s, kind, X, y, md in _problems(240, 1000):
            try:
                ref = REF.DecisionTreeClassifier(max_depth=md).fit(X, y)
                ref_txt = ref.export_text(precision=17)
            except RecursionError:
                stats["ref_recursion"] += 1
                continue
            stats["total"] += 1
            ours = DecisionTreeClassifier(max_depth=md, device="cpu").fit(X, y)
            our_txt = ours.export_text(precision=17)
            if _canon(our_txt) == _canon(ref_txt):
                stats["equal"] += 1
                np.testing.assert_array_equal(ours.predict(X), ref.predict(X))
                np.testing.assert_array_equal(ours.predict_proba(X), ref.predict_proba(X))
                continue
            div = _divergence(ref.tree_, ours.tree_, X, y)
            assert div is not None, f"seed {s}: same splits, different text"
            rows, sa, sb = div
            assert sa is not None and sb is not None, f"seed {s}: leaf vs split at {sa} {sb}"
            Xn, yn = X[rows], y[rows]
            best, canon = _canonical_best(Xn, yn)
            ca, cb = _cost_exact(Xn, yn, *sa), _cost_exact(Xn, yn, *sb)
            tol = decimal.Decimal("1e-40")
            assert abs(cb - best) < tol, f"seed {s}: our split {sb} is not optimal"
            assert abs(ca - best) < tol, f"seed {s}: reference split {sa} is not optimal"
            assert sb == canon, f"seed {s}: ours {sb} is not the tie rule's {canon}"
            stats["tie_breaks"] += 1
            ties.append((s, kind, sa, sb))
    finally:
        sys.setrecursionlimit(old)
    print(f"\nreference parity: {stats}; reference-rounding tie breaks: {ties}")
    assert stats["total"] >= 200
    assert stats["equal"] + stats["tie_breaks"] == stats["total"]
    # ties decided by the reference's rounding are rare on these problem sizes
    assert stats["tie_breaks"] <= stats["total"] // 10


@pytest.mark.parametrize("seed", range(5))
def test_continuous_default_is_exact(seed):
    """Continuous features (> 256 unique values): the default estimator uses
    every unique value as a threshold, like the reference (verdict r1: the
    quantile-binned default disagreed on 5/5 such problems)."""
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(400, 2))
    y = (X[:, 0] + 0.5 * X[:, 1] + rng.normal(scale=0.5, size=400) > 0).astype(np.int64)
    ref = REF.DecisionTreeClassifier(max_depth=4).fit(X, y)
    ours = DecisionTreeClassifier(max_depth=4, device="cpu").fit(X, y)
    assert _canon(ours.export_text(precision=17)) == _canon(ref.export_text(precision=17))
    np.testing.assert_array_equal(ours.predict(X), ref.predict(X))
