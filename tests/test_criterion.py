"""Integer-form split criteria: numpy mirror == native C++ (bitwise), and the
terms equal m * impurity of the reference's probability formulas."""

import numpy as np
import pytest

from mpitree_amd.core.criterion import entropy_term, gini_term, mse_term, xlog2x
from mpitree_amd.ops import native


def test_xlog2x_small_values():
    assert xlog2x(np.array([0, 1]))[0] == 0.0 and xlog2x(np.array([0, 1]))[1] == 0.0
    assert xlog2x(np.array([2]))[0] == 2.0
    assert xlog2x(np.array([4]))[0] == 8.0


def test_xlog2x_accuracy():
    x = np.concatenate([np.arange(2, 100000), np.random.default_rng(0).integers(2, 2**45, 20000)])
    ref = x * np.log2(x.astype(np.float64))
    np.testing.assert_allclose(xlog2x(x), ref, rtol=4e-16 * 4)


@pytest.mark.skipif(not native.has_cpu(), reason="native module not built")
def test_xlog2x_numpy_matches_native_bitwise():
    x = np.concatenate([np.arange(0, 70000), np.random.default_rng(1).integers(0, 2**50, 50000)])
    a = xlog2x(x)
    b = native.cpu().xlog2x(x.astype(np.int64))
    assert np.array_equal(a.view(np.int64), b.view(np.int64))


def _ref_entropy(c):
    c = np.asarray(c, dtype=np.float64)
    c = c[c > 0]
    p = c / c.sum()
    return -np.sum(p * np.log2(p))


def test_terms_match_impurity():
    rng = np.random.default_rng(2)
    for _ in range(200):
        c = rng.integers(0, 50, size=rng.integers(1, 6))
        if c.sum() == 0:
            continue
        m = c.sum()
        assert entropy_term(c) == pytest.approx(m * _ref_entropy(c), rel=1e-12, abs=1e-12)
        g = 1 - np.sum((c / m) ** 2)
        assert gini_term(c) == pytest.approx(m * g, rel=1e-12, abs=1e-12)


def test_mse_term_ordering_matches_sse():
    # cost ordering of -(S_L^2/m_L + S_R^2/m_R) equals the SSE ordering
    rng = np.random.default_rng(3)
    y = rng.integers(-100, 100, size=40)
    costs, sse = [], []
    for k in range(1, 40):
        L, R = y[:k], y[k:]
        costs.append(mse_term(len(L), L.sum()) + mse_term(len(R), R.sum()))
        sse.append(((L - L.mean()) ** 2).sum() + ((R - R.mean()) ** 2).sum())
    assert np.argmin(costs) == np.argmin(sse)


@pytest.mark.skipif(not native.has_cpu(), reason="native module not built")
def test_node_terms_native_matches_numpy():
    rng = np.random.default_rng(4)
    st = rng.integers(0, 1000, size=(500, 4)).astype(np.int64)
    cpu = native.cpu()
    assert np.array_equal(cpu.node_terms(st, 0), entropy_term(st))
    assert np.array_equal(cpu.node_terms(st, 1), gini_term(st))
    assert np.array_equal(cpu.node_terms(st[:, :2], 2), mse_term(st[:, 0], st[:, 1]))
