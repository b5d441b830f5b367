"""MPITREE_DEBUG: tree invariant validation and device input checks."""

import numpy as np
import pytest

from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
from mpitree_amd.utils.debug import TreeInvariantError, validate_tree
from tests.helpers import random_problem


@pytest.fixture
def debug_env(monkeypatch):
    monkeypatch.setenv("MPITREE_DEBUG", "1")


def test_debug_fit_validates(debug_env):
    rng = np.random.default_rng(3)
    X, y = random_problem(rng, 400, 5, 3, 9)
    clf = DecisionTreeClassifier(device="cpu").fit(X, y)
    validate_tree(clf._arrays, n_rows=400, n_features=5)
    Xr, yr = random_problem(rng, 300, 4, 0, 7, regression=True)
    reg = DecisionTreeRegressor(device="cpu", min_samples_leaf=2).fit(Xr, yr)
    validate_tree(reg._arrays, n_rows=300, n_features=4)


def _fitted():
    rng = np.random.default_rng(5)
    X, y = random_problem(rng, 200, 4, 2, 8)
    return DecisionTreeClassifier(device="cpu").fit(X, y)._arrays


@pytest.mark.parametrize("corrupt", ["rows", "counts", "link", "depth", "feature", "root"])
def test_validate_tree_catches_corruption(corrupt):
    ta = _fitted()
    validate_tree(ta, n_rows=200, n_features=4)
    inner = np.nonzero(ta.feature >= 0)[0]
    i = int(inner[len(inner) // 2])
    if corrupt == "rows":
        ta.n_samples = ta.n_samples.copy()
        ta.n_samples[ta.left[i]] += 1
    elif corrupt == "counts":
        ta.count = ta.count.copy()  # row sums kept, class conservation broken
        ta.count[ta.left[i], 0] += 1
        ta.count[ta.left[i], 1] -= 1
    elif corrupt == "link":
        ta.right = ta.right.copy()
        ta.right[i] = ta.left[i]
    elif corrupt == "depth":
        ta.depth = ta.depth.copy()
        ta.depth[ta.right[i]] += 1
    elif corrupt == "feature":
        ta.feature = ta.feature.copy()
        ta.feature[i] = 7
    elif corrupt == "root":
        ta.n_samples = ta.n_samples.copy()
    with pytest.raises(TreeInvariantError):
        validate_tree(ta, n_rows=199 if corrupt == "root" else 200, n_features=4)


@pytest.mark.gpu
def test_debug_gpu_fit_checks_inputs_and_tree(debug_env):
    import torch

    from mpitree_amd.utils.datasets import make_classification

    X, y = make_classification(50_000, 16, n_classes=3, seed=1, device="cuda")
    clf = DecisionTreeClassifier(device="cuda").fit(X, y)
    assert clf.fit_stats_["engine"].startswith("hip")
    validate_tree(clf._arrays, n_rows=50_000, n_features=16)
    assert torch.cuda.is_available()


def test_leaf_count_identity():
    """n_leaves uses N = 2L - 1 (every internal node has two children)."""
    for seed in range(4):
        rng = np.random.default_rng(seed)
        X, y = random_problem(rng, 300 + 50 * seed, 4, 3, 6)
        ta = DecisionTreeClassifier(max_depth=[None, 0, 3, 5][seed], device="cpu").fit(X, y)._arrays
        assert ta.n_leaves == int((ta.feature < 0).sum())
