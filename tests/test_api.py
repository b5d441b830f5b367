"""Estimator API, reference behaviours, goldens and the pickle format."""

import pickle

import numpy as np
import pytest
from sklearn.base import clone
from sklearn.exceptions import NotFittedError

from mpitree.tree import DecisionTreeClassifier as RefPathClassifier
from mpitree_amd import (BranchType, DecisionTreeClassifier, DecisionTreeRegressor, Node,
                         ParallelDecisionTreeClassifier)
from mpitree_amd.core.fit import fit_tree

from .conftest import GOLDEN_DEPTH3, GOLDEN_DEPTH5


@pytest.mark.parametrize("engine", ["native", "numpy"])
def test_iris_goldens(iris2, engine):
    X, y, iris = iris2
    for depth, prec, gold in ((3, 2, GOLDEN_DEPTH3), (5, 1, GOLDEN_DEPTH5)):
        res = fit_tree(X, y, regression=False, criterion=0, max_depth=depth, min_samples_split=2,
                       device="cpu", engine=engine)
        txt = res.arrays.export_text(feature_names=iris.feature_names,
                                     class_names=iris.target_names, precision=prec,
                                     classes=res.classes)
        assert txt == gold


def test_reference_import_path_and_estimator(iris2):
    X, y, iris = iris2
    clf = RefPathClassifier(max_depth=3).fit(X, y)
    assert clf.export_text(feature_names=iris.feature_names,
                           class_names=iris.target_names) == GOLDEN_DEPTH3
    assert RefPathClassifier is DecisionTreeClassifier


def test_get_params_and_clone():
    clf = DecisionTreeClassifier(max_depth=4)
    p = clf.get_params()
    assert p["max_depth"] == 4 and p["min_samples_split"] == 2
    c2 = clone(clf)
    assert c2.get_params() == p


def test_predict_proba_returns_counts_like_reference(iris2):
    X, y, _ = iris2
    clf = DecisionTreeClassifier(max_depth=2).fit(X, y)
    proba = clf.predict_proba(X)
    assert proba.dtype == np.int64 and proba.shape == (150, 3)
    leaves = clf.apply(X)
    np.testing.assert_array_equal(proba, clf.tree_arrays_.count[leaves])
    pn = clf.predict_proba(X, normalize=True)
    np.testing.assert_allclose(pn.sum(1), 1.0)
    np.testing.assert_array_equal(clf.predict(X), np.argmax(proba, axis=1))


def test_default_export_labels():
    X = np.array([[0.0], [1.0], [2.0], [3.0]])
    y = np.array([0, 0, 1, 1])
    txt = DecisionTreeClassifier().fit(X, y).export_text()
    assert txt.splitlines() == ["┌── feature_0", "│  ├── class: 0 [<= 1.00]",
                                "│  └── class: 1 [> 1.00]"]


def test_not_fitted_and_feature_count():
    clf = DecisionTreeClassifier()
    with pytest.raises(NotFittedError):
        clf.predict(np.zeros((1, 2)))
    clf.fit(np.zeros((4, 2)) + np.arange(4)[:, None], [0, 1, 0, 1])
    with pytest.raises(ValueError):
        clf.predict(np.zeros((1, 3)))


def test_constant_feature_does_not_recurse_forever():
    # the reference raises RecursionError here
    X = np.array([[5, 0], [5, 0], [5, 1], [5, 1]], dtype=float)
    y = np.array([0, 1, 0, 1])
    clf = DecisionTreeClassifier().fit(X, y)
    assert clf.tree_arrays_.node_count == 3  # zero-gain split on feature 1, then leaves
    assert clf.tree_arrays_.feature[0] == 1


def test_stopping_rules():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(50, 3))
    y = rng.integers(0, 2, 50)
    assert DecisionTreeClassifier(max_depth=0).fit(X, y).tree_arrays_.node_count == 1
    assert DecisionTreeClassifier(min_samples_split=51).fit(X, y).tree_arrays_.node_count == 1
    ta = DecisionTreeClassifier(min_samples_leaf=5).fit(X, y).tree_arrays_
    assert ta.n_samples[ta.feature < 0].min() >= 5
    ident = DecisionTreeClassifier().fit(np.ones((6, 2)), [0, 1, 0, 1, 0, 1])
    assert ident.tree_arrays_.node_count == 1


def test_single_sample_and_non_contiguous_labels():
    clf = DecisionTreeClassifier().fit([[1.0]], [7])
    assert clf.predict([[3.0]])[0] == 7
    X = np.arange(6, dtype=float)[:, None]
    y = np.array([1, 1, 2, 2, 5, 5])
    clf = DecisionTreeClassifier().fit(X, y)
    np.testing.assert_array_equal(clf.predict(X), y)
    ys = np.array(["a", "a", "b", "b", "c", "c"])
    np.testing.assert_array_equal(DecisionTreeClassifier().fit(X, ys).predict(X), ys)


def test_rejects_nan_and_bad_params():
    with pytest.raises(ValueError):
        DecisionTreeClassifier().fit([[np.nan]], [0])
    with pytest.raises(ValueError):
        DecisionTreeClassifier(min_samples_split=1).fit([[0.0], [1.0]], [0, 1])
    with pytest.raises(ValueError):
        DecisionTreeClassifier(criterion="squared_error").fit([[0.0], [1.0]], [0, 1])


def test_pickle_round_trip_and_reference_format(iris2):
    X, y, _ = iris2
    clf = DecisionTreeClassifier(max_depth=3).fit(X, y)
    blob = pickle.dumps(clf)
    assert b"mpitree.tree._base" in blob and b"mpitree.tree.decision_tree" in blob
    state = clf.__getstate__()
    for k in ("max_depth", "min_samples_split", "n_features_", "classes_", "tree_"):
        assert k in state
    c2 = pickle.loads(blob)
    assert c2.export_text() == clf.export_text()
    np.testing.assert_array_equal(c2.predict(X), clf.predict(X))
    root = c2.tree_
    assert isinstance(root, Node) and root._btype is BranchType.ROOT
    assert root.left.parent is root and root.left.depth == 1


def test_reference_style_pickle_without_new_params(iris2):
    # a state dict with only the reference keys (what the reference writes)
    X, y, _ = iris2
    clf = DecisionTreeClassifier(max_depth=2).fit(X, y)
    state = {k: v for k, v in clf.__getstate__().items()
             if k in ("max_depth", "min_samples_split", "n_features_", "classes_", "tree_")}
    fresh = DecisionTreeClassifier.__new__(DecisionTreeClassifier)
    fresh.__setstate__(state)
    np.testing.assert_array_equal(fresh.predict(X), clf.predict(X))
    assert fresh.export_text() == clf.export_text()


def test_safe_checkpoint_loader(tmp_path, iris2):
    from mpitree_amd.utils import checkpoint

    X, y, _ = iris2
    clf = DecisionTreeClassifier(max_depth=3).fit(X, y)
    p = tmp_path / "tree.pkl"
    clf.save(p)
    c2 = DecisionTreeClassifier.load(p)
    assert c2.export_text() == clf.export_text()

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    with pytest.raises(pickle.UnpicklingError):
        checkpoint.loads(pickle.dumps(Evil()))


def test_node_lt_side_effects_match_reference_contract():
    leaf_l = Node(value=0)
    leaf_r = Node(value=1)
    assert sorted([leaf_l, leaf_r]) == [leaf_l, leaf_r]
    assert leaf_l._btype is BranchType.INTERIOR_LIKE and leaf_r._btype is BranchType.LEAF_LIKE
    inner = Node(value=0, threshold=1.0)
    inner.left, inner.right = Node(value=0), Node(value=1)
    out = sorted([leaf_l, inner])
    assert out == [inner, leaf_l] and inner._btype is BranchType.INTERIOR_LIKE


def test_agreement_with_sklearn_entropy_tree():
    from sklearn.tree import DecisionTreeClassifier as SK

    rng = np.random.default_rng(8)
    X = rng.integers(0, 20, size=(2000, 5)).astype(float)
    y = ((X[:, 0] + X[:, 1] * 0.5 + rng.normal(scale=3, size=2000)) > 14).astype(int)
    ours = DecisionTreeClassifier(max_depth=6).fit(X, y)
    sk = SK(criterion="entropy", max_depth=6, random_state=0).fit(X, y)
    agree = (ours.predict(X) == sk.predict(X)).mean()
    assert agree > 0.97
    assert abs(ours.score(X, y) - sk.score(X, y)) < 0.02


def test_regressor_api():
    rng = np.random.default_rng(9)
    X = rng.integers(0, 10, size=(300, 3)).astype(float)
    y = X[:, 0] * 2.5 + rng.normal(scale=0.1, size=300)
    reg = DecisionTreeRegressor(max_depth=4).fit(X, y)
    assert reg.score(X, y) > 0.9
    full = DecisionTreeRegressor().fit(X, y)
    assert full.score(X, y) > 0.99
    from sklearn.tree import DecisionTreeRegressor as SKR

    sk = SKR(max_depth=4, random_state=0).fit(X, y)
    np.testing.assert_allclose(reg.predict(X), sk.predict(X), rtol=1e-9, atol=1e-9)


def test_parallel_class_attributes_without_process_group():
    assert ParallelDecisionTreeClassifier.WORLD_RANK == 0
    assert ParallelDecisionTreeClassifier.WORLD_SIZE == 1
    clf = ParallelDecisionTreeClassifier(max_depth=2)
    assert clf.WORLD_RANK == 0


def test_tree_digest_and_logger():
    import logging

    from mpitree_amd import DecisionTreeClassifier
    from mpitree_amd.utils.observability import logger, tree_digest

    rng = np.random.default_rng(0)
    X = rng.integers(0, 9, size=(300, 4))
    y = rng.integers(0, 3, size=300)
    a = DecisionTreeClassifier(device="cpu").fit(X, y).tree_arrays_
    b = DecisionTreeClassifier(device="cpu").fit(X, y).tree_arrays_
    c = DecisionTreeClassifier(max_depth=2, device="cpu").fit(X, y).tree_arrays_
    assert tree_digest(a) == tree_digest(b) != tree_digest(c)
    assert 0 <= tree_digest(a) < 2**63
    assert logger.name == "mpitree" and logger.level == logging.NOTSET


def test_fault_injection_helper(monkeypatch):
    from mpitree_amd.utils.observability import InjectedFault, maybe_inject_fault

    maybe_inject_fault(0)  # unset: no-op
    monkeypatch.setenv("MPITREE_FAULT_RANK", "1")
    maybe_inject_fault(0)
    with pytest.raises(InjectedFault):
        maybe_inject_fault(1)
    monkeypatch.setenv("MPITREE_FAULT_AT", "level")
    maybe_inject_fault(1)  # different site
