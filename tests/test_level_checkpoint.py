"""Level-granular checkpoint / resume (utils/level_checkpoint.py)."""

import os

import numpy as np
import pytest

from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
from mpitree_amd.utils.level_checkpoint import CheckpointInterrupt, LevelCheckpoint
from tests.helpers import random_problem


def _interrupted_then_resumed(make, X, y, path, stop):
    ck = LevelCheckpoint(path)
    ck.fail_after_level = stop
    with pytest.raises(CheckpointInterrupt):
        make().fit(X, y, checkpoint=ck)
    assert os.path.exists(path)
    est = make().fit(X, y, checkpoint=str(path))
    assert est.fit_stats_["resumed_from_level"] == stop
    assert not os.path.exists(path)  # removed once the fit completes
    return est


@pytest.mark.parametrize("stop", [1, 3, 6])
@pytest.mark.parametrize("crit", ["entropy", "gini"])
def test_classifier_resume_equals_uninterrupted(tmp_path, stop, crit):
    rng = np.random.default_rng(11)
    X, y = random_problem(rng, 3000, 6, 4, 13)
    make = lambda: DecisionTreeClassifier(criterion=crit, device="cpu")  # noqa: E731
    ref = make().fit(X, y)
    full = make().fit(X, y, checkpoint=str(tmp_path / "a.npz"))
    assert full.fit_stats_["engine"] == "numpy-levelwise"
    assert full.fit_stats_["checkpoint_levels_saved"] >= stop
    assert full._arrays.equal(ref._arrays)
    res = _interrupted_then_resumed(make, X, y, tmp_path / "b.npz", stop)
    assert res._arrays.equal(ref._arrays)
    assert res.export_text() == ref.export_text()


def test_regressor_resume_equals_uninterrupted(tmp_path):
    rng = np.random.default_rng(12)
    X, y = random_problem(rng, 2000, 5, 0, 11, regression=True)
    make = lambda: DecisionTreeRegressor(max_depth=9, device="cpu")  # noqa: E731
    ref = make().fit(X, y)
    res = _interrupted_then_resumed(make, X, y, tmp_path / "r.npz", 4)
    assert res._arrays.equal(ref._arrays, check_impurity=False)
    np.testing.assert_array_equal(res.predict(X), ref.predict(X))


def test_checkpoint_of_other_data_is_ignored(tmp_path):
    rng = np.random.default_rng(13)
    X, y = random_problem(rng, 1500, 4, 3, 9)
    path = tmp_path / "c.npz"
    ck = LevelCheckpoint(path)
    ck.fail_after_level = 2
    with pytest.raises(CheckpointInterrupt):
        DecisionTreeClassifier(device="cpu").fit(X, y, checkpoint=ck)
    y2 = (y + 1) % 3
    est = DecisionTreeClassifier(device="cpu").fit(X, y2, checkpoint=str(path))
    assert "resumed_from_level" not in est.fit_stats_
    assert est._arrays.equal(DecisionTreeClassifier(device="cpu").fit(X, y2)._arrays)


@pytest.mark.gpu
def test_gpu_resume_equals_device_loop(tmp_path):
    import torch

    from mpitree_amd.utils.datasets import make_classification

    X, y = make_classification(200_000, 16, n_classes=3, seed=2, device="cuda")
    make = lambda: DecisionTreeClassifier(device="cuda")  # noqa: E731
    ref = make().fit(X, y)
    assert ref.fit_stats_["engine"] == "hip-device-loop"
    res = _interrupted_then_resumed(make, X, y, tmp_path / "g.npz", 3)
    assert res.fit_stats_["engine"] == "hip-levelwise"
    assert res._arrays.equal(ref._arrays, check_impurity=False)
    assert torch.cuda.is_available()


def test_signature_covers_every_row():
    """a change to any single row must change the signature."""
    from mpitree_amd.core.levelwise import GrowParams
    from mpitree_amd.utils.level_checkpoint import problem_signature

    rng = np.random.default_rng(0)
    codes = rng.integers(0, 8, size=(20000, 3)).astype(np.uint8)
    y = rng.integers(0, 2, size=20000).astype(np.int32)
    p = GrowParams()
    base = problem_signature(codes, y, p, 2)
    for r in (1, 4097, 19999):
        c2 = codes.copy()
        c2[r, 1] ^= 1
        assert problem_signature(c2, y, p, 2) != base
        y2 = y.copy()
        y2[r] ^= 1
        assert problem_signature(codes, y2, p, 2) != base
