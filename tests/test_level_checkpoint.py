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
@pytest.mark.parametrize("regression", [False, True])
def test_gpu_resume_equals_device_loop(tmp_path, regression):
    """A checkpointed GPU fit keeps the device-driven level loop; interrupted
    after level 3 and resumed, it restores the loop's device state and builds
    the uninterrupted tree."""
    from mpitree_amd.utils.datasets import make_classification, make_regression

    if regression:
        X, y = make_regression(150_000, 12, levels=64, seed=3, device="cuda")
        make = lambda: DecisionTreeRegressor(device="cuda")  # noqa: E731
    else:
        X, y = make_classification(200_000, 16, n_classes=3, seed=2, device="cuda")
        make = lambda: DecisionTreeClassifier(device="cuda")  # noqa: E731
    ref = make().fit(X, y)
    assert ref.fit_stats_["engine"] == "hip-device-loop"
    full = make().fit(X, y, checkpoint=str(tmp_path / "f.npz"))
    assert full.fit_stats_["engine"] == "hip-device-loop"
    assert full.fit_stats_["checkpoint_levels_saved"] >= 3
    assert full._arrays.equal(ref._arrays, check_impurity=False)
    res = _interrupted_then_resumed(make, X, y, tmp_path / "g.npz", 3)
    assert res.fit_stats_["engine"] == "hip-device-loop"
    assert res._arrays.equal(ref._arrays, check_impurity=False)
    a, b = res.predict(X[:5000]), ref.predict(X[:5000])
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("regression,stop", [(False, 3), (False, 11), (True, 5)])
def test_gpu_exact_resume_equals_uninterrupted(tmp_path, regression, stop):
    """The exact (continuous-threshold) list engine resumes too: interrupted after
    a level -- before and after the first finisher jobs -- and resumed, it
    restores both list buffers, the frontier, the position space and the jobs,
    and builds the uninterrupted tree."""
    from mpitree_amd.utils.datasets import make_classification, make_regression

    if regression:
        X, y = make_regression(60_000, 10, levels=None, seed=4, device="cuda")
        make = lambda: DecisionTreeRegressor(device="cuda")  # noqa: E731
    else:
        X, y = make_classification(80_000, 10, levels=None, seed=4, device="cuda")
        make = lambda: DecisionTreeClassifier(device="cuda")  # noqa: E731
    ref = make().fit(X, y)
    assert ref.fit_stats_["engine"] == "hip-exact"
    res = _interrupted_then_resumed(make, X, y, tmp_path / "x.npz", stop)
    assert res.fit_stats_["engine"] == "hip-exact"
    assert res.fit_stats_["checkpoint_levels_saved"] >= 1
    assert res._arrays.equal(ref._arrays, check_impurity=False)
    np.testing.assert_array_equal(res.tree_arrays_.threshold, ref.tree_arrays_.threshold)


def _ckpt_rank(rank, world, path, strategy, stop):
    import torch

    from mpitree_amd import ParallelDecisionTreeClassifier
    from mpitree_amd.utils.datasets import make_classification

    dev = torch.device("cuda", 0)
    if strategy == "exact":  # continuous features: the feature-parallel list engine
        X, y = make_classification(80_000, 10, levels=None, seed=9, device=dev)
        strategy = "auto"
    else:
        X, y = make_classification(200_000, 16, seed=9, device=dev)
    make = lambda: ParallelDecisionTreeClassifier(strategy=strategy, device="cuda")  # noqa: E731
    ck = LevelCheckpoint(path)
    ck.fail_after_level = stop
    try:
        make().fit(X, y, checkpoint=ck)
        raised = 0
    except CheckpointInterrupt:
        raised = 1
    est = make().fit(X, y, checkpoint=path)
    ta = est.tree_arrays_
    left = [f for f in os.listdir(os.path.dirname(path)) if f.startswith(os.path.basename(path))]
    return dict(feature=ta.feature, threshold=ta.threshold, n=ta.n_samples,
                raised=np.array([raised]), resumed=np.array([est.fit_stats_["resumed_from_level"]]),
                engine=np.array([est.fit_stats_["engine"]]), left=np.array([len(left)]))


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["data", "feature", "exact"])
def test_gpu_ranks_resume(tmp_path, strategy):
    """Two ranks (gloo, sharing one GPU): per-rank device-loop (or exact list
    engine) checkpoints, the ranks agree on the level to resume from, and the
    resumed trees equal the single-GPU tree."""
    import torch

    from mpitree_amd.utils.datasets import make_classification
    from tests.dist_utils import run_ranks

    path = str(tmp_path / "d.npz")
    outs = run_ranks(_ckpt_rank, 2, path, strategy, 2, start_method="spawn")
    dev = torch.device("cuda", 0)
    if strategy == "exact":
        X, y = make_classification(80_000, 10, levels=None, seed=9, device=dev)
    else:
        X, y = make_classification(200_000, 16, seed=9, device=dev)
    ref = DecisionTreeClassifier(device="cuda").fit(X, y).tree_arrays_
    for o in outs:
        assert int(o["raised"][0]) == 1 and int(o["resumed"][0]) == 2
        assert str(o["engine"][0]) == ("hip-exact" if strategy == "exact" else "hip-device-loop")
        assert int(o["left"][0]) == 0  # every rank's files removed after the fit
        np.testing.assert_array_equal(o["feature"], ref.feature)
        np.testing.assert_array_equal(o["threshold"], ref.threshold)
        np.testing.assert_array_equal(o["n"], ref.n_samples)


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


def test_device_checkpoint_generations_agree(tmp_path):
    """Multi-rank device checkpoints: two generations per rank, and the ranks
    resume from the newest level all of them hold (a crash between two ranks'
    writes leaves them one level apart)."""
    path = str(tmp_path / "m.npz")
    cks = [LevelCheckpoint(path, "sig") for _ in range(2)]
    for lvl in (1, 2, 3):
        cks[0].save_device(lvl, {"x": np.array([lvl])}, rank=0, world=2)
    for lvl in (1, 2):  # rank 1 died before writing level 3
        cks[1].save_device(lvl, {"x": np.array([lvl])}, rank=1, world=2)
    have = [np.array([2, 3]), np.array([1, 2])]
    gather = lambda a: np.stack(have)  # noqa: E731
    for r in range(2):
        st = LevelCheckpoint(path, "sig").load_device(rank=r, world=2, gather=gather)
        assert int(st["level"][0]) == 2 and int(st["x"][0]) == 2
    assert LevelCheckpoint(path, "other").load_device(0, 2, lambda a: np.stack(
        [a, a])) is None  # different problem: nothing to resume
    for r, ck in enumerate(cks):
        ck.clear()
    assert not [f for f in os.listdir(tmp_path) if f.startswith("m.npz")]


def test_device_checkpoint_every_other_level_keeps_two_generations(tmp_path):
    """MPITREE_CKPT_EVERY=2 saves levels 1, 3, 5 (one parity): the generations
    alternate by save count, so the two newest levels are both on disk."""
    path = str(tmp_path / "e.npz")
    ck = LevelCheckpoint(path, "sig")
    for lvl in (1, 3, 5):
        ck.save_device(lvl, {"x": np.array([lvl])}, rank=0, world=2)
    levels = set()
    for g in (0, 1):
        with np.load(f"{path}.r0of2.g{g}.npz", allow_pickle=False) as z:
            levels.add(int(z["level"][0]))
    assert levels == {3, 5}
    ck.clear()


def test_device_checkpoint_of_other_layout_is_ignored(tmp_path):
    """A device-loop state saved with other finisher rows / buffer sizes (ADVICE
    r5: MPITREE_EXACT_FINISHER_ROWS or chunk size changed between the runs) is
    ignored instead of failing to copy into differently sized buffers."""
    path = str(tmp_path / "l.npz")
    ck = LevelCheckpoint(path, "sig")
    ck.layout = "exact fr=256 K=10"
    ck.save_device(4, {"x": np.array([4])})
    same = LevelCheckpoint(path, "sig")
    same.layout = "exact fr=256 K=10"
    assert int(same.load_device()["level"][0]) == 4
    other = LevelCheckpoint(path, "sig")
    other.layout = "exact fr=0 K=99"
    assert other.load_device() is None
    ck.clear()
