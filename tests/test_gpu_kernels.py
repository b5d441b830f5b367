"""gfx950 kernels vs the host oracle (exact equality: every quantity is integer
or produced by the shared criterion with identical IEEE operations)."""

import numpy as np
import pytest
import torch

from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
from mpitree_amd.core.criterion import Criterion, xlog2x

from .helpers import oracle, random_problem

pytestmark = pytest.mark.gpu


def test_native_extension_loaded():
    from mpitree_amd.ops import native

    hip = native.hip()
    assert hip.__file__.startswith(str(__import__("pathlib").Path(__file__).parents[1]))


def test_xlog2x_device_matches_host_bitwise():
    from mpitree_amd.ops import native

    n = 1 << 20
    out = torch.empty(n, dtype=torch.float64, device="cuda")
    native.hip().xlog2x_device(torch.cuda.current_stream().cuda_stream, out.data_ptr(), n)
    dev = out.cpu().numpy()
    host = xlog2x(np.arange(n, dtype=np.int64))
    assert np.array_equal(dev.view(np.int64), host.view(np.int64))


def test_hw_log_terms_error_bound():
    # the exact engine's two-class fp32 prefilter (exact2.hip) computes its terms
    # as x * v_log_f32(x); its 2^-17 T(m) candidate pad assumes |error| <= 4 * 2^-24 *
    # x log2 x for every count (checked here up to 2^22) and exact zeros at 0, 1
    from mpitree_amd.ops import native

    n = 1 << 22
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    native.hip().hw_xlog2x_device(torch.cuda.current_stream().cuda_stream, out.data_ptr(), n)
    dev = out.cpu().numpy().astype(np.float64)
    exact = xlog2x(np.arange(n, dtype=np.int64))
    assert dev[0] == 0.0 and dev[1] == 0.0
    rel = np.abs(dev[2:] - exact[2:]) / exact[2:]
    assert rel.max() <= 4 * 2.0 ** -24, rel.max()


@pytest.mark.parametrize("crit", ["entropy", "gini"])
@pytest.mark.parametrize("seed", range(4))
def test_gpu_classifier_matches_oracle(crit, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(50, 3000))
    F = int(rng.integers(1, 12))
    C = int(rng.integers(2, 6))
    X, y = random_problem(rng, n, F, C, levels=int(rng.integers(2, 40)))
    md = [None, 4, 8, None][seed]
    ref = oracle(X, y, Criterion.ENTROPY if crit == "entropy" else Criterion.GINI, md)
    clf = DecisionTreeClassifier(max_depth=md, criterion=crit, device="cuda").fit(X, y)
    assert clf.fit_stats_["engine"].startswith("hip")
    assert clf.tree_arrays_.equal(ref), (clf.tree_arrays_.node_count, ref.node_count)
    Xd = torch.from_numpy(X).cuda()
    np.testing.assert_array_equal(clf.predict(Xd).cpu().numpy(), clf.predict(X))


@pytest.mark.parametrize("F", [600, 1000])
def test_gpu_wide_regression_tiny_kernel_matches_host(F):
    # past ~300 features the regression tiny-subtree kernel runs 2-wave (past ~590:
    # 1-wave) workgroups; the tree must equal the host builder's
    rng = np.random.default_rng(F)
    n = 3000
    X = rng.integers(0, 200, size=(n, F)).astype(np.float32)
    y = X[:, 0] * 0.5 + X[:, 1] - X[:, 7] + rng.normal(0, 5, n)
    g = DecisionTreeRegressor(device="cuda").fit(torch.from_numpy(X).cuda(),
                                                  torch.from_numpy(y).cuda())
    h = DecisionTreeRegressor(device="cpu").fit(X, y)
    assert g.fit_stats_["engine"].startswith("hip")
    assert g.tree_arrays_.equal(h.tree_arrays_, check_impurity=False)


@pytest.mark.parametrize("seed", range(3))
def test_gpu_regressor_matches_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(50, 2000))
    F = int(rng.integers(1, 8))
    X, y = random_problem(rng, n, F, 0, levels=int(rng.integers(2, 30)), regression=True)
    md = [None, 5, 3][seed]
    ref = oracle(X, y, Criterion.SQUARED_ERROR, md, regression=True)
    reg = DecisionTreeRegressor(max_depth=md, device="cuda").fit(X, y)
    assert reg.tree_arrays_.equal(ref, check_impurity=False)
    np.testing.assert_array_equal(reg.tree_arrays_.value, ref.value)


def test_gpu_iris_goldens(iris2):
    from .conftest import GOLDEN_DEPTH3, GOLDEN_DEPTH5

    X, y, iris = iris2
    clf = DecisionTreeClassifier(max_depth=3, device="cuda").fit(X, y)
    assert clf.export_text(feature_names=iris.feature_names,
                           class_names=iris.target_names) == GOLDEN_DEPTH3
    clf = DecisionTreeClassifier(max_depth=5, device="cuda").fit(X, y)
    assert clf.export_text(feature_names=iris.feature_names, class_names=iris.target_names,
                           precision=1) == GOLDEN_DEPTH5


def test_gpu_large_multiitem_and_u16_bins():
    # > 2048 rows per node -> multi-item slabs + reduce; 300 unique values -> u16 codes
    rng = np.random.default_rng(7)
    n, F = 20000, 5
    X = rng.integers(0, 300, size=(n, F)).astype(np.float32)
    y = (X[:, 0] + rng.normal(scale=40, size=n) > 150).astype(np.int64)
    ref = oracle(X.astype(np.float64), y, Criterion.ENTROPY, 6, max_bins=512)
    clf = DecisionTreeClassifier(max_depth=6, max_bins=512, device="cuda").fit(
        torch.from_numpy(X).cuda(), torch.from_numpy(y).cuda())
    assert clf.tree_arrays_.equal(ref)


def test_gpu_quantile_bins_consistent_predict():
    rng = np.random.default_rng(3)
    n, F = 50000, 8
    X = rng.normal(size=(n, F)).astype(np.float32)
    y = (X[:, 0] * X[:, 1] > 0).astype(np.int64)
    Xd = torch.from_numpy(X).cuda()
    # quantile bins are opt-in (exact thresholds are the default; on this XOR
    # problem the exact greedy tree scores 0.807 at depth 8 on CPU and GPU alike)
    clf = DecisionTreeClassifier(max_depth=8, max_bins=256, device="cuda").fit(
        Xd, torch.from_numpy(y).cuda())
    # device and host traversal agree exactly on the raw values
    np.testing.assert_array_equal(clf.apply(Xd).cpu().numpy(), clf.tree_arrays_.apply(X))
    assert clf.score(X, y) > 0.9


@pytest.mark.parametrize("rows", ["16", "200", "5000"])
@pytest.mark.parametrize("crit", ["entropy", "gini"])
def test_gpu_finisher_matches_oracle(monkeypatch, rows, crit):
    monkeypatch.setenv("MPITREE_FINISHER_ROWS", rows)
    rng = np.random.default_rng(int(rows) + len(crit))
    n, F, C = 6000, 6, 3
    X, y = random_problem(rng, n, F, C, levels=12)
    for md in (None, 7):
        ref = oracle(X, y, Criterion.ENTROPY if crit == "entropy" else Criterion.GINI, md)
        clf = DecisionTreeClassifier(max_depth=md, criterion=crit, device="cuda").fit(X, y)
        assert clf.tree_arrays_.equal(ref), (rows, md, clf.tree_arrays_.node_count, ref.node_count)
        if rows != "5000":
            assert clf.fit_stats_.get("finisher_subtrees", 0) > 0


def test_gpu_finisher_deep_chain(monkeypatch):
    # a fully grown tree whose splits peel one row at a time (deep, skinny)
    monkeypatch.setenv("MPITREE_FINISHER_ROWS", "1000")
    monkeypatch.setenv("MPITREE_SMALL_FIT", "0")  # (600 rows: the finisher, not small_fit)
    n = 600
    X = np.arange(n, dtype=np.float64).reshape(-1, 1)
    y = np.arange(n) % 7
    ref = oracle(X, y, Criterion.ENTROPY, None, max_bins=1024)
    clf = DecisionTreeClassifier(max_bins=1024, device="cuda").fit(X, y)
    assert clf.tree_arrays_.equal(ref)


@pytest.mark.parametrize("tiny", ["0", "8", "64"])
def test_gpu_tiny_subtree_wave_path(monkeypatch, tiny):
    # wave-per-subtree path for <= 64-row subtrees vs the oracle, many classes
    monkeypatch.setenv("MPITREE_TINY_ROWS", tiny)
    monkeypatch.setenv("MPITREE_FINISHER_ROWS", "400")
    rng = np.random.default_rng(77)
    n, F, C = 8000, 10, 5
    X, y = random_problem(rng, n, F, C, levels=30)
    for crit in ("entropy", "gini"):
        ref = oracle(X, y, Criterion.ENTROPY if crit == "entropy" else Criterion.GINI, None,
                     msl=2 if crit == "gini" else 1)
        clf = DecisionTreeClassifier(criterion=crit, device="cuda",
                                     min_samples_leaf=2 if crit == "gini" else 1).fit(X, y)
        assert clf.tree_arrays_.equal(ref), (tiny, crit)


@pytest.mark.parametrize("regression", [False, True])
def test_gpu_device_assembly_matches_host(monkeypatch, regression):
    """Pre-order position space + device compaction == host renumbering."""
    from mpitree_amd.core.fit import fit_tree

    rng = np.random.default_rng(7)
    n, F = 6000, 9
    X = rng.integers(0, 40, size=(n, F)).astype(np.float32)
    y = rng.normal(size=n) if regression else rng.integers(0, 3, size=n)
    kw = dict(regression=regression, criterion=2 if regression else 0, max_depth=None,
              min_samples_split=2, device="cuda", finisher_rows=None if regression else 700)
    monkeypatch.setenv("MPITREE_DEVICE_ASSEMBLY", "1")
    dev = fit_tree(X, y, **kw).arrays
    monkeypatch.setenv("MPITREE_DEVICE_ASSEMBLY", "0")
    host = fit_tree(X, y, **kw).arrays
    assert dev.equal(host, check_impurity=False)
    assert np.array_equal(dev.impurity, host.impurity, equal_nan=True)
    if regression:
        # (the device columns carry no fixed-point sums: value = sum / count is
        # computed on the device from the same int64 sums)
        assert np.array_equal(dev.value, host.value)


def test_gpu_edges_match_host_mapper():
    """Device edges (hash-set exact mode, bitonic-sort quantiles) == host BinMapper."""
    from mpitree_amd.core.binning import fit_bin_mapper
    from mpitree_amd.ops.hip_backend import gpu_bin_features

    rng = np.random.default_rng(3)
    n = 20000  # below the device sample size: both sides see every row
    X = np.stack([
        rng.normal(size=n),                       # continuous -> quantiles
        rng.integers(0, 7, size=n),               # 7 levels -> exact
        rng.integers(0, 256, size=n),             # 256 levels -> exact at the limit
        rng.integers(0, 300, size=n),             # 300 levels -> quantiles
        np.where(rng.random(n) < 0.5, -0.0, 0.0),  # signed zeros are one value
    ], 1).astype(np.float32)
    host = fit_bin_mapper(X, 256)
    mapper, codes_rm, codes_fm, nb = gpu_bin_features(torch.from_numpy(X).cuda(), 256)
    for f in range(X.shape[1]):
        assert bool(mapper.exact[f]) == bool(host.exact[f]), f
        assert np.array_equal(mapper.edges[f], host.edges[f]), f
    assert np.array_equal(codes_fm.cpu().numpy().T[:, :5], host.transform(X))


def test_gpu_bin_rows_consecutive_integer_edges():
    """Row-streaming binning (F % 4 == 0): columns whose edges are consecutive
    integers take the subtraction path; every other column the LDS search.
    Both code layouts equal the host BinMapper's transform."""
    from mpitree_amd.core.binning import fit_bin_mapper
    from mpitree_amd.ops.hip_backend import gpu_bin_features

    rng = np.random.default_rng(11)
    n = 20000
    cols = [
        rng.integers(0, 256, size=n),              # 0..255: consecutive
        rng.integers(1000, 1100, size=n),          # offset range: consecutive
        rng.integers(-50, 50, size=n),             # negative start: consecutive
        2 * rng.integers(0, 100, size=n),          # even values: gaps -> search
        rng.integers(0, 100, size=n) + 0.5,        # half-integers -> search
        rng.normal(size=n),                        # quantiles -> search
        rng.integers(0, 3, size=n),                # 3 levels: consecutive
        np.full(n, 7.0),                           # constant: one edge
    ]
    X = np.stack(cols, 1).astype(np.float32)
    host = fit_bin_mapper(X, 256)
    mapper, codes_rm, codes_fm, nb = gpu_bin_features(torch.from_numpy(X).cuda(), 256)
    want = host.transform(X)
    assert np.array_equal(codes_fm.cpu().numpy().T[:, : X.shape[1]], want)
    assert np.array_equal(codes_rm.cpu().numpy()[:, : X.shape[1]], want)


@pytest.mark.parametrize("labels", ["int64", "int32-gaps", "negative", "float", "host"])
def test_gpu_label_prepare_paths(labels):
    """Device label encoding (range count + LUT, gpu_prepare) == host np.unique,
    and the tree equals the one grown from host labels."""
    from mpitree_amd.core.fit import fit_tree

    rng = np.random.default_rng(11)
    n = 20000
    X = rng.integers(0, 30, size=(n, 5)).astype(np.float32)
    base = (X[:, 0] + rng.integers(0, 9, size=n)) % 3
    yh = {"int64": base, "int32-gaps": np.array([3, 7, 100])[base.astype(int)],
          "negative": base.astype(int) - 5, "float": base * 0.5, "host": base}[labels]
    if labels == "int32-gaps":
        yh = yh.astype(np.int32)
    yd = yh if labels == "host" else torch.from_numpy(np.ascontiguousarray(yh)).cuda()
    kw = dict(regression=False, criterion=0, max_depth=None, min_samples_split=2,
              device="cuda")
    r_dev = fit_tree(torch.from_numpy(X).cuda(), yd, **kw)
    r_cpu = fit_tree(X, yh, **{**kw, "device": "cpu"})
    assert np.array_equal(r_dev.classes, np.unique(yh))
    assert r_dev.classes.dtype == np.unique(yh).dtype
    assert r_dev.arrays.equal(r_cpu.arrays, check_impurity=False)


def test_gpu_regression_prepare_device_targets():
    """Fixed-point targets and root stats computed on the device == host path."""
    from mpitree_amd.core.fit import fit_tree

    rng = np.random.default_rng(12)
    n = 30000
    X = rng.integers(0, 40, size=(n, 6)).astype(np.float32)
    y = X[:, 0] * 0.25 + rng.normal(size=n)
    kw = dict(regression=True, criterion=2, max_depth=None, min_samples_split=2, device="cuda")
    a = fit_tree(torch.from_numpy(X).cuda(), torch.from_numpy(y).cuda(), **kw)
    b = fit_tree(X, y, **kw)
    assert a.y_scale_exp == b.y_scale_exp
    assert a.arrays.equal(b.arrays, check_impurity=False)
    assert np.array_equal(a.arrays.value, b.arrays.value)
    with pytest.raises(ValueError, match="NaN or infinity"):
        yb = torch.from_numpy(y).cuda()
        yb[5] = float("inf")
        fit_tree(torch.from_numpy(X).cuda(), yb, **kw)


def test_gpu_job_sort_kernel_matches_torch_order(monkeypatch):
    """The one-workgroup job sort and the torch argsort fallback give the same tree."""
    from mpitree_amd.core.fit import fit_tree
    from mpitree_amd.ops import native

    rng = np.random.default_rng(13)
    n = 50000
    X = rng.integers(0, 50, size=(n, 7)).astype(np.float32)
    y = (X[:, 1] + rng.integers(0, 20, size=n)) % 2
    kw = dict(regression=False, criterion=1, max_depth=None, min_samples_split=2,
              device="cuda", finisher_rows=300)
    a = fit_tree(X, y, **kw)
    assert a.stats["finisher_subtrees"] > 1
    monkeypatch.setattr(native.hip(), "job_sort_max", lambda: 0)
    b = fit_tree(X, y, **kw)
    assert a.arrays.equal(b.arrays)


def test_gpu_sample_missed_value_redoes_fit():
    """The first sync no longer waits for the bin kernel's flags: a value the
    strided edge sample skipped is found after growth and the fit is redone
    with the flags checked first -- the tree equals the host fit."""
    from mpitree_amd.core.fit import fit_tree
    from mpitree_amd.ops.hip_backend import DeviceBinning

    rng = np.random.default_rng(21)
    n = 200_000
    X = rng.integers(0, 8, size=(n, 3)).astype(np.float32)
    y = ((X[:, 0] + X[:, 1]) > 7).astype(np.int64)
    for r in range(1, 64):
        X2, y2 = X.copy(), y.copy()
        X2[r, 0], y2[r] = 3.5, 1 - y2[r]
        job = DeviceBinning(torch.from_numpy(X2).cuda(), 256)
        torch.cuda.synchronize()
        job.launch_bin()
        torch.cuda.synchronize()
        if np.array(job._host_flags)[0] & 1:
            break
    else:
        pytest.skip("the edge sample covers every probed row")
    kw = dict(regression=False, criterion=1, max_depth=None, min_samples_split=2)
    a = fit_tree(torch.from_numpy(X2).cuda(), torch.from_numpy(y2).cuda(), device="cuda", **kw)
    b = fit_tree(X2, y2, device="cpu", **kw)
    assert 3.5 in a.mapper.edges[0]
    assert a.arrays.equal(b.arrays)


def test_gpu_rejects_nonfinite_tensor():
    X = torch.zeros((1000, 3), device="cuda")
    X[17, 1] = float("nan")
    with pytest.raises(ValueError, match="NaN or infinity"):
        DecisionTreeClassifier(device="cuda").fit(X, torch.zeros(1000, device="cuda"))


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("max_depth", [None, 7])
def test_gpu_device_loop_matches_host_loop(monkeypatch, seed, max_depth):
    """Device-planned level loop (grow.hip) == host-driven level-wise builder."""
    from mpitree_amd.core.fit import fit_tree

    rng = np.random.default_rng(100 + seed)
    n, F, C = 30000 + 7000 * seed, 11, 2 + seed
    X = rng.integers(0, 60, size=(n, F)).astype(np.float32)
    y = (X[:, 0] + X[:, 1] * (seed + 1) + rng.integers(0, 40, size=n)) % C
    kw = dict(regression=False, criterion=seed % 2, max_depth=max_depth, min_samples_split=2,
              device="cuda", finisher_rows=500)
    monkeypatch.setenv("MPITREE_DEVICE_LOOP", "1")
    r1 = fit_tree(X, y, **kw)
    assert r1.engine == "hip-device-loop"
    monkeypatch.setenv("MPITREE_DEVICE_LOOP", "0")
    r2 = fit_tree(X, y, **kw)
    assert r2.engine == "hip-levelwise"
    assert r1.arrays.equal(r2.arrays)
    assert np.array_equal(r1.arrays.impurity, r2.arrays.impurity)


@pytest.mark.parametrize("C,crit,levels", [(2, 0, 1000), (3, 1, 600), (2, 1, 4000), (5, 0, 300)])
def test_gpu_device_loop_wide_bins(monkeypatch, C, crit, levels):
    """More than 256 bins (16-bit codes): the device level loop and the block
    finisher's multi-pass scans (finish.hip) == the host-driven builder."""
    from mpitree_amd.core.fit import fit_tree

    rng = np.random.default_rng(levels + C)
    n, F = 60000, 7
    X = rng.integers(0, levels, size=(n, F)).astype(np.float32)
    y = (X[:, 0] * 3 // levels + X[:, 1] * 2 // levels + rng.integers(0, 2, size=n)) % C
    kw = dict(regression=False, criterion=crit, max_depth=None, min_samples_split=2,
              device="cuda", max_bins=4096)
    monkeypatch.setenv("MPITREE_DEVICE_LOOP", "1")
    r1 = fit_tree(X, y, **kw)
    assert r1.engine == "hip-device-loop"
    assert r1.stats["finisher_subtrees"] > 0
    monkeypatch.setenv("MPITREE_DEVICE_LOOP", "0")
    r2 = fit_tree(X, y, **kw)
    assert r2.engine == "hip-levelwise"
    assert r1.arrays.equal(r2.arrays)
    assert np.array_equal(r1.arrays.impurity, r2.arrays.impurity)


def test_gpu_profile_mode_level_events(monkeypatch):
    monkeypatch.setenv("MPITREE_PROFILE", "1")
    rng = np.random.default_rng(5)
    X = rng.integers(0, 50, size=(40000, 6)).astype(np.float32)
    y = (X[:, 0] + rng.integers(0, 30, size=40000)) % 2
    est = DecisionTreeClassifier(device="cuda").fit(X, y)
    st = est.fit_stats_
    assert st["engine"] == "hip-device-loop"
    prof = st["level_profile"]
    assert len(prof) == st["levels"] and all(v >= 0 for row in prof for v in row.values())
    assert st["timings"]["device_hist"] > 0


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("max_depth", [None, 9])
def test_gpu_regression_device_loop_matches_host(monkeypatch, seed, max_depth):
    """Regression: device loop + regression finisher == host loop == numpy oracle."""
    from mpitree_amd.core.fit import fit_tree

    rng = np.random.default_rng(300 + seed)
    n, F = 20000 + 5000 * seed, 7
    X = rng.integers(0, 40, size=(n, F)).astype(np.float32)
    # repeated target values so that pure (all-equal) nodes occur
    y = np.round(X[:, 0] * 0.5 + X[:, 1] * (seed + 1) + rng.integers(0, 5, size=n), 1)
    kw = dict(regression=True, criterion=2, max_depth=max_depth, min_samples_split=2,
              device="cuda", finisher_rows=400)
    monkeypatch.setenv("MPITREE_DEVICE_LOOP", "1")
    r1 = fit_tree(X, y, **kw)
    assert r1.engine == "hip-device-loop"
    monkeypatch.setenv("MPITREE_DEVICE_LOOP", "0")
    r2 = fit_tree(X, y, **kw)
    assert r2.engine == "hip-levelwise"
    assert r1.arrays.equal(r2.arrays)
    assert np.array_equal(r1.arrays.value, r2.arrays.value)
    r3 = fit_tree(X, y, **{**kw, "device": "cpu"})
    assert r1.arrays.equal(r3.arrays)


@pytest.mark.parametrize("regression,C", [(False, 2), (False, 7), (True, 0)])
def test_gpu_derive_free_levels_match_host(monkeypatch, regression, C):
    """Derive-free levels (one histogram buffer; every child built from rows --
    what many-class fits too large for two level parities take): the same tree as
    the host builder."""
    from mpitree_amd.core.fit import fit_tree

    monkeypatch.setenv("MPITREE_DERIVE_FREE", "1")
    rng = np.random.default_rng(41 + C)
    X, y = random_problem(rng, 30000, 9, max(C, 2), 40, regression=regression)
    kw = dict(regression=regression, criterion=2 if regression else 0, max_depth=None,
              min_samples_split=2, finisher_rows=500)
    g = fit_tree(X, y, device="cuda", **kw)
    assert g.engine == "hip-device-loop" and g.stats.get("derive_free")
    h = fit_tree(X, y, device="cpu", **kw)
    assert g.arrays.equal(h.arrays)
    if regression:
        assert np.array_equal(g.arrays.value, h.arrays.value)


@pytest.mark.parametrize("F", [300, 600])
def test_gpu_regression_wide_features_device_loop(F):
    """Regression past 256 features runs the device level loop and the block
    finisher (features past its per-feature LDS arrays read their bin counts from
    memory; past ~512 features no tiny kernel): the host-built tree bit for bit."""
    from mpitree_amd.core.fit import fit_tree

    rng = np.random.default_rng(F)
    n = 6000
    X = rng.integers(0, 24, size=(n, F)).astype(np.float32)
    y = np.round(X[:, 0] * 0.5 + X[:, F - 1] * 1.5 + rng.integers(0, 5, size=n), 1)
    kw = dict(regression=True, criterion=2, max_depth=None, min_samples_split=2)
    g = fit_tree(X, y, device="cuda", **kw)
    assert g.engine == "hip-device-loop" and g.stats.get("finisher_subtrees", 0) > 0
    h = fit_tree(X, y, device="cpu", **kw)
    assert g.arrays.equal(h.arrays)
    assert np.array_equal(g.arrays.value, h.arrays.value)


@pytest.mark.parametrize("F", [100, 128])
def test_gpu_many_features_tiny_paths_match_host(F):
    """F > 64: the tiny kernels' lane-per-feature small-node path walks several
    64-feature chunks (the winning chunk's codes decide the partition)."""
    from mpitree_amd.utils.datasets import make_classification

    X, y = make_classification(60000, F, seed=F, device=torch.device("cuda"))
    g = DecisionTreeClassifier(device="cuda").fit(X, y)
    h = DecisionTreeClassifier(device="cpu").fit(X.cpu().numpy(), y.cpu().numpy())
    assert g.tree_arrays_.equal(h.tree_arrays_)


@pytest.mark.parametrize("kind", ["gauss", "mixed_scale", "cancel"])
def test_gpu_regression_tiny_prefilter_matches_host(kind):
    """Continuous targets (every row its own leaf): the tiny regression kernel's
    fp32 prefilter + exact rescoring gives the host builder's tree bit for bit,
    also for targets spanning many magnitudes and for sums that cancel."""
    from mpitree_amd.core.fit import fit_tree

    rng = np.random.default_rng({"gauss": 1, "mixed_scale": 2, "cancel": 3}[kind])
    n, F = 30000, 9
    X = rng.integers(0, 256, size=(n, F)).astype(np.float32)
    base = X[:, 0] / 64.0 + np.sin(X[:, 1] / 20.0)
    if kind == "gauss":
        y = base + rng.normal(size=n)
    elif kind == "mixed_scale":
        y = base * 10.0 ** rng.integers(-3, 7, size=n) * rng.choice([-1.0, 1.0], size=n)
    else:  # large opposite-sign pairs: node sums far below sum |y|
        y = 1e6 * rng.choice([-1.0, 1.0], size=n) + rng.normal(size=n)
    kw = dict(regression=True, criterion=2, max_depth=None, min_samples_split=2)
    g = fit_tree(X, y, device="cuda", **kw)
    assert g.engine == "hip-device-loop"
    h = fit_tree(X, y, device="cpu", **kw)
    assert g.arrays.equal(h.arrays)
    assert np.array_equal(g.arrays.value, h.arrays.value)


@pytest.mark.parametrize("crit", ["entropy", "gini"])
@pytest.mark.parametrize("shape", [(3000, 3, 2, None, 1), (20000, 6, 3, None, 1),
                                   (5000, 4, 5, 6, 1), (12000, 70, 2, None, 1),
                                   (8000, 5, 2, None, 3)])
def test_gpu_exact_engine_matches_host(crit, shape):
    """Continuous features (> 256 unique values) with the exact default: the
    presorted-list engine (exact2.hip), whose <= 256-row subtrees continue in the
    histogram finisher on local codes, builds the host builder's tree bit for bit."""
    n, F, C, md, msl = shape
    rng = np.random.default_rng(n + F)
    X = np.round(rng.normal(size=(n, F)), 4).astype(np.float32)
    X[:, 0] = np.round(X[:, 0], 1)  # many ties on one feature
    s = X[:, 0] + 0.7 * X[:, 1] + rng.normal(scale=0.8, size=n)
    y = np.digitize(s, np.quantile(s, np.linspace(0, 1, C + 1)[1:-1]))
    kw = dict(criterion=crit, max_depth=md, min_samples_leaf=msl, min_samples_split=2 * msl + 1)
    g = DecisionTreeClassifier(device="cuda", **kw).fit(X, y)
    assert g.fit_stats_["engine"] == "hip-exact"
    if md is None:
        assert g.fit_stats_.get("finisher_subtrees", 0) > 0
    h = DecisionTreeClassifier(device="cpu", **kw).fit(X, y)
    assert g.tree_arrays_.equal(h.tree_arrays_)
    np.testing.assert_array_equal(g.tree_arrays_.threshold, h.tree_arrays_.threshold)
    assert g.export_text(precision=17) == h.export_text(precision=17)
    np.testing.assert_array_equal(g.predict(X), h.predict(X))


def test_gpu_exact_setup_native_equals_torch_path():
    """float32 inputs take the native setup (exact_setup.hip: transposed keys,
    one radix sort, rank passes, xe_emit); float64 inputs the torch sort path.
    Negative zeros, negatives, many ties and > 256 values per feature: the same
    tree either way, equal to the host builder's."""
    rng = np.random.default_rng(21)
    n, F = 9000, 70
    X = np.round(rng.normal(size=(n, F)), 3).astype(np.float32)
    X[rng.random((n, F)) < 0.05] = -0.0
    X[:, 5] = np.round(X[:, 5], 0)
    y = rng.integers(0, 3, size=n)
    g32 = DecisionTreeClassifier(device="cuda").fit(X, y)
    g64 = DecisionTreeClassifier(device="cuda").fit(X.astype(np.float64), y)
    assert g32.fit_stats_["engine"] == g64.fit_stats_["engine"] == "hip-exact"
    assert g32.tree_arrays_.equal(g64.tree_arrays_)
    h = DecisionTreeClassifier(device="cpu").fit(X, y)
    assert g32.tree_arrays_.equal(h.tree_arrays_)


@pytest.mark.parametrize("n", [1, 4095, 4097, 300_001])
def test_gpu_exact_setup_sort_equals_stable_sort(n):
    """The batched one-sweep radix sort (exact_setup.hip) against torch's stable
    sort of each column (ties by row id, -0.0 == 0.0): sorted rows, per-chunk
    value-change counts and unique counts; a column block of a wider X (f_lo, xs)."""
    from mpitree_amd.ops import native

    hip = native.hip()
    rng = np.random.default_rng(n)
    F, f_lo, xs = 9, 2, 12
    Xh = rng.normal(size=(n, xs)).astype(np.float32)
    Xh[:, 3] = np.round(Xh[:, 3], 1)  # many ties
    Xh[:, 4] = 7.0  # one value
    Xh[rng.random((n, xs)) < 0.03] = -0.0
    Xh[rng.random((n, xs)) < 0.03] = 0.0
    X = torch.from_numpy(Xh).cuda()
    dev = X.device
    keys = [torch.empty((F, n), dtype=torch.int32, device=dev) for _ in range(2)]
    rows = [torch.empty((F, n), dtype=torch.int32, device=dev) for _ in range(2)]
    tb = int(hip.exact_setup_temp_bytes(n, F))
    temp = torch.empty(tb, dtype=torch.uint8, device=dev)
    chunk = int(hip.exact_setup_chunk())
    nc = -(-n // chunk)
    cnt = torch.empty((F, nc), dtype=torch.int32, device=dev)
    nuniq = torch.empty(F, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    hip.exact_setup_sort(s, X.data_ptr(), n, F, keys[0].data_ptr(), keys[1].data_ptr(),
                         rows[0].data_ptr(), rows[1].data_ptr(), temp.data_ptr(), tb,
                         cnt.data_ptr(), nuniq.data_ptr(), xs=xs, f_lo=f_lo)
    torch.cuda.synchronize()
    xt = (X[:, f_lo:f_lo + F] + 0.0).t().contiguous()
    vals, order = torch.sort(xt, dim=1, stable=True)
    assert torch.equal(rows[1].long(), order)
    new = torch.ones_like(vals, dtype=torch.int32)
    new[:, 1:] = (vals[:, 1:] != vals[:, :-1]).int()
    assert torch.equal(nuniq.cpu(), new.sum(1).int().cpu())
    pad = torch.zeros((F, nc * chunk), dtype=torch.int32, device=dev)
    pad[:, :n] = new
    per = pad.view(F, nc, chunk).sum(2)
    excl = torch.cumsum(per, 1) - per
    assert torch.equal(cnt.cpu(), excl.int().cpu())


@pytest.mark.parametrize("C", [130, 300])
def test_gpu_exact_many_classes_matches_host(C):
    """More than 128 classes on continuous features: labels leave the list
    entries (gathered by row); more than 256 classes also skip the local-code
    finisher (the list engine grows every level). Same tree as the host."""
    rng = np.random.default_rng(C)
    n, F = 6000, 3
    X = np.round(rng.normal(size=(n, F)), 3).astype(np.float32)
    s = X[:, 0] + 0.5 * X[:, 1]
    y = np.digitize(s, np.quantile(s, np.linspace(0, 1, C + 1)[1:-1]))
    g = DecisionTreeClassifier(device="cuda").fit(torch.from_numpy(X).cuda(),
                                                  torch.from_numpy(y).cuda())
    assert g.fit_stats_["engine"] == "hip-exact"
    assert "quantile" not in str(g.fit_stats_.get("thresholds", ""))
    h = DecisionTreeClassifier(device="cpu").fit(X, y)
    assert g.tree_arrays_.equal(h.tree_arrays_)
    np.testing.assert_array_equal(g.tree_arrays_.threshold, h.tree_arrays_.threshold)


def test_gpu_exact_n_classes_published_workload():
    """The reference's published timing workload at n = 5000: X = arange(n)
    (one feature), y = arange(n) (every row its own class). On the GPU the exact
    list engine grows it to n leaves -- the CPU tree, node for node."""
    n = 5000
    X = np.arange(n, dtype=np.float64).reshape(-1, 1)
    y = np.arange(n)
    g = DecisionTreeClassifier(device="cuda").fit(torch.from_numpy(X).cuda(),
                                                  torch.from_numpy(y).cuda())
    assert g.fit_stats_["engine"] == "hip-exact"
    h = DecisionTreeClassifier(device="cpu").fit(X, y)
    assert g.tree_arrays_.equal(h.tree_arrays_)
    assert int((g.tree_arrays_.feature < 0).sum()) == n
    np.testing.assert_array_equal(np.asarray(g.predict(X)), y)


@pytest.mark.parametrize("regression", [False, True])
def test_gpu_exact_wide_features_device_engine(regression):
    """More than 256 continuous features run the device-driven list engine
    (feature-tiled local-code finisher), equal to the host builder."""
    from mpitree_amd import DecisionTreeRegressor

    rng = np.random.default_rng(300)
    n, F = 4000, 300
    X = np.round(rng.normal(size=(n, F)), 3).astype(np.float32)
    s = X[:, 0] + X[:, 7] * X[:, 290] + rng.normal(scale=0.3, size=n)
    cls = DecisionTreeRegressor if regression else DecisionTreeClassifier
    yv = np.round(s, 2) if regression else (s > 0).astype(np.int64)
    g = cls(device="cuda", max_depth=12).fit(X, yv)
    assert g.fit_stats_["engine"] == "hip-exact"
    h = cls(device="cpu", max_depth=12).fit(X, yv)
    assert g.tree_arrays_.equal(h.tree_arrays_)


@pytest.mark.parametrize("F", [67, 131])
def test_gpu_exact_feature_count_without_batch_divisor(F):
    """F with no divisor in 4..16: the partition pads each sub-chunk's tickets to a
    multiple of its 16-ticket claims (skipped padding tickets); same tree as the
    host builder. (Unpadded, 500k x 67 took 123 ms against 10 ms.)"""
    rng = np.random.default_rng(F)
    n = 30000
    X = rng.normal(size=(n, F)).astype(np.float32)
    y = (X[:, 0] + X[:, F - 1] * X[:, 3] > 0).astype(np.int64)
    g = DecisionTreeClassifier(device="cuda").fit(X, y)
    assert g.fit_stats_["engine"] == "hip-exact"
    h = DecisionTreeClassifier(device="cpu").fit(X, y)
    assert g.tree_arrays_.equal(h.tree_arrays_)


def test_gpu_exact_finisher_handoff_same_tree(monkeypatch):
    """The exact engine's finisher hand-off changes no split: the same tree with
    the list engine growing every level (MPITREE_EXACT_FINISHER_ROWS=0)."""
    rng = np.random.default_rng(11)
    X = rng.normal(size=(30000, 12)).astype(np.float32)
    X[:, 3] = np.round(X[:, 3], 2)
    y = ((X[:, 0] + X[:, 1] * X[:, 2] + rng.normal(scale=0.5, size=30000)) > 0).astype(np.int64)
    a = DecisionTreeClassifier(device="cuda").fit(X, y)
    assert a.fit_stats_.get("finisher_subtrees", 0) > 0
    monkeypatch.setenv("MPITREE_EXACT_FINISHER_ROWS", "0")
    b = DecisionTreeClassifier(device="cuda").fit(X, y)
    assert b.fit_stats_.get("finisher_subtrees", 0) == 0
    assert a.tree_arrays_.equal(b.tree_arrays_)
    np.testing.assert_array_equal(a.tree_arrays_.threshold, b.tree_arrays_.threshold)


@pytest.mark.parametrize("n,F,regression", [(40000, 12, False), (30000, 40, False),
                                             (30000, 10, True), (1_300_000, 3, False)])
def test_gpu_exact_counted_partition_same_tree(monkeypatch, n, F, regression):
    """The counted partition (count, per-segment prefix, scatter; the default for
    <= 16 lists a rank) and the single-pass look-back partition build the same
    tree -- with the flags in LDS and, past 1.18M rows, read from global memory."""
    from mpitree_amd import DecisionTreeRegressor

    rng = np.random.default_rng(n + F)
    X = rng.normal(size=(n, F)).astype(np.float32)
    X[:, 1] = np.round(X[:, 1], 2)  # ties
    s = X[:, 0] + X[:, 1] * X[:, 2] + rng.normal(scale=0.5, size=n)
    y = s.astype(np.float64) if regression else (s > 0).astype(np.int64)
    cls = DecisionTreeRegressor if regression else DecisionTreeClassifier
    Xd, yd = torch.from_numpy(X).cuda(), torch.from_numpy(y).cuda()
    out = []
    for mode in ("0", "1"):
        monkeypatch.setenv("MPITREE_EXACT_PART_COUNTED", mode)
        est = cls(device="cuda", max_depth=14 if n > 10**6 else None).fit(Xd, yd)
        assert est.fit_stats_["engine"] == "hip-exact"
        out.append(est.tree_arrays_)
    assert out[0].equal(out[1], check_impurity=not regression)
    np.testing.assert_array_equal(out[0].threshold, out[1].threshold)


@pytest.mark.parametrize("shape", [(50000, 6, None, 1), (8000, 3, 5, 2)])
def test_gpu_exact_regression_matches_host(shape):
    """Regression on continuous features: exact thresholds on the GPU (the
    presorted-list engine's target prefix sums), equal to the host builder."""
    from mpitree_amd import DecisionTreeRegressor

    n, F, md, msl = shape
    rng = np.random.default_rng(n + F)
    X = rng.normal(size=(n, F)).astype(np.float32)
    X[:, 1] = np.round(X[:, 1], 2)  # ties on one feature
    y = X[:, 0] * 2.0 + np.sin(3 * X[:, 1]) + rng.normal(scale=0.3, size=n)
    kw = dict(max_depth=md, min_samples_leaf=msl)
    g = DecisionTreeRegressor(device="cuda", **kw).fit(X, y)
    assert g.fit_stats_["engine"] == "hip-exact", g.fit_stats_
    assert g.fit_stats_["thresholds"] == "exact (presorted lists)"
    h = DecisionTreeRegressor(device="cpu", **kw).fit(X, y)
    assert g.tree_arrays_.equal(h.tree_arrays_, check_impurity=False)
    np.testing.assert_array_equal(g.tree_arrays_.value, h.tree_arrays_.value)
    np.testing.assert_array_equal(g.predict(X), h.predict(X))


def test_gpu_exact_threshold_bins_beyond_16_bits():
    """More than 65,536 unique values in a feature: split value ranks (the exact
    engine's threshold bins) travel as full int32 columns and equal the host's."""
    rng = np.random.default_rng(3)
    n = 120_000
    X = rng.normal(size=(n, 2)).astype(np.float32)
    y = ((X[:, 0] + 0.5 * X[:, 1] + rng.normal(scale=0.7, size=n)) > 0).astype(np.int64)
    g = DecisionTreeClassifier(max_depth=6, device="cuda").fit(X, y)
    h = DecisionTreeClassifier(max_depth=6, device="cpu").fit(X, y)
    assert g.fit_stats_["engine"] == "hip-exact"
    assert int(g.tree_arrays_.threshold_bin.max()) > 65535
    np.testing.assert_array_equal(g.tree_arrays_.threshold_bin, h.tree_arrays_.threshold_bin)
    assert g.tree_arrays_.equal(h.tree_arrays_)


def test_gpu_exact_engine_device_tensors_and_quantile_optin():
    rng = np.random.default_rng(7)
    X = torch.from_numpy(rng.normal(size=(50000, 8)).astype(np.float32)).cuda()
    y = (X[:, 0] + X[:, 1] * X[:, 2] > 0).long()
    g = DecisionTreeClassifier(max_depth=10, device="cuda").fit(X, y)
    assert g.fit_stats_["engine"] == "hip-exact"
    acc = float((g.predict(X) == y).float().mean())
    assert acc > 0.9
    q = DecisionTreeClassifier(max_depth=10, max_bins=256, device="cuda").fit(X, y)
    assert q.fit_stats_["engine"].startswith("hip-") and q.fit_stats_["engine"] != "hip-exact"


def test_gpu_exact_probe_fallback_and_nonfinite(monkeypatch):
    """The exact-threshold probe skips quantile edges and codes when a feature has
    more than 256 values; when the exact engine cannot take the fit (monkeypatched
    here; >= 2^24 rows or >= 2^20 classes for real) the fit bins again and equals
    the explicit 256-quantile-bin fit; a non-finite value still raises."""
    from mpitree_amd.core import fit as fit_mod

    rng = np.random.default_rng(11)
    X = rng.normal(size=(20000, 6)).astype(np.float32)
    X[:, 2] = rng.integers(0, 5, size=20000)
    y = (X[:, 0] + X[:, 1] > 0).astype(np.int64) + (X[:, 2] > 2)
    q = DecisionTreeClassifier(max_depth=8, max_bins=256, device="cuda").fit(X, y)
    monkeypatch.setattr(fit_mod, "_exact_device_ok", lambda *a, **k: False)
    g = DecisionTreeClassifier(max_depth=8, device="cuda").fit(X, y)
    assert g.fit_stats_["engine"] != "hip-exact"
    assert g.tree_arrays_.equal(q.tree_arrays_)
    monkeypatch.undo()
    Xb = X.copy()
    Xb[12345, 4] = np.nan
    with pytest.raises(ValueError, match="NaN or infinity"):
        DecisionTreeClassifier(device="cuda").fit(Xb, y)
    Xb[12345, 4] = np.inf
    with pytest.raises(ValueError, match="NaN or infinity"):
        DecisionTreeClassifier(device="cuda").fit(Xb, y)


@pytest.mark.parametrize("shape", [(2, 1, 2), (7, 3, 3), (150, 4, 3), (241, 1, 241), (600, 5, 40),
                                   (1024, 9, 2), (1000, 2, 300)])
@pytest.mark.parametrize("crit", ["entropy", "gini"])
@pytest.mark.parametrize("md_msl", [(None, 1), (3, 1), (None, 4)])
def test_gpu_small_fit_matches_host(shape, crit, md_msl):
    """<= 1024 rows: the one-workgroup whole-tree kernel (small_fit.hip) builds
    the host builder's tree bit for bit, for any class count."""
    n, F, C = shape
    md, msl = md_msl
    rng = np.random.default_rng(n * 31 + F * 7 + C)
    X = rng.integers(0, max(3, min(n // 3, 250)), size=(n, F)).astype(np.float32)
    y = (X[:, 0].astype(np.int64) * 7 + rng.integers(0, 3, size=n)) % C
    kw = dict(criterion=crit, max_depth=md, min_samples_leaf=msl)
    g = DecisionTreeClassifier(device="cuda", **kw).fit(X, y)
    assert g.fit_stats_["engine"] == "hip-small"
    h = DecisionTreeClassifier(device="cpu", **kw).fit(X, y)
    assert g.tree_arrays_.equal(h.tree_arrays_)
    assert g.export_text(precision=17) == h.export_text(precision=17)
    np.testing.assert_array_equal(g.predict(X), h.predict(X))


def test_gpu_published_sweep_workload():
    """The reference's published benchmark (experiments.ipynb:198-209): one
    feature, n rows, n classes -- on the GPU, equal to the CPU tree."""
    for n in (1, 11, 121, 241):
        X = np.arange(n, dtype=np.float64).reshape(-1, 1)
        y = np.arange(n)
        g = DecisionTreeClassifier(device="cuda").fit(X, y)
        h = DecisionTreeClassifier(device="cpu").fit(X, y)
        assert g.tree_arrays_.equal(h.tree_arrays_), n
        assert g.tree_arrays_.n_leaves == n


@pytest.mark.parametrize("regression", [False, True])
def test_gpu_finisher_handoff_queue_single_job(monkeypatch, regression):
    """The whole tree is ONE finisher job: every other workgroup only works on
    children handed off through the queue (and the watchdog never fires)."""
    from mpitree_amd.core.fit import fit_tree

    monkeypatch.setenv("MPITREE_FINISHER_ROWS", "60000")
    rng = np.random.default_rng(21 + regression)
    n, F = 50000, 12
    X = rng.integers(0, 64, size=(n, F)).astype(np.float32)
    if regression:
        y = X[:, 0] * 0.1 + rng.normal(size=n)
    else:
        y = ((X[:, 0] + X[:, 1] + rng.integers(0, 30, size=n)) // 40) % 2
    kw = dict(regression=regression, criterion=2 if regression else 0, max_depth=None,
              min_samples_split=2)
    g = fit_tree(X, y, device="cuda", **kw)
    assert g.engine == "hip-device-loop" and g.stats.get("finisher_subtrees") == 1
    h = fit_tree(X, y, device="cpu", **kw)
    assert g.arrays.equal(h.arrays, check_impurity=not regression)
    monkeypatch.setenv("MPITREE_FIN_STEAL", "-1")  # same tree without the queue
    g2 = fit_tree(X, y, device="cuda", **kw)
    assert g2.arrays.equal(h.arrays, check_impurity=not regression)


@pytest.mark.parametrize("C,F,n,levels", [(64, 16, 40000, 48), (200, 8, 30000, 48),
                                          (2, 300, 20000, 48), (5, 300, 8000, 48),
                                          (200, 6, 30000, 256), (300, 5, 12000, 256)])
def test_gpu_finisher_many_classes_and_features(C, F, n, levels):
    # the block finisher tiles features through LDS when one node's histogram does
    # not fit (many classes: 16-bit class pairs per bin; many features), keeps the
    # DFS stack's class counts in global scratch past 16 classes, and the sorted
    # tiny kernel runs with fewer waves per workgroup for wide rows. Level
    # histograms past the LDS budget (256 bins x 200 classes) are class-tiled;
    # past 256 classes the finisher jobs hold <= 255 rows -- every shape runs the
    # device level loop
    rng = np.random.default_rng(C * 1000 + F + levels)
    X, y = random_problem(rng, n, F, C, levels=levels)
    cpu = DecisionTreeClassifier(device="cpu").fit(X, y)
    gpu = DecisionTreeClassifier(device="cuda").fit(torch.from_numpy(X).cuda(),
                                                    torch.from_numpy(y).cuda())
    st = gpu.fit_stats_
    assert st.get("finisher_subtrees", 0) > 0, st
    assert st["engine"] == "hip-device-loop", st["engine"]
    assert gpu.tree_arrays_.equal(cpu.tree_arrays_), (gpu.tree_arrays_.node_count,
                                                      cpu.tree_arrays_.node_count)


def test_gpu_exact_engine_matches_reference_source(monkeypatch):
    """The GPU exact-threshold engines against the reference implementation's own
    outputs: continuous problems (every value unique) fitted by the reference
    source on a CPU (tools/make_reference_exact_fixtures.py; the GPU box has no
    reference checkout). ``export_text(precision=17)`` and ``predict`` agree."""
    import json
    import pathlib
    import re

    monkeypatch.setenv("MPITREE_SMALL_FIT", "0")  # (<= 1024 rows: the exact list engine)
    path = pathlib.Path(__file__).parent / "fixtures" / "reference_exact.json"
    canon = lambda t: re.sub(r"-(0\.0+)\]", r"\1]", t)  # noqa: E731
    for p in json.loads(path.read_text()):
        X = np.asarray(p["X"])
        y = np.asarray(p["y"])
        g = DecisionTreeClassifier(max_depth=p["max_depth"], device="cuda").fit(
            torch.from_numpy(X).cuda(), torch.from_numpy(y).cuda())
        assert g.fit_stats_["engine"] == "hip-exact", g.fit_stats_["engine"]
        assert canon(g.export_text(precision=17)) == canon(p["text"])
        np.testing.assert_array_equal(np.asarray(g.predict(X)), np.asarray(p["predict"]))
