"""Every host builder grows the oracle's tree exactly (exact-bin mode)."""

import numpy as np
import pytest

from mpitree_amd.core.backend_numpy import NumpyBackend
from mpitree_amd.core.binning import fit_bin_mapper
from mpitree_amd.core.criterion import Criterion
from mpitree_amd.core.levelwise import GrowParams, LevelwiseBuilder
from mpitree_amd.core.reference import fit_reference
from mpitree_amd.ops import native

CRITS = [Criterion.ENTROPY, Criterion.GINI]


def _problem(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    F = int(rng.integers(1, 6))
    C = int(rng.integers(1, 5))
    X = rng.integers(0, int(rng.integers(1, 30)), size=(n, F)).astype(np.float64)
    y = rng.integers(0, C, size=n)
    return rng, X, y, C


@pytest.mark.parametrize("seed", range(30))
def test_levelwise_numpy_matches_oracle(seed):
    rng, X, y, C = _problem(seed)
    crit = CRITS[seed % 2]
    md = [None, 2, 5][seed % 3]
    msl = 1 + seed % 3
    mss = 2 + seed % 4
    fr = [0, 7, 60][seed % 3]
    mapper = fit_bin_mapper(X)
    codes = mapper.transform(X)
    ref = fit_reference(codes, y, n_classes=C, n_bins=mapper.max_n_bins, criterion=crit,
                        max_depth=md, min_samples_split=mss, min_samples_leaf=msl)
    be = NumpyBackend()
    be.setup(codes, y, n_bins=mapper.max_n_bins, n_classes=C, criterion=crit)
    p = GrowParams(criterion=crit, max_depth=md, min_samples_split=mss, min_samples_leaf=msl,
                   finisher_rows=fr)
    ta = LevelwiseBuilder(be, p).fit(len(y), C, X.shape[1])
    assert ta.equal(ref)


@pytest.mark.skipif(not native.has_cpu(), reason="native module not built")
@pytest.mark.parametrize("seed", range(30))
def test_native_matches_oracle(seed):
    from mpitree_amd.ops.cpu_builder import fit_native

    rng, X, y, C = _problem(100 + seed)
    crit = CRITS[seed % 2]
    md = [None, 3, 6][seed % 3]
    msl = 1 + seed % 2
    mapper = fit_bin_mapper(X)
    codes = mapper.transform(X)
    ref = fit_reference(codes, y, n_classes=C, n_bins=mapper.max_n_bins, criterion=crit,
                        max_depth=md, min_samples_leaf=msl)
    ta = fit_native(codes, y, mapper, C, GrowParams(criterion=crit, max_depth=md,
                                                    min_samples_leaf=msl), n_threads=1 + seed % 3)
    assert ta.equal(ref)


@pytest.mark.parametrize("seed", range(12))
def test_regression_builders_match_oracle(seed):
    rng = np.random.default_rng(200 + seed)
    n = int(rng.integers(2, 300))
    F = int(rng.integers(1, 5))
    X = rng.integers(0, 12, size=(n, F)).astype(np.float64)
    yf = rng.integers(-50, 50, size=n).astype(np.int64)
    md = [None, 4][seed % 2]
    mapper = fit_bin_mapper(X)
    codes = mapper.transform(X)
    ref = fit_reference(codes, yf, n_classes=0, n_bins=mapper.max_n_bins,
                        criterion=Criterion.SQUARED_ERROR, max_depth=md)
    be = NumpyBackend()
    be.setup(codes, yf, n_bins=mapper.max_n_bins, n_classes=0, criterion=Criterion.SQUARED_ERROR)
    ta = LevelwiseBuilder(be, GrowParams(criterion=Criterion.SQUARED_ERROR, max_depth=md,
                                         finisher_rows=[0, 20][seed % 2])).fit(n, 0, F)
    assert ta.equal(ref)
    assert np.array_equal(ta.meta["sum_fixed"], ref.meta["sum_fixed"])
    if native.has_cpu():
        from mpitree_amd.ops.cpu_builder import fit_native

        tn = fit_native(codes, yf, mapper, 0, GrowParams(criterion=Criterion.SQUARED_ERROR,
                                                         max_depth=md))
        assert tn.equal(ref)
        assert np.array_equal(tn.meta["sum_fixed"], ref.meta["sum_fixed"])


def test_quantile_binning_edges_are_data_values():
    rng = np.random.default_rng(5)
    X = rng.normal(size=(5000, 3))
    m = fit_bin_mapper(X, max_bins=32)
    codes = m.transform(X)
    for f in range(3):
        e = m.edges[f]
        assert len(e) <= 32 and not m.exact[f]
        assert np.isin(e, X[:, f]).all()
        # x <= edges[b]  <=>  code <= b
        for b in (0, 5, len(e) - 2):
            np.testing.assert_array_equal(X[:, f] <= e[b], codes[:, f] <= b)


def test_exact_binning_when_few_uniques():
    X = np.array([[1.5, 3], [2.5, 3], [1.5, 4]], dtype=np.float64)
    m = fit_bin_mapper(X)
    assert m.exact.all()
    np.testing.assert_array_equal(m.edges[0], [1.5, 2.5])
    np.testing.assert_array_equal(m.transform(X), [[0, 0], [1, 0], [0, 1]])
