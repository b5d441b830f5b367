"""TreeArrays built from the device assembly's compact columns: the deferred
columns (left children, node sizes, int64 counts, impurities, leaf values)
equal what the host builders compute, bit for bit, and survive pickling."""
import pickle

import numpy as np
import pytest

from mpitree_amd.core.fit import fit_tree
from mpitree_amd.models.tree_arrays import TreeArrays


def _compact(ta, regression):
    if regression:
        stats = np.stack([ta.n_samples, ta.meta["sum_fixed"]], 1).astype(np.int64)
    else:
        stats = ta.count.astype(np.int32)
    f, b = ta.feature.astype(np.int64), ta.threshold_bin.astype(np.int64)
    split = np.where(f >= 0, (f << 16) | b, -1).astype(np.int32)  # assemble.hip's packing
    return dict(stats=stats, threshold=ta.threshold.copy(), split=split,
                right=ta.right.astype(np.int32), max_depth=int(ta.depth.max()))


@pytest.mark.parametrize("crit", [0, 1, 2])
def test_device_columns_derive_host_columns(crit):
    rng = np.random.default_rng(crit)
    X = rng.integers(0, 30, size=(3000, 5)).astype(np.float64)
    reg = crit == 2
    if reg:
        y = X[:, 0] * 0.3 + rng.normal(size=3000)
    else:
        y = ((X[:, 0] + X[:, 1] + rng.integers(0, 9, 3000)) % 3).astype(np.int64)
    r = fit_tree(X, y, regression=reg, criterion=crit, max_depth=None, min_samples_split=2,
                 device="cpu")
    host = r.arrays
    dev = TreeArrays.from_device_columns(**_compact(host, reg), criterion=crit, regression=reg,
                                         y_exp=r.y_scale_exp)
    assert "left" not in dev.__dict__  # still deferred
    assert dev.max_depth == host.max_depth and "depth" not in dev.__dict__
    assert dev.equal(host)
    assert np.array_equal(dev.depth, host.depth)  # derived from the right links
    assert dev.left.dtype == np.int32 and dev.n_samples.dtype == np.int64
    if reg:
        assert np.array_equal(dev.value, host.value)
        assert dev.count is None
    else:
        assert dev.count.dtype == np.int64 and dev.value is None
    back = pickle.loads(pickle.dumps(dev))
    assert back.equal(host) and "_derive" not in back.__dict__


def test_deferred_missing_attribute_raises():
    ta = TreeArrays.deferred({}, feature=np.zeros(1, np.int32))
    with pytest.raises(AttributeError):
        _ = ta.nonexistent


def test_device_columns_thresholds_from_edge_table():
    from mpitree_amd.core.binning import fit_bin_mapper

    rng = np.random.default_rng(9)
    X = rng.integers(0, 40, size=(2000, 4)).astype(np.float64)
    y = (X[:, 0] + rng.integers(0, 5, 2000)) % 2
    r = fit_tree(X, y, regression=False, criterion=0, max_depth=None, min_samples_split=2,
                 device="cpu")
    table = fit_bin_mapper(X, 256).padded_edges()
    cols = _compact(r.arrays, False)
    cols["threshold"] = None
    dev = TreeArrays.from_device_columns(**cols, criterion=0, regression=False,
                                         edges_table=table)
    assert "threshold" not in dev.__dict__
    assert dev.equal(r.arrays)
    from mpitree_amd.utils.observability import tree_digest

    assert tree_digest(dev) == tree_digest(dev)  # stable; hashes the edge table, not thresholds
