"""The exact (presorted-list) engine's workspace estimate and the quantile
fallback decision, checked at large shapes without allocating."""

import pytest

GB = 1 << 30


@pytest.fixture(scope="module")
def xe():
    from mpitree_amd.ops import native

    if not native.has_hip():
        pytest.skip("HIP extension not built")
    from mpitree_amd.ops import exact_grower

    return exact_grower


def test_many_classes_without_finisher_fall_back(xe):
    # thousands of classes: the finisher's per-node class arrays exceed LDS, so
    # no local-code finisher -- levels grow to the leaves and the (items x
    # features x classes) chunk totals would need terabytes
    assert xe.exact_finisher_rows(64, 5000, False) == 0
    need = xe.exact_workspace_bytes(1_000_000, 64, 5000, False, 0, 2048, 5007)
    assert need > 1000 * GB
    assert not xe.exact_fits_memory(1_000_000, 64, 5000, False, free_bytes=288 * GB)


def test_past_256_classes_list_engine_grows_to_the_leaves(xe):
    # 300 classes on continuous data: no local-code finisher, the list engine's
    # levels grow every node (the estimate sizes the level buffers for that)
    assert xe.exact_finisher_rows(64, 300, False) == 0
    assert xe.exact_finisher_rows(64, 256, False) > 0


def test_flagship_shapes_fit(xe):
    assert xe.exact_finisher_rows(64, 2, False) > 0
    assert xe.exact_fits_memory(1_000_000, 64, 2, False, free_bytes=288 * GB)
    assert xe.exact_fits_memory(1_000_000, 64, 0, True, free_bytes=288 * GB)
    # the tests' small many-class shapes still take the list engine
    assert xe.exact_fits_memory(6000, 64, 300, False, free_bytes=288 * GB)


def test_feature_parallel_ranks_divide_the_estimate(xe):
    one = xe.exact_workspace_bytes(1_000_000, 64, 2, False, 256, 2048, 9)
    eight = xe.exact_workspace_bytes(1_000_000, 8, 2, False, 256, 2048, 9)
    assert eight < one / 4


def test_fit_dispatch_uses_the_estimate(xe, monkeypatch):
    from mpitree_amd.core import fit

    assert not fit._exact_device_ok(1_000_000, 64, 5000, False, free_bytes=288 * GB)
    assert fit._exact_device_ok(1_000_000, 64, 2, False, free_bytes=288 * GB)
    assert not fit._exact_device_ok(1 << 24, 64, 2, False, free_bytes=288 * GB)  # row limit
