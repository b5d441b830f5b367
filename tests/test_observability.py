"""Profiling / logging hooks (CPU)."""

import logging

import numpy as np


def test_fit_logs_summary(caplog):
    from mpitree_amd import DecisionTreeClassifier

    rng = np.random.default_rng(1)
    X = rng.integers(0, 5, size=(200, 3))
    y = rng.integers(0, 2, size=200)
    with caplog.at_level(logging.DEBUG, logger="mpitree"):
        DecisionTreeClassifier(device="cpu").fit(X, y)
    msgs = [r.getMessage() for r in caplog.records if r.name == "mpitree"]
    assert any(m.startswith("fit: engine=") for m in msgs)
    assert any(m.startswith("fit timings") for m in msgs)


def test_profile_flag_and_roctx_noop(monkeypatch):
    from mpitree_amd.utils.observability import profiling, roctx_range

    monkeypatch.delenv("MPITREE_PROFILE", raising=False)
    assert not profiling()
    with roctx_range("x"):
        pass
    monkeypatch.setenv("MPITREE_PROFILE", "1")
    assert profiling()
    with roctx_range("x"):  # no GPU runtime here: must still be harmless
        pass


def test_fit_stats_exposed():
    from mpitree_amd import DecisionTreeClassifier

    rng = np.random.default_rng(2)
    X = rng.integers(0, 7, size=(300, 4))
    y = rng.integers(0, 3, size=300)
    est = DecisionTreeClassifier(device="cpu").fit(X, y)
    st = est.fit_stats_
    assert st["node_count"] == est.tree_arrays_.node_count
    assert "total" in st["timings"] and st["engine"]
