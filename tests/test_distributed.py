"""Distributed strategies on CPU ranks (gloo): every rank returns the same
tree, and it is identical to the single-process tree."""

import os

import numpy as np
import pytest

from .dist_utils import run_ranks

FIELDS = ("feature", "threshold_bin", "left", "right", "n_samples", "depth")


def _data(seed=0, n=700, F=7, C=3, regression=False):
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 16, size=(n, F)).astype(np.float64)
    s = X @ rng.normal(size=F) + rng.normal(scale=2.0, size=n)
    if regression:
        return X, np.round(s, 2)
    y = np.digitize(s, np.quantile(s, np.linspace(0, 1, C + 1)[1:-1]))
    return X, y


def _fit_rank(rank, world, strategy, seed, md, regression):
    from mpitree_amd import ParallelDecisionTreeClassifier, ParallelDecisionTreeRegressor

    X, y = _data(seed, regression=regression)
    cls = ParallelDecisionTreeRegressor if regression else ParallelDecisionTreeClassifier
    est = cls(max_depth=md, strategy=strategy, device="cpu").fit(X, y)
    ta = est.tree_arrays_
    out = {k: getattr(ta, k) for k in FIELDS}
    out["value"] = ta.value if regression else ta.count
    out["rank"] = np.array([est.WORLD_RANK, est.WORLD_SIZE])
    out["strategy"] = np.array([est.fit_stats_.get("strategy", "local")])
    return out


def _serial(seed, md, regression):
    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor

    X, y = _data(seed, regression=regression)
    cls = DecisionTreeRegressor if regression else DecisionTreeClassifier
    return cls(max_depth=md, device="cpu").fit(X, y).tree_arrays_


@pytest.mark.parametrize("strategy", ["feature", "data", "subtree", "auto"])
@pytest.mark.parametrize("world", [2, 3])
def test_parallel_equals_serial_classifier(strategy, world):
    md = None if world == 2 else 6
    outs = run_ranks(_fit_rank, world, strategy, 1, md, False)
    ref = _serial(1, md, False)
    for r, o in enumerate(outs):
        assert tuple(o["rank"]) == (r, world)
        for k in FIELDS:
            np.testing.assert_array_equal(o[k], getattr(ref, k), err_msg=f"{k} rank {r}")
        np.testing.assert_array_equal(o["value"], ref.count)


@pytest.mark.parametrize("strategy", ["feature", "data", "subtree"])
def test_parallel_equals_serial_regressor(strategy):
    outs = run_ranks(_fit_rank, 2, strategy, 2, 7, True)
    ref = _serial(2, 7, True)
    for o in outs:
        for k in FIELDS:
            np.testing.assert_array_equal(o[k], getattr(ref, k))
        np.testing.assert_array_equal(o["value"], ref.value)


def test_four_ranks_feature_parallel_deep():
    outs = run_ranks(_fit_rank, 4, "feature", 3, None, False)
    ref = _serial(3, None, False)
    for o in outs:
        for k in FIELDS:
            np.testing.assert_array_equal(o[k], getattr(ref, k))


def test_lpt_assignment_balances_rows():
    from mpitree_amd.parallel.strategies import feature_blocks, lpt_assign

    m = np.array([100, 90, 80, 10, 10, 10, 5])
    owner = lpt_assign(m, 3)
    loads = [m[owner == r].sum() for r in range(3)]
    assert max(loads) - min(loads) <= 30
    assert feature_blocks(64, 8) == [(8 * r, 8 * r + 8) for r in range(8)]
    blocks = feature_blocks(7, 3)
    assert blocks[0][0] == 0 and blocks[-1][1] == 7


def _fit_rank_gpu(rank, world, strategy, seed, md):
    import torch

    from mpitree_amd import ParallelDecisionTreeClassifier

    X, y = _data(seed, n=5000, F=9, C=3)
    Xd = torch.from_numpy(X).cuda()
    yd = torch.from_numpy(y).cuda()
    est = ParallelDecisionTreeClassifier(max_depth=md, strategy=strategy, device="cuda").fit(Xd, yd)
    ta = est.tree_arrays_
    out = {k: getattr(ta, k) for k in FIELDS}
    out["value"] = ta.count
    out["engine"] = np.array([est.fit_stats_["engine"]])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["feature", "data", "subtree", "auto"])
def test_gpu_ranks_equal_serial(strategy, monkeypatch):
    # two ranks sharing one MI355X over gloo: exercises the HIP backend with
    # every strategy's collectives (RCCL itself needs one GPU per rank)
    monkeypatch.setenv("MPITREE_FINISHER_ROWS", "300")
    from mpitree_amd import DecisionTreeClassifier

    outs = run_ranks(_fit_rank_gpu, 2, strategy, 4, None, start_method="spawn")
    X, y = _data(4, n=5000, F=9, C=3)
    ref = DecisionTreeClassifier(device="cpu").fit(X, y).tree_arrays_
    for o in outs:
        # every strategy runs the device level loop (feature / data / replicated
        # levels, split finisher, node exchange)
        assert str(o["engine"][0]) == "hip-device-loop"
        for k in FIELDS:
            np.testing.assert_array_equal(o[k], getattr(ref, k))


def _fit_rank_gpu_large(rank, world, regression, strategy="auto"):
    import torch

    from mpitree_amd import ParallelDecisionTreeClassifier, ParallelDecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    dev = torch.device("cuda", 0)
    # "subtree": the replicated prefix levels forced feature-parallel (the
    # heuristic keeps these small shapes replicated, as "auto" shows)
    os.environ["MPITREE_OWN_FP_PREFIX"] = "1" if strategy == "subtree" else "0"
    if strategy == "subtree":  # /dev/shm "full" on every rank: the node exchange
        os.environ["MPITREE_SHM_MARGIN_MB"] = str(1 << 40)
    if regression:
        X, y = make_regression(200_000, 16, levels=64, seed=5, device=dev)
        cls = ParallelDecisionTreeRegressor
    else:
        X, y = make_classification(300_000, 16, seed=5, device=dev)
        cls = ParallelDecisionTreeClassifier
    outs = {}
    for it in range(2):  # repeated fits: the job split must not depend on append order
        est = cls(strategy=strategy, device="cuda").fit(X, y)
        ta = est.tree_arrays_
        for k in FIELDS + ("threshold", "impurity"):
            outs[f"{k}{it}"] = getattr(ta, k)
        outs[f"stat{it}"] = ta.value if regression else ta.count
        outs[f"engine{it}"] = np.array([est.fit_stats_["engine"]])
        outs[f"mode{it}"] = np.array([est.fit_stats_.get("mode", "")])
        outs[f"bytes{it}"] = np.array(est.fit_stats_.get("comm_bytes_per_level", [0]) or [0])
        outs[f"xbytes{it}"] = np.array([est.fit_stats_.get("comm_bytes_exchange", 0)])
        outs[f"own_rows{it}"] = np.array([est.fit_stats_.get("own_rows", -1)])
        outs[f"asm{it}"] = np.array([est.fit_stats_.get("assembly", "")])
        outs[f"fpx{it}"] = np.array([est.fit_stats_.get("fp_prefix_levels", 0)])
        outs[f"dpr{it}"] = np.array([est.fit_stats_.get("dp_reduce", "")])
        outs[f"dprows{it}"] = np.array([est.fit_stats_.get("dp_rows_exchanged", -1)])
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("regression", [False, True])
@pytest.mark.parametrize("strategy,world", [("auto", 2), ("auto", 4), ("feature", 2),
                                            ("data", 2), ("data", 4), ("subtree", 3)])
def test_gpu_ranks_equal_single_gpu_at_scale(regression, strategy, world):
    """Thousands of finisher jobs (many with equal row counts) over 2-4 ranks:
    subtree ownership (auto / subtree: replicated levels until the LPT switch,
    then each rank grows its own units), feature-parallel and data-parallel
    levels -- every rank, every repeat, equals the single-GPU device-loop tree."""
    import torch

    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    outs = run_ranks(_fit_rank_gpu_large, world, regression, strategy, start_method="spawn")
    want = {"auto": "subtree-owned", "data": "data", "subtree": "subtree-owned",
            "feature": "feature"}[strategy]
    dev = torch.device("cuda", 0)
    if regression:
        X, y = make_regression(200_000, 16, levels=64, seed=5, device=dev)
        ref = DecisionTreeRegressor(device="cuda").fit(X, y).tree_arrays_
    else:
        X, y = make_classification(300_000, 16, seed=5, device=dev)
        ref = DecisionTreeClassifier(device="cuda").fit(X, y).tree_arrays_
    for o in outs:
        for it in range(2):
            assert str(o[f"engine{it}"][0]) == "hip-device-loop"
            assert str(o[f"mode{it}"][0]) == want
            if want == "subtree-owned":
                # "subtree": feature-parallel levels until the switch (one record
                # all-gather each), then none; "auto": no per-level collective.
                # One segment-count exchange at the end.
                nfp = int(o[f"fpx{it}"][0])
                b = o[f"bytes{it}"]
                if strategy == "subtree":
                    assert nfp > 0 and b.size == nfp and (b > 0).all(), (nfp, b)
                else:
                    assert nfp == 0 and b.sum() == 0, (nfp, b)
                assert o[f"xbytes{it}"][0] > 0
                assert o[f"own_rows{it}"][0] > 0  # every rank owns units
                # ranks of one node: each wrote its own nodes into the shared tree
                # (the first fit's tree is still held: the repeat takes another
                # slot); "subtree" runs with /dev/shm too short for any slot
                assert str(o[f"asm{it}"][0]) == ("exchange (/dev/shm short)"
                                                 if strategy == "subtree" else "shared-host")
            else:
                assert o[f"bytes{it}"].sum() > 0  # per-level collectives ran
            if want == "data":
                # one reduce-scatter per level (equal feature blocks), the finisher
                # rows routed to their owners, the owners' nodes in the shared tree
                assert str(o[f"dpr{it}"][0]) == "reduce-scatter"
                assert o[f"dprows{it}"][0] > 0
                assert str(o[f"asm{it}"][0]) == "shared-host"
            for k in FIELDS + ("threshold", "impurity"):
                np.testing.assert_array_equal(o[f"{k}{it}"], getattr(ref, k), err_msg=k)
            np.testing.assert_array_equal(o[f"stat{it}"], ref.value if regression else ref.count)


def _fit_rank_gpu_exact(rank, world, regression):
    import torch

    from mpitree_amd import ParallelDecisionTreeClassifier, ParallelDecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    dev = torch.device("cuda", 0)
    if regression:
        X, y = make_regression(60_000, 10, levels=None, seed=3, device=dev)
        est = ParallelDecisionTreeRegressor(device="cuda").fit(X, y)
    else:
        X, y = make_classification(80_000, 10, levels=None, seed=3, device=dev)
        est = ParallelDecisionTreeClassifier(device="cuda").fit(X, y)
    ta = est.tree_arrays_
    out = {k: getattr(ta, k) for k in FIELDS + ("threshold",)}
    out["value" if regression else "count"] = ta.value if regression else ta.count
    out["engine"] = np.array([est.fit_stats_["engine"]])
    out["mode"] = np.array([est.fit_stats_.get("mode", "")])
    out["block"] = np.array(est.fit_stats_.get("feature_block", [-1, -1]))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("regression", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_exact_feature_parallel_equals_single_gpu(regression, world):
    """Continuous features (every value a threshold) over 2-3 ranks sharing one
    MI355X: the exact engine runs feature-parallel (each rank sorts, scans and
    partitions its feature block; per level one record all-gather and one flag
    all-reduce) and every rank builds the single-GPU tree bit for bit."""
    import torch

    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    outs = run_ranks(_fit_rank_gpu_exact, world, regression, start_method="spawn")
    dev = torch.device("cuda", 0)
    if regression:
        X, y = make_regression(60_000, 10, levels=None, seed=3, device=dev)
        ref = DecisionTreeRegressor(device="cuda").fit(X, y)
    else:
        X, y = make_classification(80_000, 10, levels=None, seed=3, device=dev)
        ref = DecisionTreeClassifier(device="cuda").fit(X, y)
    assert ref.fit_stats_["engine"] == "hip-exact"
    blocks = sorted(tuple(o["block"]) for o in outs)
    assert blocks[0][0] == 0 and blocks[-1][1] == 10  # the ranks cover every feature
    for o in outs:
        assert str(o["engine"][0]) == "hip-exact" and str(o["mode"][0]) == "feature"
        for k in FIELDS + ("threshold",):
            np.testing.assert_array_equal(o[k], getattr(ref.tree_arrays_, k), err_msg=k)
        key = "value" if regression else "count"
        np.testing.assert_array_equal(o[key], getattr(ref.tree_arrays_, key))


def _fit_rank_rccl(rank, world, strategy, regression, continuous=False):
    import torch
    import torch.distributed as dist

    from mpitree_amd.parallel.process_group import rank_topology

    assert dist.get_backend() == "nccl"
    dev = torch.device("cuda", rank)
    # "subtree": the replicated prefix levels forced feature-parallel (the record
    # all-gather + combine of every prefix level runs over RCCL)
    os.environ["MPITREE_OWN_FP_PREFIX"] = "1" if strategy == "subtree" else "0"
    X, y, cls = _rccl_data(regression, continuous, dev)
    est = cls(strategy=strategy, device="cuda")
    for _ in range(2):  # (the second fit reuses workspaces, pools and the watchdog)
        est.fit(X, y)
    ta = est.tree_arrays_
    outs = {k: getattr(ta, k) for k in FIELDS + ("threshold",)}
    outs["stat"] = ta.value if regression else ta.count
    outs["mode"] = np.array([est.fit_stats_.get("mode", "")])
    outs["engine"] = np.array([est.fit_stats_.get("engine", "")])
    topo = rank_topology()
    outs["world_seen"] = np.array([topo["world_size_seen"]])
    outs["gpus"] = np.array([topo["distinct_gpus"]])
    outs["device"] = np.array([torch.cuda.current_device()])
    return outs


def _rccl_data(regression, continuous, dev):
    from mpitree_amd import ParallelDecisionTreeClassifier, ParallelDecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    if regression:
        X, y = make_regression(200_000, 16, levels=None if continuous else 64, seed=5,
                               device=dev)
        return X, y, ParallelDecisionTreeRegressor
    X, y = make_classification(100_000 if continuous else 300_000, 16,
                               levels=None if continuous else 256, seed=5, device=dev)
    return X, y, ParallelDecisionTreeClassifier


def _gpus() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


_RCCL_WORLDS = sorted({2, max(2, min(8, _gpus()))})
_RCCL_CASES = [
    # (strategy, regression, continuous, expected mode)
    ("auto", False, False, "subtree-owned"),
    ("subtree", False, False, "subtree-owned"),
    ("feature", False, False, "feature"),
    ("data", False, False, "data"),
    ("auto", True, False, "subtree-owned"),
    ("data", True, False, "data"),
    ("auto", False, True, "feature"),  # exact engine, feature-parallel lists
    ("auto", True, True, "feature"),
]


@pytest.mark.gpu
@pytest.mark.skipif(_gpus() < 2, reason="RCCL needs one GPU per rank (>= 2 visible)")
@pytest.mark.parametrize("world", _RCCL_WORLDS)
@pytest.mark.parametrize("strategy,regression,continuous,want", _RCCL_CASES)
def test_rccl_ranks_equal_single_gpu(world, strategy, regression, continuous, want):
    """Real RCCL (nccl backend, device_id init, on-stream collectives over xGMI):
    2 and min(8, visible) ranks on as many GPUs build the single-GPU tree bit for
    bit -- subtree ownership (with and without the feature-parallel prefix),
    feature-parallel, data-parallel (async reduce-to-owner, device all_to_all),
    and the exact engine's feature-parallel lists (codes all_to_all, flag
    all-reduce). Every rank reports the world the group saw and a distinct GPU."""
    import torch

    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor

    if world > _gpus():
        pytest.skip(f"{world} ranks need {world} GPUs")
    outs = run_ranks(_fit_rank_rccl, world, strategy, regression, continuous,
                     start_method="spawn", backend="nccl")
    dev = torch.device("cuda", 0)
    X, y, _ = _rccl_data(regression, continuous, dev)
    cls = DecisionTreeRegressor if regression else DecisionTreeClassifier
    ref = cls(device="cuda").fit(X, y).tree_arrays_
    assert sorted(int(o["device"][0]) for o in outs) == list(range(world))
    for o in outs:
        assert int(o["world_seen"][0]) == world and int(o["gpus"][0]) == world
        assert str(o["mode"][0]) == want, (str(o["mode"][0]), str(o["engine"][0]))
        for k in FIELDS + ("threshold",):
            np.testing.assert_array_equal(o[k], getattr(ref, k), err_msg=k)
        np.testing.assert_array_equal(o["stat"], ref.value if regression else ref.count)


@pytest.mark.gpu
@pytest.mark.skipif(_gpus() < 2, reason="RCCL needs one GPU per rank (>= 2 visible)")
@pytest.mark.parametrize("where", ["level:2", "exchange"])
def test_rccl_fault_raises_everywhere(where):
    """nccl fault injection: rank 1 raises inside the level loop or after the
    ownership switch; every rank raises within 30 s (the failing rank's
    communicator abort, or the peer's watchdog aborting its own RCCL
    communicator -- parallel/failure.py) instead of hanging in a collective."""
    outs = run_ranks(_fault_mid_loop_gpu, 2, "auto", where, False, start_method="spawn",
                     backend="nccl")
    kinds = [str(o["kind"][0]) for o in outs]
    assert kinds[1] == "injected" and kinds[0] != "ok", kinds
    assert max(float(o["s"][0]) for o in outs) < 30


def _fault_rank(rank, world, fault_rank):
    import os

    from mpitree_amd import ParallelDecisionTreeClassifier
    from mpitree_amd.utils.observability import InjectedFault

    os.environ["MPITREE_FAULT_RANK"] = str(fault_rank)
    X, y = _data(3)
    kind = "ok"
    try:
        ParallelDecisionTreeClassifier(max_depth=4, strategy="feature", device="cpu").fit(X, y)
    except InjectedFault:
        kind = "injected"
    except RuntimeError as e:
        kind = "peer" if "another rank" in str(e) else f"other:{e}"
    # the group is still usable afterwards: a clean fit succeeds on every rank
    os.environ.pop("MPITREE_FAULT_RANK")
    est = ParallelDecisionTreeClassifier(max_depth=4, strategy="feature", device="cpu").fit(X, y)
    return {"kind": np.array([kind]), "nodes": np.array([est.tree_arrays_.node_count])}


@pytest.mark.parametrize("fault_rank", [0, 1])
def test_fault_on_one_rank_raises_everywhere(fault_rank):
    outs = run_ranks(_fault_rank, 2, fault_rank)
    kinds = [str(o["kind"][0]) for o in outs]
    assert kinds[fault_rank] == "injected"
    assert kinds[1 - fault_rank] == "peer"
    assert outs[0]["nodes"][0] == outs[1]["nodes"][0] > 1


def _fault_mid_loop(rank, world, strategy):
    import os
    import time

    from mpitree_amd import ParallelDecisionTreeClassifier
    from mpitree_amd.parallel.failure import CollectiveFitAborted
    from mpitree_amd.utils.observability import InjectedFault

    os.environ.update(MPITREE_FAULT_RANK="1", MPITREE_FAULT_AT="level:2", MPITREE_FAIL_WAIT="2")
    X, y = _data(3, n=3000)
    kind, t0 = "ok", time.monotonic()
    try:
        ParallelDecisionTreeClassifier(strategy=strategy, device="cpu").fit(X, y)
    except InjectedFault:
        kind = "injected"
    except CollectiveFitAborted as e:
        kind = "peer" if "rank 1" in str(e) and "InjectedFault" in str(e) else f"other:{e}"
    except Exception as e:  # noqa: BLE001
        kind = f"other:{type(e).__name__}:{e}"
    return {"kind": np.array([kind]), "s": np.array([time.monotonic() - t0])}


@pytest.mark.parametrize("strategy", ["feature", "data", "subtree"])
def test_fault_inside_level_loop_raises_everywhere(strategy):
    """A rank that fails inside the level loop (peers blocked in that level's
    collective, or still growing) makes every rank raise within seconds -- not
    after the process-group timeout (parallel/failure.py)."""
    outs = run_ranks(_fault_mid_loop, 2, strategy)
    kinds = [str(o["kind"][0]) for o in outs]
    assert kinds == ["peer", "injected"], kinds
    assert max(float(o["s"][0]) for o in outs) < 30


def _digest_rank(rank, world):
    from mpitree_amd.parallel.strategies import FeatureParallelComm

    comm = FeatureParallelComm()
    same = comm.check_consistent(12345)
    differ = comm.check_consistent(1000 + rank)
    return {"r": np.array([same, differ])}


def test_cross_rank_digest_check():
    outs = run_ranks(_digest_rank, 2)
    for o in outs:
        assert list(o["r"]) == [True, False]


def _sharded_data(seed, regression):
    """Shards with different value and label sets: rank 0 sees feature values
    0..7 and labels {0, 1}; rank 1 sees 4..15 and labels {1, 2, 5}."""
    rng = np.random.default_rng(seed)
    n = 400
    X0 = rng.integers(0, 8, size=(n, 4)).astype(np.float64)
    X1 = rng.integers(4, 16, size=(n, 4)).astype(np.float64) + 0.5
    s0, s1 = X0 @ [1, -1, 0.5, 0], X1 @ [1, -1, 0.5, 0]
    if regression:
        return [X0, X1], [s0 * 0.25, s1 * 3.0]
    y0 = (s0 > 2).astype(np.int64)
    y1 = np.choose(np.digitize(s1, [0, 5]), [1, 2, 5])
    return [X0, X1], [y0, y1]


def _fit_sharded(rank, world, regression):
    from mpitree_amd import ParallelDecisionTreeClassifier, ParallelDecisionTreeRegressor
    from mpitree_amd.utils.observability import tree_digest

    Xs, ys = _sharded_data(5, regression)
    cls = ParallelDecisionTreeRegressor if regression else ParallelDecisionTreeClassifier
    est = cls(strategy="data", device="cpu").fit(Xs[rank], ys[rank], data_sharded=True)
    ta = est.tree_arrays_
    out = {k: getattr(ta, k) for k in FIELDS}
    out["threshold"] = ta.threshold
    out["value"] = ta.value if regression else ta.count
    out["digest"] = np.array([tree_digest(ta)])
    if not regression:
        out["classes"] = est.classes_
    return out


@pytest.mark.parametrize("regression", [False, True])
def test_data_sharded_agrees_with_concatenated_fit(regression):
    """shards must agree on bin edges, classes and the fixed-point
    scale; the tree equals the single-process fit of the concatenated data."""
    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor

    outs = run_ranks(_fit_sharded, 2, regression)
    Xs, ys = _sharded_data(5, regression)
    X, y = np.concatenate(Xs), np.concatenate(ys)
    cls = DecisionTreeRegressor if regression else DecisionTreeClassifier
    ref = cls(device="cpu").fit(X, y)
    ta = ref.tree_arrays_
    for o in outs:
        assert o["digest"][0] == outs[0]["digest"][0]
        for k in FIELDS:
            np.testing.assert_array_equal(o[k], getattr(ta, k), err_msg=k)
        np.testing.assert_array_equal(o["threshold"], ta.threshold)
        if regression:
            np.testing.assert_allclose(o["value"], ta.value, rtol=1e-12)
        else:
            np.testing.assert_array_equal(o["classes"], ref.classes_)
            np.testing.assert_array_equal(o["value"], ta.count)


def _fit_sharded_gpu(rank, world, regression):
    """The row-shard fit on GPU ranks (ranks sharing one card over gloo): the
    agreed bin mapper is applied on the device (gpu_prepare.prepare_with_mapper)."""
    from mpitree_amd import ParallelDecisionTreeClassifier, ParallelDecisionTreeRegressor
    from mpitree_amd.utils.observability import tree_digest

    Xs, ys = _sharded_data(5, regression)
    cls = ParallelDecisionTreeRegressor if regression else ParallelDecisionTreeClassifier
    est = cls(strategy="data", device="cuda").fit(Xs[rank], ys[rank], data_sharded=True)
    ta = est.tree_arrays_
    out = {k: getattr(ta, k) for k in FIELDS}
    out["threshold"] = ta.threshold
    out["value"] = ta.value if regression else ta.count
    out["digest"] = np.array([tree_digest(ta)])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("regression", [False, True])
def test_gpu_data_sharded_agrees_with_concatenated_fit(regression):
    """Row shards on GPU ranks build the single-process tree of the concatenated
    data (agreed edges, classes and fixed-point scale; device binning of each
    shard with the agreed table)."""
    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor

    outs = run_ranks(_fit_sharded_gpu, 2, regression, start_method="spawn")
    Xs, ys = _sharded_data(5, regression)
    X, y = np.concatenate(Xs), np.concatenate(ys)
    cls = DecisionTreeRegressor if regression else DecisionTreeClassifier
    ta = cls(device="cpu").fit(X, y).tree_arrays_
    for o in outs:
        assert o["digest"][0] == outs[0]["digest"][0]
        for k in FIELDS:
            np.testing.assert_array_equal(o[k], getattr(ta, k), err_msg=k)
        np.testing.assert_array_equal(o["threshold"], ta.threshold)
        if regression:
            np.testing.assert_allclose(o["value"], ta.value, rtol=1e-12)
        else:
            np.testing.assert_array_equal(o["value"], ta.count)


def _fit_sharded_continuous(rank, world, max_bins):
    from mpitree_amd import ParallelDecisionTreeClassifier
    from mpitree_amd.utils.observability import tree_digest

    rng = np.random.default_rng(40 + rank)  # every shard its own continuous rows
    X = rng.normal(size=(3000, 5)) * (1 + rank)
    y = (X[:, 0] + X[:, 1] ** 2 > 1).astype(np.int64)
    est = ParallelDecisionTreeClassifier(strategy="data", device="cpu", max_bins=max_bins)
    try:
        est.fit(X, y, data_sharded=True)
    except ValueError as e:
        return {"error": np.array([str(e)])}
    ta = est.tree_arrays_
    return {"digest": np.array([tree_digest(ta)]), "nodes": np.array([ta.node_count]),
            "acc": np.array([est.score(X, y)]), "thr": ta.threshold}


def test_data_sharded_continuous_quantile_summary():
    """Continuous row shards with max_bins: the per-rank summaries merge into one
    agreed quantile table (no gather of every unique value); every rank grows
    the same tree and its thresholds are data values of some shard."""
    outs = run_ranks(_fit_sharded_continuous, 2, 64)
    assert "error" not in outs[0], outs[0].get("error")
    assert outs[0]["digest"][0] == outs[1]["digest"][0]
    assert outs[0]["nodes"][0] > 10 and min(o["acc"][0] for o in outs) > 0.9
    vals = np.concatenate([np.random.default_rng(40 + r).normal(size=(3000, 5)) * (1 + r)
                           for r in range(2)]).ravel()
    thr = outs[0]["thr"]
    assert np.isin(thr[~np.isnan(thr)], vals).all()


def test_data_sharded_exact_continuous_raises():
    """max_bins=None (exact) with > 256 distinct values in a sharded feature:
    an explicit error naming the limit and the options, on every rank."""
    outs = run_ranks(_fit_sharded_continuous, 2, None)
    for o in outs:
        msg = str(o["error"][0])
        assert "256 distinct values" in msg and "max_bins" in msg


def test_tree_digest_covers_thresholds():
    from mpitree_amd import DecisionTreeClassifier
    from mpitree_amd.utils.observability import tree_digest

    X = np.array([[0.0], [1.0], [2.0], [3.0]])
    y = np.array([0, 0, 1, 1])
    a = DecisionTreeClassifier(device="cpu").fit(X, y).tree_arrays_
    b = DecisionTreeClassifier(device="cpu").fit(X * 10, y).tree_arrays_
    assert tree_digest(a) != tree_digest(b)  # same structure, different thresholds


def _counted_rows(rank, world):
    import torch

    from mpitree_amd.parallel.strategies import SubtreeComm

    comm = SubtreeComm()
    # rank r packed 3 + 4 r rows into a buffer of 8 rows (rank 1's 7 rows fit, a
    # later rank would exceed rank 0's buffer: the exchange pads a copy)
    k = 3 + 4 * rank
    buf = torch.full((max(k, 8), 5), -1, dtype=torch.int32)
    buf[:k] = torch.arange(k * 5, dtype=torch.int32).reshape(k, 5) + 1000 * rank
    out = comm.all_gather_rows_counted(buf, torch.tensor([k], dtype=torch.int64))
    return {"rows": out.numpy()}


def test_all_gather_rows_counted_pads_and_concatenates():
    """The one-wait row exchange (device-side counts) equals the concatenation of
    every rank's first k rows, also when a peer has more rows than this buffer."""
    outs = run_ranks(_counted_rows, 3)
    want = np.concatenate([np.arange((3 + 4 * r) * 5).reshape(-1, 5) + 1000 * r
                           for r in range(3)])
    for o in outs:
        np.testing.assert_array_equal(o["rows"], want)


def _counted_rows_overflow(rank, world):
    import torch

    from mpitree_amd.parallel.strategies import SubtreeComm

    comm = SubtreeComm()
    # rank 1 reports 9 packed rows for a 4-row buffer: every rank must raise at
    # the count exchange (no rank goes on into the row all-gather)
    k = 9 if rank == 1 else 2
    buf = torch.zeros((4, 3), dtype=torch.int32)
    try:
        comm.all_gather_rows_counted(buf, torch.tensor([k], dtype=torch.int64))
    except RuntimeError as e:
        return {"err": str(e)}
    return {"err": None}


def test_all_gather_rows_counted_overflow_raises_on_every_rank():
    outs = run_ranks(_counted_rows_overflow, 3)
    for o in outs:
        assert "rank 1 packed 9 rows" in str(o["err"])


def _fault_mid_loop_gpu(rank, world, strategy, where, continuous):
    import os
    import time

    import torch

    from mpitree_amd import ParallelDecisionTreeClassifier
    from mpitree_amd.parallel.failure import CollectiveFitAborted
    from mpitree_amd.utils.datasets import make_classification
    from mpitree_amd.utils.observability import InjectedFault

    dev = torch.device("cuda", torch.cuda.current_device())  # (nccl: one GPU per rank)
    X, y = make_classification(200_000, 16, levels=None if continuous else 256, seed=7,
                               device=dev)
    os.environ.update(MPITREE_FAULT_RANK="1", MPITREE_FAULT_AT=where, MPITREE_FAIL_WAIT="2")
    kind, t0 = "ok", time.monotonic()
    mode = ""
    try:
        est = ParallelDecisionTreeClassifier(strategy=strategy, device="cuda")
        est.fit(X, y)
        mode = est.fit_stats_.get("mode", "")
    except InjectedFault:
        kind = "injected"
    except CollectiveFitAborted as e:
        kind = "peer" if "rank 1" in str(e) and "InjectedFault" in str(e) else f"other:{e}"
    except Exception as e:  # noqa: BLE001
        kind = f"other:{type(e).__name__}:{e}"
    torch.cuda.synchronize()
    return {"kind": np.array([kind]), "s": np.array([time.monotonic() - t0]),
            "mode": np.array([mode])}


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,where,continuous", [
    ("auto", "level:2", False),     # replicated levels (before the ownership switch)
    ("auto", "exchange", False),    # after the switch: the peer waits in the node exchange
    ("feature", "level:2", False),  # the peer waits in that level's record all-gather
    ("auto", "level:2", True),      # exact engine, feature-parallel levels
    ("auto", "exchange", True),     # exact engine: the peer waits in the finisher exchange
])
def test_gpu_fault_inside_fit_raises_everywhere(strategy, where, continuous):
    """Two gloo ranks sharing one MI355X, rank 1 raising inside the device level
    loop, after the ownership switch, or inside the exact engine: every rank
    raises (the injected error, or CollectiveFitAborted naming rank 1) within
    30 s instead of blocking in a collective (parallel/failure.py)."""
    outs = run_ranks(_fault_mid_loop_gpu, 2, strategy, where, continuous, start_method="spawn")
    kinds = [str(o["kind"][0]) for o in outs]
    assert kinds == ["peer", "injected"], kinds
    assert max(float(o["s"][0]) for o in outs) < 30


def _topology_rank(rank, world, agreed):
    from mpitree_amd.ops.device_grower import agreed_free_bytes
    from mpitree_amd.parallel.process_group import rank_topology
    from mpitree_amd.parallel.strategies import FeatureParallelComm

    topo = rank_topology()
    out = {"backend": np.array([topo["dist_backend"]]),
           "world": np.array([topo["world_size_seen"]]),
           "ranks": np.array([r["rank"] for r in topo["ranks"]]),
           "gpus": np.array([topo["distinct_gpus"]])}
    if agreed:
        # ranks reading different free memory decide from the minimum
        os.environ["MPITREE_FREE_BYTES"] = str((rank + 1) * 1000)
        out["free"] = np.array([agreed_free_bytes(FeatureParallelComm(), None)])
    return out


def test_rank_topology_and_agreed_free_bytes():
    """The bench JSON's process-group fields (backend, world size the group saw,
    every rank's device) over gloo, and the engine choice's free-memory reading
    agreed as the minimum over the ranks."""
    outs = run_ranks(_topology_rank, 3, True)
    for o in outs:
        assert str(o["backend"][0]) == "gloo" and int(o["world"][0]) == 3
        assert list(o["ranks"]) == [0, 1, 2]
        assert int(o["free"][0]) == 1000
