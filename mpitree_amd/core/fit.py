"""Fit dispatch: input validation, label encoding, binning and engine choice.

One entry point, :func:`fit_tree`, used by every estimator. It owns the
parts of the reference's ``fit`` (``mpitree/tree/decision_tree.py:168-190``)
that are not tree growth: ``check_X_y``-style validation (finite 2-D
features), class discovery (``classes_ = np.unique(y)``) -- labels are encoded
to ``0..K-1`` internally so non-contiguous labels work -- and it picks the
engine:

* ``device="cuda"`` (or ``"auto"`` with a GPU and a device tensor or a large
  input): binning and growth on the current MI355X through the HIP kernels;
* ``device="cpu"``: the native C++ builder when built, else the numpy
  level-wise engine.

Distributed fits pass a communication strategy (``comm``) and use the same
level-wise engine on either device.
"""

from __future__ import annotations

import logging
import math
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .binning import BinMapper, fit_bin_mapper
from .criterion import Criterion
from .levelwise import GrowParams, LevelwiseBuilder, LocalComm
from ..models.tree_arrays import TreeArrays
from ..ops import native
from ..utils.debug import check_device_inputs, debug_enabled, validate_tree
from ..utils.observability import logger, profiling, roctx_range

__all__ = ["FitResult", "fit_tree", "resolve_device", "AUTO_GPU_MIN_CELLS"]

AUTO_GPU_MIN_CELLS = 1 << 18  # n*F below this stays on the host in device="auto"


@dataclass
class FitResult:
    arrays: TreeArrays
    classes: np.ndarray | None
    n_features: int
    mapper: BinMapper
    y_scale_exp: int = 0
    engine: str = ""
    timings: dict = field(default_factory=dict)
    stats: dict = field(default_factory=dict)


def _is_tensor(x) -> bool:
    return isinstance(x, torch.Tensor)


def resolve_device(device, X) -> str:
    """Map ``device`` ('auto'|'cpu'|'cuda'|'gpu'|torch.device) to 'cpu' or 'cuda'."""
    if isinstance(device, torch.device):
        device = device.type
    device = (device or "auto").lower()
    if device in ("cuda", "gpu", "hip", "rocm"):
        if not torch.cuda.is_available():
            raise RuntimeError("device='cuda' requested but no GPU is visible")
        return "cuda"
    if device == "cpu":
        return "cpu"
    if device != "auto":
        raise ValueError(f"unknown device {device!r}")
    if _is_tensor(X) and X.is_cuda:
        return "cuda"
    if torch.cuda.is_available() and native.has_hip():
        n, F = X.shape
        if n * F >= AUTO_GPU_MIN_CELLS:
            return "cuda"
    return "cpu"


def _validate_X(X, allow_tensor=True):
    if _is_tensor(X):
        if X.dim() != 2:
            raise ValueError(f"Expected 2D array, got {X.dim()}D tensor")
        if X.shape[0] < 1:
            raise ValueError("Found array with 0 sample(s)")
        if not torch.is_floating_point(X):
            X = X.double()
        # device tensors are checked by the bin kernel (no extra pass / sync)
        if not X.is_cuda and not bool(torch.isfinite(X).all()):
            raise ValueError("Input X contains NaN or infinity.")
        return X
    X = np.asarray(X)
    if X.dtype == object:
        X = X.astype(np.float64)
    if X.ndim != 2:
        raise ValueError(f"Expected 2D array, got {X.ndim}D array instead")
    if X.shape[0] < 1:
        raise ValueError("Found array with 0 sample(s) (shape=%s)" % (X.shape,))
    if X.shape[1] < 1:
        raise ValueError("Found array with 0 feature(s)")
    if not np.issubdtype(X.dtype, np.number) and X.dtype != bool:
        raise ValueError(f"Unsupported feature dtype {X.dtype}")
    if X.dtype not in (np.float32, np.float64):
        X = X.astype(np.float64)
    if not np.isfinite(X).all():
        raise ValueError("Input X contains NaN or infinity.")
    return X


def _encode_labels(y, n):
    if _is_tensor(y):
        if y.dim() != 1 or y.shape[0] != n:
            raise ValueError("y must be 1-D with one label per row")
        if not torch.is_floating_point(y) and y.dtype != torch.bool and n > 0:
            # integer labels: a presence table instead of a sort (one small sync)
            lo, hi = torch.stack(torch.aminmax(y)).tolist()
            if hi - lo < (1 << 22):
                yz = (y - lo).long() if lo else y.long()
                present = torch.bincount(yz, minlength=hi - lo + 1) > 0
                lut = torch.cumsum(present, 0, dtype=torch.int32) - 1
                classes = (torch.nonzero(present).squeeze(1) + lo).to(y.dtype)
                return classes.cpu().numpy(), lut[yz]
        classes, enc = torch.unique(y, return_inverse=True)
        return classes.cpu().numpy(), enc.to(torch.int32)
    y = np.asarray(y)
    if y.ndim == 2 and y.shape[1] == 1:
        y = y.ravel()
    if y.ndim != 1 or y.shape[0] != n:
        raise ValueError(f"y must be 1-D with {n} labels, got shape {y.shape}")
    classes, enc = np.unique(y, return_inverse=True)
    return classes, enc.astype(np.int32)


def _ceil_log2(x: float) -> int:
    """ceil(log2(x)) for x > 0, exact (frexp: x = m 2^k, m in [0.5, 1)); the
    device encoder (misc.hip target_encode_kernel) computes it the same way."""
    m, k = math.frexp(x)
    return k - 1 if m == 0.5 else k


def fixed_point_exponent(absmax: float, n: int) -> int:
    """Exponent e with sum(|round(y * 2**e)|) < 2**62 for n rows."""
    if absmax <= 0 or not math.isfinite(absmax):
        return 0
    e = 62 - _ceil_log2(float(max(n, 1)) + 1.0) - _ceil_log2(absmax * (1 + 2**-40))
    return int(max(min(e, 1000), -1000))


def _encode_targets(y, n):
    if _is_tensor(y):
        if y.dim() != 1 or y.shape[0] != n:
            raise ValueError("y must be 1-D")
        yd = y.double()
        if not bool(torch.isfinite(yd).all()):
            raise ValueError("Input y contains NaN or infinity.")
        e = fixed_point_exponent(float(yd.abs().max().item()), n)
        return torch.round(torch.ldexp(yd, torch.tensor(float(e), device=y.device))).long(), e
    y = np.asarray(y, dtype=np.float64)
    if y.ndim == 2 and y.shape[1] == 1:
        y = y.ravel()
    if y.ndim != 1 or y.shape[0] != n:
        raise ValueError("y must be 1-D")
    if not np.isfinite(y).all():
        raise ValueError("Input y contains NaN or infinity.")
    e = fixed_point_exponent(float(np.abs(y).max()), n)
    return np.round(np.ldexp(y, e)).astype(np.int64), e


def _level_checkpoint(path, codes, y, params, n_classes):
    """A LevelCheckpoint for ``fit(..., checkpoint=path)`` (None: no checkpointing)."""
    if path is None:
        return None
    from ..utils.level_checkpoint import LevelCheckpoint, problem_signature

    if isinstance(path, LevelCheckpoint):  # tests pass a configured instance
        if not path.signature:
            path.signature = problem_signature(codes, y, params, n_classes)
        return path
    return LevelCheckpoint(path, problem_signature(codes, y, params, n_classes))


def _finalize(ta: TreeArrays, mapper: BinMapper, regression: bool, y_exp: int) -> TreeArrays:
    if ta.meta.pop("final", False):  # device assembly produced finished columns
        return ta
    if not ta.meta.pop("thresholds_set", False):
        ta.with_thresholds(mapper.edges)
    m = ta.n_samples.astype(np.float64)
    term = ta.impurity
    with np.errstate(invalid="ignore", divide="ignore"):
        if regression:
            s = ta.meta["sum_fixed"].astype(np.float64)
            ta.value = np.ldexp(s / np.maximum(m, 1), -y_exp)
            ta.meta["term"] = term
            ta.impurity = np.full(ta.node_count, np.nan)
        else:
            ta.meta["term"] = term
            ta.impurity = np.where(m > 0, term / np.maximum(m, 1), 0.0)
    return ta


def _exact_device_ok(n, F, C, regression, P=1, free_bytes=None, comm=None) -> bool:
    """The device-driven exact engine (``ops/exact_grower.py``) takes any
    feature count and any class count below 2^20 on fewer than 2^24 rows (its
    <= 256-row finisher jobs run where the local-code finishers fit: at most 256
    classes; otherwise its level loop grows to the leaves) -- when its workspace
    fits the device (no finisher: buffers grow as n F C)."""
    from ..ops.exact_grower import exact_fits_memory, exact_supported

    if not exact_supported(n, C, regression):
        return False
    return exact_fits_memory(n, F, C, regression, P, free_bytes, comm=comm)


def _fit_exact_device(Xd, prep, C, crit, params, comm, timings, t_bin, t_start, F, regression,
                      checkpoint=None):
    """Every unique value a threshold on continuous features, classification or
    regression: the device-driven presorted-list engine; feature-parallel over
    the ranks of a multi-GPU fit (``ops/exact_grower.py``). ``checkpoint``:
    level resume of the list engine (the signature covers the raw features)."""
    from ..ops.exact_grower import ExactGrower

    timings["bin"] = time.perf_counter() - t_bin
    root = prep.root
    yd = prep.y
    if root is None:  # (host-encoded labels / targets): one small device reduction
        if regression:
            mn, mx = torch.aminmax(yd)
            root = torch.stack([torch.tensor(yd.numel(), device=yd.device), yd.sum(), mn,
                                mx]).cpu().numpy()
        else:
            root = torch.bincount(yd.long(), minlength=C).cpu().numpy()
    # feature-parallel needs a feature block per rank; with fewer features than
    # ranks every rank grows the same tree on all features (replicated, as the
    # reference's ranks do above their split level)
    fp = comm.world_size > 1 and F >= comm.world_size
    if checkpoint is not None and comm.world_size > 1 and not fp:
        logger.warning("replicated exact fits (fewer features than ranks) keep no level "
                       "checkpoint: fitting without one")
        checkpoint = None
    ckpt = _level_checkpoint(checkpoint, Xd, yd, params, C)
    g = ExactGrower(params, comm if fp else None, checkpoint=ckpt)
    with roctx_range("mpitree.grow"):
        ta = g.fit(Xd, yd, root, C, crit, prep.y_exp, timings=timings)
    stats = dict(g.stats)
    stats["thresholds"] = "exact (presorted lists)"
    if comm.world_size > 1:
        stats["strategy"] = comm.kind
        if not fp:
            stats["mode"] = "replicated-exact"
    timings["total"] = time.perf_counter() - t_start
    mapper = BinMapper(edges=[], exact=np.ones(F, bool), max_bins=None)
    from ..ops.hip_backend import run_deferred

    run_deferred()
    return FitResult(arrays=ta, classes=prep.classes, n_features=F, mapper=mapper,
                     y_scale_exp=prep.y_exp, engine="hip-exact", timings=timings, stats=stats)


def fit_tree(
    X,
    y,
    *,
    regression: bool,
    criterion,
    max_depth,
    min_samples_split,
    min_samples_leaf=1,
    max_bins=None,
    device="auto",
    comm=None,
    finisher_rows=None,
    engine: str | None = None,
    checkpoint=None,
    _sync_prepare: bool = False,
) -> FitResult:
    t_start = time.perf_counter()
    X = _validate_X(X)
    n, F = X.shape
    crit = Criterion(criterion)
    if max_depth is not None and (int(max_depth) != max_depth or max_depth < 0):
        raise ValueError("max_depth must be None or a non-negative int")
    if int(min_samples_split) < 2:
        raise ValueError("min_samples_split must be >= 2")
    if int(min_samples_leaf) < 1:
        raise ValueError("min_samples_leaf must be >= 1")
    dev = resolve_device(device, X)
    comm = comm or LocalComm()
    classes, yv, y_exp, C = None, None, 0, 0
    sharded = bool(getattr(comm, "sharded", False))
    g_mapper = None
    if sharded:  # row shards: every rank must agree on bins, labels and the target scale
        from ..parallel.agreement import global_bin_mapper, global_classes, global_target_scale

        g_mapper = global_bin_mapper(comm, X, max_bins)
        if regression:
            absmax, n_tot = global_target_scale(comm, y)
            y_exp = fixed_point_exponent(absmax, n_tot)
            yh = np.asarray(y.detach().cpu().numpy() if _is_tensor(y) else y, np.float64).ravel()
            if yh.shape[0] != n:
                raise ValueError("y must be 1-D with one target per row")
            yv = np.round(np.ldexp(yh, y_exp)).astype(np.int64)
        else:
            classes = global_classes(comm, y)
            yh = np.asarray(y.detach().cpu().numpy() if _is_tensor(y) else y).ravel()
            if yh.shape[0] != n:
                raise ValueError("y must be 1-D with one label per row")
            yv = np.searchsorted(classes, yh).astype(np.int32)
            C = len(classes)
    elif dev != "cuda":  # the GPU path encodes labels alongside binning (gpu_prepare)
        if regression:
            yv, y_exp = _encode_targets(y, n)
        else:
            classes, yv = _encode_labels(y, n)
            C = len(classes)
    params = GrowParams(
        criterion=crit,
        max_depth=None if max_depth is None else int(max_depth),
        min_samples_split=int(min_samples_split),
        min_samples_leaf=int(min_samples_leaf),
    )
    timings = {}
    quantile_fallback = False
    if dev == "cuda":
        from ..ops.gpu_prepare import prepare
        from ..ops.hip_backend import HipBackend

        Xd = X if _is_tensor(X) else torch.from_numpy(np.ascontiguousarray(X))
        Xd = Xd.to("cuda")
        if Xd.dtype not in (torch.float32, torch.float64):
            Xd = Xd.double()
        Xd = Xd.contiguous()
        t0 = time.perf_counter()
        # a data-parallel rank of a replicated input bins only its own row shard
        # (the edges still come from every row, so all ranks derive one table; the
        # bin flags -- a missed exact value, non-finite input -- are combined over
        # the ranks before anyone grows)
        bin_rows, bin_agree = None, None
        lo, hi = comm.local_rows(n)
        if (lo, hi) != (0, n) and g_mapper is None:
            import torch.distributed as tdist

            bin_rows = (lo, hi)
            bin_agree = lambda fl: comm._all_reduce(fl, op=tdist.ReduceOp.MAX)  # noqa: E731
        with roctx_range("mpitree.bin"):
            if g_mapper is not None:  # globally agreed edges / encodings (row shards)
                from ..ops.gpu_prepare import prepare_with_mapper

                prep = prepare_with_mapper(Xd, yv, g_mapper, classes, y_exp)
            else:
                # max_bins=None (exact): bin at 256 first -- one code byte, the
                # histogram engines -- and take the presorted exact engine only
                # when some feature turns out to have more than 256 values
                from ..ops.exact_grower import MAX_ROWS

                probe = max_bins is None and 0 < n < MAX_ROWS
                # split: wait for the labels only, set up the label-dependent device
                # buffers while the edges / bin kernels run, then read the edge table
                split = bin_rows is None and os.environ.get("MPITREE_PREP_SPLIT", "1") != "0"
                prep = prepare(Xd, y, regression=regression,
                               max_bins=256 if max_bins is None else max_bins,
                               encode_labels=_encode_labels, encode_targets=_encode_targets,
                               exponent=fixed_point_exponent, sync=_sync_prepare,
                               exact_probe=probe, rows=bin_rows, agree=bin_agree, split=split)
                # the bin kernel's flags are read after growth (see prepare): a
                # sampled exact-mode feature that missed a value redoes the fit with
                # the flags checked first
                redo = dict(regression=regression, criterion=criterion,
                            max_depth=max_depth, min_samples_split=min_samples_split,
                            min_samples_leaf=min_samples_leaf, max_bins=max_bins,
                            device=device, comm=comm, finisher_rows=finisher_rows,
                            engine=engine, checkpoint=checkpoint, _sync_prepare=True)
        be_early = None
        if prep.resolve is not None:
            # the labels are known and the edges / bin kernels still run: the
            # histogram engine's label-dependent setup (row permutation, tables)
            # happens now, ahead of the edge table (unused if the fit goes exact)
            if (lo, hi) == (0, n):
                be_early = HipBackend()
                be_early.setup(prep.codes_rm, prep.codes_fm, prep.y.contiguous(), prep.nbins,
                               n_bins=256, n_classes=0 if regression else len(prep.classes),
                               criterion=crit)
            prep.resolve()
        mapper, codes_rm, codes_fm, nb = prep.mapper, prep.codes_rm, prep.codes_fm, prep.nbins
        yd, classes, y_exp, root = prep.y, prep.classes, prep.y_exp, prep.root
        C = 0 if regression else len(classes)
        from ..ops.exact_grower import needs_exact

        if max_bins is None and g_mapper is None and needs_exact(mapper):
            P_fp = comm.world_size if comm.world_size > 1 and F >= comm.world_size else 1
            if _exact_device_ok(n, F, C, regression, P_fp, comm=comm):
                # (the bin pass's flags -- non-finite input -- are read after the fit,
                # so the host enqueues the setup without waiting for them)
                try:
                    res = _fit_exact_device(Xd, prep, C, crit, params, comm, timings, t0,
                                            t_start, F, regression, checkpoint)
                except Exception:
                    # non-finite input (the bin pass's flags) explains any failure of
                    # the engine on it: that ValueError takes precedence
                    if prep.verify is not None and not prep.verify():
                        return fit_tree(X, y, **redo)
                    raise
                if prep.verify is not None and not prep.verify():
                    return fit_tree(X, y, **redo)
                return res
            logger.warning("exact thresholds on > 256-value features are not available on "
                           "the GPU for this fit (>= 2^24 rows, >= 2^20 classes, or a list "
                           "engine workspace beyond half the free device memory): using "
                           "256 quantile bins per feature")
            quantile_fallback = True
            if probe:  # the probe left out the quantile edges and the codes: bin again
                prep = prepare(Xd, y, regression=regression, max_bins=256,
                               encode_labels=_encode_labels, encode_targets=_encode_targets,
                               exponent=fixed_point_exponent, sync=True, rows=bin_rows,
                               agree=bin_agree)
                mapper, codes_rm, codes_fm, nb = (prep.mapper, prep.codes_rm, prep.codes_fm,
                                                  prep.nbins)
                yd, classes, y_exp, root = prep.y, prep.classes, prep.y_exp, prep.root
                be_early = None
        if (lo, hi) != (0, n):  # data-parallel shard of a replicated input
            if bin_rows is None:  # (binned every row: keep this rank's)
                codes_rm = codes_rm[lo:hi].contiguous()
                codes_fm = codes_fm[:, lo:hi].contiguous()
            yd = yd[lo:hi]
            root = None
        yd = yd.contiguous()
        timings["bin"] = time.perf_counter() - t0
        if debug_enabled():
            check_device_inputs(codes_rm, codes_fm, nb, yd, C, regression)
        if be_early is not None:  # (set up before the edge table: only B was open)
            be = be_early
            be.B = int(mapper.max_n_bins)
        else:
            be = HipBackend()
            be.setup(codes_rm, codes_fm, yd, nb, n_bins=mapper.max_n_bins, n_classes=C,
                     criterion=crit)
        be.timing = profiling()  # synchronised per-phase timers (host-driven loop)
        env = os.environ.get("MPITREE_FINISHER_ROWS")
        # subtree jobs of up to n / 128 rows: idle finisher workgroups split big
        # jobs between them (hand-off queue), so fewer replicated levels win
        # (profiles/kernel_experiments.md: 1M x 64 3.52 -> 3.33 ms at 2048 -> 8192)
        # (regression: the hand-off queue gains 0.35 ms at any of n/512 .. n/128)
        # (regression, round 6, tiny subtrees largest first: 1M x 64 2048 -> 3000 rows
        # 8.59 -> 8.49 ms over three A/B runs, profiles/r6/ab_reg_finisher_rows.log)
        # (classification below 524k rows, round 6: 100k x 32 2048 -> 4096 rows 1.20 ->
        # 1.11 ms at full depth, 1.13 -> 1.05 ms at depth 12; profiles/r6/ab_100k_*.log)
        # (a rank of a multi-GPU regression fit keeps 2048: its finisher holds 1/P of
        # the jobs, and fewer, larger ones balance worse -- simulated P = 8 rank 4.03
        # ms at 2048 vs 4.12 at 3000, profiles/r6/sim_reg_p8_floor2048.jsonl,
        # sim_own_after_tuning.jsonl)
        reg_floor = 3000 if comm.world_size == 1 else 2048
        default_fr = int(env) if env else (max(reg_floor, n // 512) if regression
                                           else max(4096, min(n // 128, 32768)))
        if not env and F > 128:
            # a finisher node scans F x B bins whatever its rows: past 128 features
            # smaller jobs (more level-loop levels, which scan many nodes at once) win
            # (200k x 512: classification 20.5 -> 11.8 ms at 512 rows; regression,
            # whose features past 256 read their bins from memory, 313 -> 76 ms at 128;
            # profiles/baseline_configs.md)
            # (wide regression, round 6: the tiny-subtree kernel now runs narrower
            # workgroups past ~300 features instead of handing those subtrees to the
            # block kernel -- 200k x 512 75 -> 24.7 ms -- and then 512-row jobs win:
            # 21.3 ms vs 22.6 at 256, 23.5 at 1024, 24.7 at 128;
            # profiles/r6/ab_reg_wide_tiny*.log. Past ~1100 features no tiny kernel.)
            wide_reg = 512 if F <= 1024 else 128
            default_fr = min(default_fr, wide_reg if (regression and F > 256)
                             else max(256, (1 << 18) // F))
        if not env and C > 2:
            # (more classes: no hand-off queue, and a node's histogram scan grows
            # with B * C -- smaller jobs keep every finisher workgroup busy)
            # (C = 64: 4096 -> 116.7 ms, 2048 -> 119.0, 1024 -> 134.5, 512 -> 168.0;
            # profiles/r4/ab_c64_finisher_rows.log; round 6, with the tiny subtrees
            # largest first: 4096 -> 88.5 ms, 3000 -> 85.1, 2600 -> 87.5, 3400 -> 86.9,
            # profiles/r6/ab_c64_finisher_rows.log -- measured at C = 64 only, so
            # fewer classes keep 4096)
            default_fr = min(default_fr, 4096 if C <= 16 else (3000 if C <= 64 else 2048))
        if not env and be.B > 256:
            # the same scan per node over B bins (16-bit codes): jobs shrink by 256 / B
            # (1M x 64, 1024 quantile bins: 7812 -> 2048 rows 33.8 -> 15.0 ms; 1024 rows
            # 15.6, 4096 rows 22.0; profiles/r6/ab_q1024_finisher_rows*.log)
            default_fr = max(1024, default_fr * 256 // int(be.B))
        if finisher_rows is None or (comm.world_size > 1 and comm.kind == "data"):
            # data-parallel GPU ranks finish subtrees on their owners (rows sent
            # there first), so the finisher applies as on one GPU
            finisher_rows = default_fr
        if not be.finisher_supported():
            finisher_rows = 0
        finisher_rows = min(int(finisher_rows), be.max_finisher_rows)
        params.finisher_rows = int(finisher_rows)
        from ..ops.device_grower import DeviceGrower, device_loop_supported

        if (lo, hi) == (0, n) and be.small_fit_supported(comm):
            checkpoint = None  # one kernel launch: nothing to resume
        ckpt = _level_checkpoint(checkpoint, codes_rm, yd, params, C)
        if ckpt is None and (lo, hi) == (0, n) and be.small_fit_supported(comm):
            # <= 1024 rows: the whole tree in one workgroup, any class count
            edges_h = None if prep.d_edges64 is not None else mapper.padded_edges()
            with roctx_range("mpitree.grow"):
                ta = be.fit_small(params, edges_h, d_edges=prep.d_edges64)
            eng = "hip-small"
            stats = {}
        elif device_loop_supported(be, params, comm):
            if comm.world_size > 1:  # the redundant top levels use the 1-GPU split point
                params.finisher_rows = min(default_fr, be.max_finisher_rows)
            builder = DeviceGrower(be, params, comm, checkpoint=ckpt)
            with roctx_range("mpitree.grow"):
                ta = builder.fit(hi - lo, C, F, mapper, y_exp, root=root,
                                 d_edges=prep.d_edges64)
            eng = "hip-device-loop"
        else:  # (host-driven levels: per-process checkpoints only)
            builder = LevelwiseBuilder(be, params, comm,
                                       checkpoint=ckpt if comm.world_size == 1 else None)
            with roctx_range("mpitree.grow"):
                ta = builder.fit(hi - lo, C, F, edges=mapper.padded_edges(), y_exp=y_exp)
            eng = "hip-levelwise"
        if eng != "hip-small":
            timings.update(builder.timings)
            stats = dict(builder.stats)
        if prep.verify is not None and not prep.verify():  # (the assembly has synced)
            return fit_tree(X, y, **redo)
    else:
        Xh = X.cpu().numpy() if _is_tensor(X) else X
        if _is_tensor(X) and X.is_cuda and not np.isfinite(Xh).all():
            raise ValueError("Input X contains NaN or infinity.")
        yh = yv.cpu().numpy() if _is_tensor(yv) else yv
        t0 = time.perf_counter()
        mapper = g_mapper if g_mapper is not None else fit_bin_mapper(Xh, max_bins)
        codes = mapper.transform(Xh)
        lo, hi = comm.local_rows(n)
        if (lo, hi) != (0, n):
            codes, yh = codes[lo:hi], yh[lo:hi]
        timings["bin"] = time.perf_counter() - t0
        use_native = (
            engine in (None, "native") and comm.world_size == 1 and native.has_cpu()
            and checkpoint is None  # the native builder is depth-first: no level state
        )
        if use_native:
            from ..ops.cpu_builder import fit_native

            ta = fit_native(codes, yh, mapper, C, params)
            eng = "cpu-native"
            stats = {}
        else:
            from .backend_numpy import NumpyBackend

            be = NumpyBackend()
            be.setup(codes, yh, n_bins=mapper.max_n_bins, n_classes=C, criterion=crit)
            params.finisher_rows = int(finisher_rows or 0)
            if checkpoint is not None and comm.world_size > 1:
                logger.warning("level checkpoints of multi-process CPU fits are not kept")
                checkpoint = None
            builder = LevelwiseBuilder(be, params, comm,
                                       checkpoint=_level_checkpoint(checkpoint, codes, yh,
                                                                    params, C))
            ta = builder.fit(hi - lo, C, F, edges=mapper.padded_edges())
            eng = "numpy-levelwise"
            timings.update(builder.timings)
            stats = dict(builder.stats)
    if comm.world_size > 1:
        stats["strategy"] = comm.kind
        stats["bytes_communicated"] = getattr(comm, "bytes_communicated", 0)
    if quantile_fallback:
        stats["thresholds"] = "quantile-256 fallback (exact thresholds unavailable for this fit)"
    t0 = time.perf_counter()
    ta = _finalize(ta, mapper, regression, y_exp)
    timings["finalize"] = time.perf_counter() - t0
    if debug_enabled():
        sharded = getattr(comm, "sharded", False)  # then n is this rank's rows only
        validate_tree(ta, n_rows=None if sharded else n, n_features=F, n_bins=mapper.n_bins)
    timings["total"] = time.perf_counter() - t_start
    if logger.isEnabledFor(logging.INFO):
        logger.info("fit: engine=%s n=%d F=%d nodes=%d depth=%d %.3f ms", eng, n, F,
                    ta.node_count, ta.max_depth, timings["total"] * 1e3)
        logger.debug("fit timings (ms): %s", {k: round(v * 1e3, 3) for k, v in timings.items()})
    if dev == "cuda":
        from ..ops.hip_backend import run_deferred

        run_deferred()  # (host work the level loop did not take: mapper tables)
    return FitResult(arrays=ta, classes=classes, n_features=F, mapper=mapper, y_scale_exp=y_exp,
                     engine=eng, timings=timings, stats=stats)
