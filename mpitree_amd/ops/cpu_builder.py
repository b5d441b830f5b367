"""Python wrapper of the native exact CPU builder (``mpitree_amd._cpu``)."""

from __future__ import annotations

import os

import numpy as np

from ..core.criterion import Criterion
from ..models.tree_arrays import TreeArrays
from . import native

__all__ = ["fit_native"]


def fit_native(codes, y, mapper, n_classes, params, n_threads=None) -> TreeArrays:
    """Depth-first exact fit on host codes with the shared integer criterion."""
    cpu = native.cpu()
    if n_threads is None:
        n_threads = int(os.environ.get("MPITREE_CPU_THREADS", min(8, os.cpu_count() or 1)))
    reg = params.criterion == Criterion.SQUARED_ERROR
    codes = np.ascontiguousarray(codes)
    yv = np.ascontiguousarray(y, dtype=np.int64 if reg else np.int32)
    out = cpu.build_tree(
        codes, yv, mapper.n_bins.astype(np.int32), int(n_classes), int(params.criterion),
        -1 if params.max_depth is None else int(params.max_depth),
        int(params.min_samples_split), int(params.min_samples_leaf), int(n_threads),
    )
    st = out["stats"]
    term = cpu.node_terms(st, int(params.criterion))
    ta = TreeArrays.from_unordered(
        feature=out["feature"], threshold_bin=out["bin"], left=out["left"], right=out["right"],
        n_samples=out["nsamp"], impurity=term, count=None if reg else st,
        value=st[:, 1].astype(np.float64) if reg else None,
    )
    if reg:
        ta.meta["sum_fixed"] = st[:, 1].astype(np.int64)  # builder ids are already pre-order
    return ta
