"""Logging, profiling switches, tree digests and fault injection.

The reference has no tracing, logging or failure handling: the notebook wraps
``fit`` in ``time.time()`` and prints on rank 0, and an exception inside one
rank's subtree deadlocks the others in ``allgather``
(``mpitree/tree/decision_tree.py:446-477``). This module is the framework's
small observability layer:

* ``logger`` -- the ``mpitree`` :mod:`logging` logger (silent by default).
* :func:`profiling` -- ``MPITREE_PROFILE=1`` turns on synchronised per-phase
  timers, per-level device event timings of the device loop, and ROCTX ranges
  (``torch.cuda.nvtx`` is ROCTX on ROCm builds) that show up in
  ``rocprofv3 --marker-trace``.
* :func:`tree_digest` -- a 63-bit digest of a fitted tree, used by the
  collective fit's cross-rank consistency check.
* :func:`maybe_inject_fault` -- ``MPITREE_FAULT_RANK=k`` makes rank k raise at
  the start of a collective fit (tests the abort path, never set in production).
"""

from __future__ import annotations

import contextlib
import hashlib
import logging
import os

import numpy as np

__all__ = [
    "logger",
    "profiling",
    "roctx_range",
    "tree_digest",
    "maybe_inject_fault",
    "InjectedFault",
]

logger = logging.getLogger("mpitree")
logger.addHandler(logging.NullHandler())


def profiling() -> bool:
    """True when ``MPITREE_PROFILE`` is set to a non-zero value."""
    return os.environ.get("MPITREE_PROFILE", "0") not in ("", "0", "false", "False")


@contextlib.contextmanager
def roctx_range(name: str):
    """A ROCTX range around a block when profiling (no-op otherwise)."""
    if not profiling():
        yield
        return
    try:
        import torch

        torch.cuda.nvtx.range_push(name)
        pushed = True
    except Exception:  # pragma: no cover - no GPU runtime
        pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


def tree_digest(ta) -> int:
    """63-bit digest of the tree: split features, bins and threshold values,
    child links and node sizes. Thresholds are hashed too, so ranks that
    disagree on bin edges (e.g. row shards binned apart) cannot match.
    xxh3 over the arrays in place: ~0.3 ms for 200k nodes."""
    thr = np.nan_to_num(np.asarray(ta.threshold, dtype=np.float64), nan=0.0)
    parts = (ta.feature, ta.threshold_bin, ta.left, ta.right, ta.n_samples, thr)
    try:
        import xxhash

        h = xxhash.xxh3_64()
        for a in parts:
            h.update(memoryview(np.ascontiguousarray(a)).cast("B"))
        d = h.intdigest()
    except ImportError:  # pragma: no cover - xxhash ships with the image
        h = hashlib.blake2b(digest_size=8)
        for a in parts:
            h.update(np.ascontiguousarray(a).tobytes())
        d = int.from_bytes(h.digest(), "little")
    return d & ((1 << 63) - 1)


class InjectedFault(RuntimeError):
    """Raised by :func:`maybe_inject_fault` on the configured rank."""


def maybe_inject_fault(rank: int, where: str = "fit") -> None:
    """Raise on rank ``MPITREE_FAULT_RANK`` (at ``MPITREE_FAULT_AT``, default fit)."""
    target = os.environ.get("MPITREE_FAULT_RANK")
    if target is None or target == "":
        return
    if int(target) == int(rank) and os.environ.get("MPITREE_FAULT_AT", "fit") == where:
        raise InjectedFault(f"injected fault on rank {rank} at {where}")
