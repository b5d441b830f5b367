"""``MPITREE_DEBUG=1``: checked fits.

The reference has no checks beyond sklearn's input validation; an
inconsistent subtree from one MPI rank is silently attached
(``mpitree/tree/decision_tree.py:456-466``). With ``MPITREE_DEBUG`` set, a fit
additionally

* checks the device inputs the kernels index with before the first tree
  kernel runs (every bin code below its feature's bin count, every label code
  in ``[0, C)``, the row-major and feature-major code copies identical), so
  an out-of-range code surfaces as a Python error instead of an
  out-of-bounds LDS/global access inside a kernel, and
* validates the finished tree's structural invariants
  (:func:`validate_tree`): pre-order layout, child links, depths, row
  conservation ``n(left) + n(right) = n(parent)``, class-count conservation,
  split features / bins in range and non-empty children.

Both raise :class:`TreeInvariantError`. The checks cost a few device
reductions and O(N) host work, so they are off by default.
"""

from __future__ import annotations

import os

import numpy as np

__all__ = ["debug_enabled", "TreeInvariantError", "validate_tree", "check_device_inputs"]


class TreeInvariantError(AssertionError):
    """A fitted tree (or a kernel input) violates an invariant."""


def debug_enabled() -> bool:
    return os.environ.get("MPITREE_DEBUG", "0") not in ("", "0", "false", "False")


def _fail(msg: str, idx=None):
    if idx is not None:
        idx = np.atleast_1d(np.asarray(idx))
        msg += f" (first offending nodes: {idx[:8].tolist()})"
    raise TreeInvariantError(msg)


def validate_tree(ta, n_rows: int | None = None, n_features: int | None = None,
                  n_bins=None) -> None:
    """Check the structural invariants of a pre-ordered :class:`TreeArrays`."""
    N = ta.node_count
    if N == 0:
        _fail("empty tree")
    feat = np.asarray(ta.feature, np.int64)
    left = np.asarray(ta.left, np.int64)
    right = np.asarray(ta.right, np.int64)
    depth = np.asarray(ta.depth, np.int64)
    ns = np.asarray(ta.n_samples, np.int64)
    for name, a in (("threshold_bin", ta.threshold_bin), ("left", left), ("right", right),
                    ("depth", depth), ("n_samples", ns)):
        if np.asarray(a).shape[0] != N:
            _fail(f"column {name} has {np.asarray(a).shape[0]} rows, expected {N}")
    if depth[0] != 0:
        _fail("root depth is not 0")
    if n_rows is not None and ns[0] != n_rows:
        _fail(f"root holds {ns[0]} rows, expected {n_rows}")
    inner = feat >= 0
    leaf = ~inner
    ii = np.nonzero(inner)[0]
    if ((left[leaf] != -1) | (right[leaf] != -1)).any():
        _fail("leaf with children", np.nonzero(leaf & ((left != -1) | (right != -1)))[0])
    if n_features is not None and (feat[ii] >= n_features).any():
        _fail("split feature out of range", ii[feat[ii] >= n_features])
    # pre-order: the left child follows its parent, the right child follows the
    # left subtree; children are deeper by one and split the parent's rows
    if (left[ii] != ii + 1).any():
        _fail("left child is not the next node in pre-order", ii[left[ii] != ii + 1])
    if ((right[ii] <= left[ii]) | (right[ii] >= N)).any():
        _fail("right child index out of order", ii[(right[ii] <= left[ii]) | (right[ii] >= N)])
    l, r = left[ii], right[ii]
    if ((depth[l] != depth[ii] + 1) | (depth[r] != depth[ii] + 1)).any():
        _fail("child depth is not parent depth + 1")
    if (ns[l] + ns[r] != ns[ii]).any():
        _fail("children do not partition the parent's rows", ii[ns[l] + ns[r] != ns[ii]])
    if ((ns[l] <= 0) | (ns[r] <= 0)).any():
        _fail("empty child (zero-gain split taken)", ii[(ns[l] <= 0) | (ns[r] <= 0)])
    # every node except the root has exactly one parent
    parents = np.zeros(N, np.int64)
    np.add.at(parents, l, 1)
    np.add.at(parents, r, 1)
    if parents[0] != 0 or (parents[1:] != 1).any():
        _fail("node without exactly one parent", np.nonzero(parents[1:] != 1)[0] + 1)
    # right = left + size(left subtree): sizes from the pre-order suffix
    size = np.ones(N, np.int64)
    for i in ii[::-1]:
        size[i] = 1 + size[left[i]] + size[right[i]]
    if (right[ii] != left[ii] + size[l]).any():
        _fail("right child does not follow the left subtree", ii[right[ii] != left[ii] + size[l]])
    if size[0] != N:
        _fail(f"tree spans {size[0]} nodes, table has {N}")
    tb = np.asarray(ta.threshold_bin, np.int64)
    if (tb[ii] < 0).any():
        _fail("internal node without a threshold bin", ii[tb[ii] < 0])
    if n_bins is not None:
        nb = np.asarray(n_bins, np.int64)
        bad = tb[ii] >= nb[feat[ii]] - 1  # the last bin sends every row left
        if bad.any():
            _fail("threshold bin out of range", ii[bad])
    if ta.count is not None:
        cnt = np.asarray(ta.count, np.int64)
        if (cnt.sum(1) != ns).any():
            _fail("class counts do not sum to n_samples", np.nonzero(cnt.sum(1) != ns)[0])
        if (cnt[l] + cnt[r] != cnt[ii]).any():
            _fail("children's class counts do not add up to the parent's")
        if (cnt < 0).any():
            _fail("negative class count")


def check_device_inputs(codes_rm, codes_fm, nbins, y, n_classes: int, regression: bool) -> None:
    """Range checks on the device tensors the kernels index with."""
    import torch

    n = codes_rm.shape[0]
    F = codes_fm.shape[0]
    if codes_fm.shape[1] != n:
        _fail(f"feature-major codes are {tuple(codes_fm.shape)}, expected ({F}, {n})")
    if n == 0:
        return
    nb = nbins.to(torch.int64)
    mx = codes_fm.to(torch.int64).amax(1)
    bad = torch.nonzero(mx >= nb).flatten()
    if bad.numel():
        _fail(f"bin code >= bin count for features {bad[:8].tolist()}")
    rm = codes_rm[:, :F]
    if not torch.equal(rm.t(), codes_fm):
        _fail("row-major and feature-major codes differ")
    if not regression:
        lo, hi = torch.aminmax(y.to(torch.int64))
        if int(lo) < 0 or int(hi) >= n_classes:
            _fail(f"label codes span [{int(lo)}, {int(hi)}], expected [0, {n_classes})")
