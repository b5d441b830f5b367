"""Cross-rank agreement on the fit's encodings for row-sharded inputs.

With ``fit(X_shard, y_shard, data_sharded=True)`` every rank sees only its
own rows, yet the per-level histogram all-reduce sums bin ``b`` of every
rank -- so bin ``b`` must mean the same threshold everywhere, class ``k``
the same label, and the regression fixed-point scale the same exponent.
The reference never shards rows (``mpitree/tree/decision_tree.py:340-361``
hands every rank the full ``X, y``); this module is what makes sharding
produce the same tree as the concatenated single-process fit when the
sharded features are exact (at most ``max_bins`` unique values globally).

* :func:`global_classes`: all-gather of each rank's sorted label set -> union.
* :func:`global_target_scale`: all-reduce of ``max |y|`` and the row count ->
  one fixed-point exponent.
* :func:`global_bin_mapper`: a mergeable quantile summary per feature. Each
  rank sorts its shard's columns on its device (16 at a time) and keeps, per
  feature, its distinct values with their counts when there are at most
  ``max_bins`` of them, else ``SKETCH_K`` order statistics at evenly spaced
  ranks, each weighted by the exact number of rows it stands for (the last is
  the shard's maximum). One all-gather of the ``[F, SKETCH_K]`` summaries
  (values, weights) -- a few MB whatever the row count -- and every rank merges
  them identically: a feature whose union of distinct values fits
  ``max_bins`` keeps exact edges (the reference's thresholds), any other takes
  weighted upper-quantile edges (every edge a data value of some rank; rank
  error <= rows / SKETCH_K per rank). With ``max_bins=None`` (exact thresholds)
  a sharded fit needs every feature to have <= 256 distinct values globally:
  the presorted exact engine is not row-sharded, and gathering every unique
  value would make B ~ n bins -- the fit raises a ValueError that names the
  feature and the options instead.

Collectives go through the comm's host helpers (``_all_gather``,
``_all_reduce``).
"""

from __future__ import annotations

import numpy as np
import torch

from ..core.binning import BinMapper, quantile_edges

__all__ = ["global_classes", "global_target_scale", "global_bin_mapper"]


def _host(a) -> np.ndarray:
    if torch.is_tensor(a):
        return a.detach().cpu().numpy()
    return np.asarray(a)


def _gather_ragged(comm, vals: np.ndarray, dtype=np.float64) -> list:
    """All-gather 1-D arrays of per-rank length -> list of P arrays."""
    vals = np.asarray(vals, dtype=dtype)
    sizes = comm._all_gather(np.array([vals.size], np.int64)).reshape(-1)
    L = int(max(1, sizes.max()))
    buf = np.zeros(L, dtype=dtype)
    buf[: vals.size] = vals
    allv = comm._all_gather(buf.view(np.int64)).reshape(comm.world_size, L)
    return [allv[r].view(dtype)[: sizes[r]] for r in range(comm.world_size)]


def global_classes(comm, y_local) -> np.ndarray:
    """Sorted union of every rank's labels (numeric labels)."""
    y = _host(y_local).ravel()
    local = np.unique(y)
    if not np.issubdtype(local.dtype, np.number) and local.dtype != bool:
        raise TypeError("data_sharded=True needs numeric labels")
    kind = np.float64 if np.issubdtype(local.dtype, np.floating) else np.int64
    parts = _gather_ragged(comm, local.astype(kind), kind)
    return np.unique(np.concatenate(parts)).astype(local.dtype if local.size else kind)


def global_target_scale(comm, y_local) -> tuple[float, int]:
    """(global max |y|, global row count) for the fixed-point exponent."""
    y = _host(y_local).astype(np.float64).ravel()
    if y.size and not np.isfinite(y).all():
        raise ValueError("Input y contains NaN or infinity.")
    absmax = float(np.abs(y).max()) if y.size else 0.0
    a = comm._all_gather(np.array([np.float64(absmax)]).view(np.int64)).view(np.float64)
    n = comm._all_reduce(np.array([y.size], np.int64))
    return float(a.max()), int(n[0])


SKETCH_K = 4096  # order statistics per feature and rank in the merged summary
EXACT_SHARDED_LIMIT = 256  # max_bins=None: distinct values per feature a sharded fit allows


def _local_summary(X_local, cap: int, K: int):
    """Per feature: (values [F, K] float64, weights [F, K] int64, distinct [F]).
    Features with <= ``cap`` distinct values list them with their counts; the
    others list ``K`` order statistics at ranks ceil((i + 1) n / K) - 1 with the
    number of rows each stands for. Sorting runs where X lives (its device)."""
    Xt = X_local if torch.is_tensor(X_local) else torch.from_numpy(np.asarray(X_local))
    n, F = int(Xt.shape[0]), int(Xt.shape[1])
    vals = np.zeros((F, K), np.float64)
    wts = np.zeros((F, K), np.int64)
    distinct = np.zeros(F, np.int64)
    if n == 0:
        return vals, wts, distinct
    r = (np.arange(1, K + 1, dtype=np.int64) * n + K - 1) // K - 1
    r = np.unique(np.clip(r, 0, n - 1))
    w = np.diff(np.concatenate([[-1], r]))
    r_t = torch.from_numpy(r).to(Xt.device)
    for f0 in range(0, F, 16):
        s, _ = torch.sort(Xt[:, f0:f0 + 16].double(), dim=0)
        nd = ((s[1:] != s[:-1]).sum(0) + 1).cpu().numpy()
        samp = s.index_select(0, r_t).cpu().numpy()  # [len(r), cols]
        for j in range(s.shape[1]):
            f = f0 + j
            distinct[f] = nd[j]
            if nd[j] <= cap:
                u, c = torch.unique_consecutive(s[:, j], return_counts=True)
                vals[f, : u.numel()] = u.cpu().numpy()
                wts[f, : u.numel()] = c.cpu().numpy()
            else:
                vals[f, : r.size] = samp[:, j]
                wts[f, : r.size] = w
    return vals, wts, distinct


def _weighted_upper_quantiles(v: np.ndarray, w: np.ndarray, max_bins: int) -> np.ndarray:
    """Upper-quantile edges of a weighted sample (values ascending): for
    k = 1..B the first value whose cumulative weight reaches k / B of the total
    (the last edge is the largest value) -- quantile_edges with weights."""
    cw = np.cumsum(w)
    tot = int(cw[-1])
    k = np.arange(1, max_bins + 1, dtype=np.int64)
    target = (k * tot + max_bins - 1) // max_bins
    idx = np.minimum(np.searchsorted(cw, target, side="left"), v.size - 1)
    return np.unique(v[idx])


def global_bin_mapper(comm, X_local, max_bins) -> BinMapper:
    """One ``BinMapper`` agreed by every rank from mergeable per-rank summaries."""
    exact_mode = max_bins is None
    limit = EXACT_SHARDED_LIMIT if exact_mode else int(max_bins)
    F = int(X_local.shape[1])
    vals, wts, distinct = _local_summary(X_local, limit, SKETCH_K)
    P = comm.world_size
    allv = comm._all_gather(vals.view(np.int64)).view(np.float64).reshape(P, F, SKETCH_K)
    allw = comm._all_gather(wts).reshape(P, F, SKETCH_K)
    alld = comm._all_gather(distinct).reshape(P, F)
    edges, exact = [], np.zeros(F, dtype=bool)
    for f in range(F):
        m = allw[:, f, :] > 0
        v, w = allv[:, f, :][m], allw[:, f, :][m]
        local_exact = bool((alld[:, f] <= limit).all())
        if local_exact:
            u = np.unique(v)
            if u.size <= limit:
                edges.append(u)
                exact[f] = True
                continue
        if exact_mode:
            raise ValueError(
                f"data_sharded=True with exact thresholds (max_bins=None): feature {f} has more "
                f"than {EXACT_SHARDED_LIMIT} distinct values across the row shards. Exact "
                f"thresholds on continuous features need every rank to hold all rows (fit "
                f"without data_sharded: the feature-parallel exact engine splits the work); "
                f"or pass max_bins (e.g. 256) for quantile bins agreed from per-rank summaries.")
        order = np.argsort(v, kind="stable")
        edges.append(_weighted_upper_quantiles(v[order], w[order], limit))
    return BinMapper(edges=edges, exact=exact, max_bins=max_bins)
