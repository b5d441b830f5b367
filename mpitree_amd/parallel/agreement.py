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
* :func:`global_bin_mapper`: all-gather of each feature's local sorted unique
  values (or, above the exact limit, ``4 * max_bins`` local quantile
  candidates) -> the union; exact edges when the union fits ``max_bins``,
  else quantile edges over the union. Every edge is a data value of some
  rank, and every rank computes the identical table.

Collectives go through the comm's host helpers (``_all_gather``,
``_all_reduce``): a few KB once per fit.
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


def global_bin_mapper(comm, X_local, max_bins) -> BinMapper:
    """One ``BinMapper`` agreed by every rank from their local feature values."""
    limit = np.iinfo(np.int64).max if max_bins is None else int(max_bins)
    if torch.is_tensor(X_local):
        F = int(X_local.shape[1])
        cols = [torch.unique(X_local[:, f].double()).cpu().numpy() for f in range(F)]
    else:
        X = np.asarray(X_local, dtype=np.float64)
        F = X.shape[1]
        cols = [np.unique(X[:, f]) for f in range(F)]
    cand_cap = limit if max_bins is None else 4 * limit
    edges, exact = [], np.zeros(F, dtype=bool)
    # one gather per feature keeps each message ragged-small; features are few
    local_exact = np.array([c.size <= cand_cap for c in cols], np.int64)
    all_exact = comm._all_reduce(local_exact, op=torch.distributed.ReduceOp.MIN).astype(bool)
    for f in range(F):
        c = cols[f]
        if c.size > cand_cap:
            c = quantile_edges(c, cand_cap)  # local candidates (data values)
        u = np.unique(np.concatenate(_gather_ragged(comm, c)))
        if all_exact[f] and u.size <= limit:
            edges.append(u)
            exact[f] = True
        else:
            edges.append(quantile_edges(u, limit))
    return BinMapper(edges=edges, exact=exact, max_bins=max_bins)
