"""Feature binning: raw feature values -> small integer codes.

The reference considers every unique value of a feature as a threshold
(``np.unique(X[:, f])``, reference ``mpitree/tree/decision_tree.py:73``) and
routes ``x <= t`` left. We keep that contract exactly whenever a feature has at
most ``max_bins`` unique values ("exact" features): the bin edges *are* the
unique values and bin ``b`` holds the values equal to ``edges[b]``, so a split
"code <= b" is the reference split "x <= edges[b]". Features with more unique
values use quantile edges drawn from the data (every edge is a data value and
``x <= edges[b]`` <=> ``code <= b`` still holds), bounding the histogram size
that the gfx950 kernels work on.

Codes are ``uint8`` when every feature fits in 256 bins, ``uint16`` up to
65536 and ``uint32`` beyond (``max_bins=None``, the default, keeps every
unique value of every feature, as the reference does).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

__all__ = ["BinMapper", "TableBinMapper", "quantile_edges", "fit_bin_mapper"]

MAX_BINS_LIMIT = 65536


def quantile_edges(sorted_values: np.ndarray, max_bins: int) -> np.ndarray:
    """Upper-quantile edges taken from sorted sample values (all data values)."""
    s = sorted_values.shape[0]
    k = np.arange(1, max_bins + 1, dtype=np.int64)
    idx = np.minimum((k * s + max_bins - 1) // max_bins - 1, s - 1)
    return np.unique(sorted_values[idx])


@dataclass
class BinMapper:
    edges: list  # per-feature float64 sorted edge values
    exact: np.ndarray  # bool [F]
    max_bins: int

    @property
    def n_features(self) -> int:
        return len(self.edges)

    @property
    def n_bins(self) -> np.ndarray:
        return np.asarray([len(e) for e in self.edges], dtype=np.int32)

    @property
    def max_n_bins(self) -> int:
        return int(self.n_bins.max()) if self.edges else 1

    @property
    def code_dtype(self):
        b = self.max_n_bins
        return np.uint8 if b <= 256 else (np.uint16 if b <= 65536 else np.uint32)

    def padded_edges(self, dtype=np.float64) -> np.ndarray:
        """[F, Bmax] edge table padded with +inf (what the kernels search)."""
        bmax = self.max_n_bins
        out = np.full((self.n_features, bmax), np.inf, dtype=dtype)
        for f, e in enumerate(self.edges):
            out[f, : len(e)] = e
        return out

    def transform(self, X: np.ndarray) -> np.ndarray:
        """Row-major codes ``[n, F]``: first edge >= x, clamped to the last bin."""
        X = np.asarray(X)
        n, F = X.shape
        codes = np.empty((n, F), dtype=self.code_dtype)
        for f, e in enumerate(self.edges):
            c = np.searchsorted(e, X[:, f], side="left")
            np.minimum(c, len(e) - 1, out=c)
            codes[:, f] = c
        return codes


class TableBinMapper(BinMapper):
    """A :class:`BinMapper` over a padded edge table ``[F, W]`` plus bin counts
    (the device binner's host copy). The per-feature edge arrays are sliced on
    first use: a device fit only needs ``max_n_bins`` before its level loop,
    so no host work sits between the fit's sync and the first tree kernels."""

    def __init__(self, table: np.ndarray, n_bins: np.ndarray, exact: np.ndarray, max_bins: int):
        self._table = table
        self._nb = np.asarray(n_bins, dtype=np.int64)
        self._edges = None
        self.exact = exact
        self.max_bins = max_bins

    def own_table(self) -> None:
        """Copy the table if it is a view of another buffer (a reused pinned one)."""
        if self._table.base is not None:
            self._table = self._table.copy()

    @property
    def edges(self) -> list:
        if self._edges is None:
            self._edges = [self._table[f, : self._nb[f]].copy() for f in range(self._nb.size)]
        return self._edges

    @property
    def n_features(self) -> int:
        return int(self._nb.size)

    @property
    def n_bins(self) -> np.ndarray:
        return self._nb.astype(np.int32)

    @property
    def max_n_bins(self) -> int:  # (without slicing the per-feature edge lists)
        return int(self._nb.max()) if self._nb.size else 1

    def padded_edges(self, dtype=np.float64) -> np.ndarray:
        bmax = self.max_n_bins
        out = np.array(self._table[:, :bmax], dtype=dtype)
        out[np.arange(bmax)[None, :] >= self._nb[:, None]] = np.inf
        return out


def fit_bin_mapper(X: np.ndarray, max_bins=256, sample: int | None = None, seed: int = 0):
    """Compute per-feature edges on the host.

    ``max_bins=None`` requests exact mode for every feature (every unique
    value is an edge, however many). ``sample`` limits the rows used for
    quantile features; exact features are always detected on the full column.
    """
    X = np.asarray(X)
    if X.ndim != 2:
        raise ValueError("X must be 2-D")
    if max_bins is not None and not 2 <= int(max_bins) <= MAX_BINS_LIMIT:
        raise ValueError(f"max_bins must be None or in [2, {MAX_BINS_LIMIT}]")
    limit = np.iinfo(np.int64).max if max_bins is None else int(max_bins)
    n, F = X.shape
    edges, exact = [], np.zeros(F, dtype=bool)
    rows = None
    if sample is not None and n > sample:
        rng = np.random.default_rng(seed)
        rows = np.sort(rng.choice(n, size=sample, replace=False))
    for f in range(F):
        col = np.asarray(X[:, f], dtype=np.float64)
        u = np.unique(col) + 0.0  # -0.0 and 0.0 are one value: print it as 0.0
        if u.shape[0] <= limit:
            edges.append(u)
            exact[f] = True
            continue
        src = np.sort(col[rows]) if rows is not None else np.sort(col)
        edges.append(quantile_edges(src, limit))
    return BinMapper(edges=edges, exact=exact, max_bins=max_bins)
