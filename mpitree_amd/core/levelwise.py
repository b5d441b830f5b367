"""Level-wise (breadth-first) tree grower shared by every backend and strategy.

The reference grows the tree depth-first, recursing per node and splitting
the MPI communicator at each split (``mpitree/tree/decision_tree.py:93-166``
serial, ``:364-479`` parallel). Each node's decision depends only on its own
rows, so growing all nodes of a depth together yields the same tree while
turning the per-node work into a handful of large batched device operations
per level:

1. **histogram** -- per frontier node, ``[F, B, C]`` class counts (or count
   and fixed-point target sum). Only the smaller child of each split is built
   from rows; its sibling is ``parent - child`` (``derive_hist``).
2. **communicate** -- strategy hook: data-parallel ranks all-reduce the built
   histograms; feature-parallel ranks skip it.
3. **scan** -- best threshold per (node, feature), best feature per node.
4. **communicate** -- feature-parallel ranks all-gather per-node candidates.
5. **partition** -- rows of split nodes are reordered inside their segment of
   the row-index permutation, left rows first.

Children whose fate is already known from the parent's split record (pure,
``max_depth`` reached, fewer than ``min_samples_split`` rows) become leaves
without any device work. Subtrees that become small enough are handed to the
backend's subtree finisher (one workgroup per subtree on gfx950), which removes
the long tail of tiny levels.
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from .criterion import Criterion, entropy_term, gini_term, mse_term
from ..models.tree_arrays import TreeArrays

__all__ = ["GrowParams", "LevelwiseBuilder", "LocalComm"]


@dataclass
class GrowParams:
    criterion: Criterion = Criterion.ENTROPY
    max_depth: int | None = None
    min_samples_split: int = 2
    min_samples_leaf: int = 1
    # Subtrees with at most this many rows are finished by the backend's
    # subtree finisher (0 disables the finisher).
    finisher_rows: int = 0


class LocalComm:
    """Single-process communication hooks (every collective is the identity)."""

    rank = 0
    world_size = 1
    kind = "local"
    rows_replicated = True  # every rank holds all rows: local left counts == global

    def feature_range(self, F: int):
        return 0, F

    def reduce_hist(self, hist, n_slots: int):
        return None

    def combine_scan(self, res: dict) -> dict:
        return res

    def reduce_stats(self, stats: np.ndarray, reg: bool) -> np.ndarray:
        return stats

    def owns_subtree(self, j: int) -> bool:
        return True


@dataclass
class _Table:
    C: int
    reg: bool
    feature: list = field(default_factory=list)
    tbin: list = field(default_factory=list)
    left: list = field(default_factory=list)
    right: list = field(default_factory=list)
    depth: list = field(default_factory=list)
    nsamp: list = field(default_factory=list)
    term: list = field(default_factory=list)
    stats: list = field(default_factory=list)  # class counts or (count, sum)

    def add(self, depth, nsamp, stats, term) -> int:
        i = len(self.feature)
        self.feature.append(-1)
        self.tbin.append(-1)
        self.left.append(-1)
        self.right.append(-1)
        self.depth.append(depth)
        self.nsamp.append(nsamp)
        self.stats.append(np.asarray(stats, dtype=np.int64))
        self.term.append(term)
        return i


def _node_term(crit, stats):
    if crit == Criterion.ENTROPY:
        return float(entropy_term(stats))
    if crit == Criterion.GINI:
        return float(gini_term(stats))
    return float(mse_term(int(stats[0]), int(stats[1])))


class LevelwiseBuilder:
    """Drive one fit through ``backend`` with communication hooks ``comm``."""

    def __init__(self, backend, params: GrowParams, comm=None):
        self.be = backend
        self.p = params
        self.comm = comm or LocalComm()
        self.timings: dict = {}
        self.stats: dict = {}

    # ------------------------------------------------------------ helpers
    def _terminal(self, depth, m, stats, minmax=None) -> bool:
        p = self.p
        if p.max_depth is not None and depth >= p.max_depth:
            return True
        if m < p.min_samples_split or m < 2 * max(1, p.min_samples_leaf):
            return True
        if p.criterion == Criterion.SQUARED_ERROR:
            return minmax is not None and minmax[0] == minmax[1]
        return int((np.asarray(stats) > 0).sum()) <= 1

    def _tick(self, key, t0):
        self.be.sync()
        self.timings[key] = self.timings.get(key, 0.0) + time.perf_counter() - t0

    # ---------------------------------------------------------------- fit
    def fit(self, n_local: int, n_classes: int, n_features: int) -> TreeArrays:
        p, be, comm = self.p, self.be, self.comm
        reg = p.criterion == Criterion.SQUARED_ERROR
        C = 2 if reg else n_classes
        f_lo, f_hi = comm.feature_range(n_features)
        tab = _Table(C=C, reg=reg)

        # root statistics (global)
        st = comm.reduce_stats(be.segment_stats(np.array([0]), np.array([n_local])), reg)[0]
        if reg:
            m_root, rstats, minmax = int(st[0]), st[:2], st[2:4]
        else:
            m_root, rstats, minmax = int(st.sum()), st, None
        root = tab.add(0, m_root, rstats, _node_term(p.criterion, rstats))
        # frontier arrays: node id, local start, local count, global count,
        # hist source (-1 = build from rows, else parent slot in prev level),
        # sibling frontier index for derived nodes
        frontier = []
        deferred = []  # (node id, start, count, depth) for the subtree finisher
        if not self._terminal(0, m_root, rstats, minmax):
            frontier.append(dict(id=root, start=0, count=n_local, m=m_root, depth=0,
                                 src=-1, sib=-1, slot_prev=-1))
        prev_hist = None
        levels = 0
        while frontier:
            levels += 1
            # small subtrees go to the finisher (global row count decides)
            if p.finisher_rows > 0 and hasattr(be, "finish_subtrees"):
                keep = []
                for nd in frontier:
                    if nd["m"] <= p.finisher_rows:
                        deferred.append(nd)
                    else:
                        keep.append(nd)
                if len(keep) != len(frontier):
                    # a derived node whose sibling left the frontier must be built
                    ids = {id(nd) for nd in keep}
                    for nd in keep:
                        if nd["src"] >= 0 and id(nd["sib_ref"]) not in ids:
                            nd["src"] = -1
                frontier = keep
                if not frontier:
                    break
            # slots: nodes built from rows first (contiguous for all-reduce)
            built = [nd for nd in frontier if nd["src"] < 0]
            derived = [nd for nd in frontier if nd["src"] >= 0]
            order = built + derived
            for s, nd in enumerate(order):
                nd["slot"] = s
            hist = be.alloc_hist(len(order), f_hi - f_lo)
            t0 = time.perf_counter()
            if built:
                be.build_hist(
                    hist,
                    np.array([nd["slot"] for nd in built]),
                    np.array([nd["start"] for nd in built]),
                    np.array([nd["count"] for nd in built]),
                    f_lo,
                    f_hi,
                )
            self._tick("hist", t0)
            t0 = time.perf_counter()
            comm.reduce_hist(hist, len(built))
            self._tick("reduce", t0)
            t0 = time.perf_counter()
            if derived:
                be.derive_hist(
                    hist,
                    prev_hist,
                    np.array([nd["slot"] for nd in derived]),
                    np.array([nd["src"] for nd in derived]),
                    np.array([nd["sib_ref"]["slot"] for nd in derived]),
                )
            self._tick("derive", t0)
            t0 = time.perf_counter()
            res = be.scan(hist, np.arange(len(order)), p.min_samples_leaf, f_lo, f_hi)
            self._tick("scan", t0)
            t0 = time.perf_counter()
            res = comm.combine_scan(res)
            self._tick("combine", t0)
            split = np.nonzero(res["gain"] > -np.inf)[0]
            # partition rows of split nodes
            t0 = time.perf_counter()
            replicated = getattr(comm, "rows_replicated", True)
            nl_local = be.partition(
                np.array([order[j]["start"] for j in split], dtype=np.int64),
                np.array([order[j]["count"] for j in split], dtype=np.int64),
                res["feature"][split],
                res["bin"][split],
                need_counts=not replicated,
            )
            if replicated:
                nl_local = np.asarray(res["n_left"])[split].astype(np.int64)
            self._tick("partition", t0)
            # children
            child_stats = None
            if reg and len(split):
                starts, counts = [], []
                for k, j in enumerate(split):
                    nd = order[j]
                    starts += [nd["start"], nd["start"] + nl_local[k]]
                    counts += [nl_local[k], nd["count"] - nl_local[k]]
                t0 = time.perf_counter()
                child_stats = comm.reduce_stats(
                    be.segment_stats(np.array(starts), np.array(counts)), reg
                )
                self._tick("stats", t0)
            nxt = []
            for k, j in enumerate(split):
                nd = order[j]
                nid = nd["id"]
                tab.feature[nid] = int(res["feature"][j])
                tab.tbin[nid] = int(res["bin"][j])
                ml = int(res["n_left"][j])
                pstats = tab.stats[nid]
                lstats = np.asarray(res["left"][j], dtype=np.int64)
                rstats = pstats - lstats
                d = nd["depth"] + 1
                kids = []
                for side, (cs, cm, lst, lct) in enumerate(
                    (
                        (lstats, ml, nd["start"], int(nl_local[k])),
                        (rstats, nd["m"] - ml, nd["start"] + int(nl_local[k]),
                         nd["count"] - int(nl_local[k])),
                    )
                ):
                    cid = tab.add(d, cm, cs, _node_term(p.criterion, cs))
                    if side == 0:
                        tab.left[nid] = cid
                    else:
                        tab.right[nid] = cid
                    mm = None
                    if reg:
                        mm = child_stats[2 * k + side][2:4]
                    if not self._terminal(d, cm, cs, mm):
                        kids.append(dict(id=cid, start=lst, count=lct, m=cm, depth=d,
                                         src=-1, sib=-1, slot_prev=nd["slot"]))
                if len(kids) == 2:
                    a, b = kids
                    # build the smaller child (ties: left), derive the larger
                    small, large = (a, b) if a["m"] <= b["m"] else (b, a)
                    large["src"] = nd["slot"]
                    large["sib_ref"] = small
                nxt.extend(kids)
            prev_hist = hist
            frontier = nxt
        self.stats["levels"] = levels
        if deferred:
            t0 = time.perf_counter()
            self._finish(tab, deferred)
            self._tick("finisher", t0)
        return self._to_arrays(tab)

    # ------------------------------------------------------------ finisher
    def _finish(self, tab: _Table, deferred: list):
        """Grow each deferred subtree with the backend's subtree finisher."""
        p = self.p
        sub = self.be.finish_subtrees(
            np.array([nd["start"] for nd in deferred], dtype=np.int64),
            np.array([nd["count"] for nd in deferred], dtype=np.int64),
            np.array([nd["depth"] for nd in deferred], dtype=np.int64),
            p,
            self.comm,
        )
        # ``sub`` holds one node table per deferred subtree, root first, with
        # local child indices; splice them into the global table.
        for nd, t in zip(deferred, sub):
            base = len(tab.feature) - 1  # local index 0 maps onto nd['id']
            nloc = len(t["feature"])
            gid = [nd["id"]] + list(range(base + 1, base + nloc))
            for li in range(nloc):
                if li > 0:
                    tab.add(int(t["depth"][li]), int(t["nsamp"][li]), t["stats"][li],
                            float(t["term"][li]))
                g = gid[li]
                if t["feature"][li] >= 0:
                    tab.feature[g] = int(t["feature"][li])
                    tab.tbin[g] = int(t["bin"][li])
                    tab.left[g] = gid[int(t["left"][li])]
                    tab.right[g] = gid[int(t["right"][li])]

    # -------------------------------------------------------------- output
    def _to_arrays(self, tab: _Table) -> TreeArrays:
        reg = tab.reg
        st = np.stack(tab.stats) if tab.stats else np.zeros((0, tab.C), np.int64)
        nsamp = np.asarray(tab.nsamp, dtype=np.int64)
        ta = TreeArrays.from_unordered(
            feature=np.asarray(tab.feature, dtype=np.int32),
            threshold_bin=np.asarray(tab.tbin, dtype=np.int32),
            left=np.asarray(tab.left, dtype=np.int64),
            right=np.asarray(tab.right, dtype=np.int64),
            n_samples=nsamp,
            impurity=np.asarray(tab.term, dtype=np.float64),
            count=None if reg else st,
            value=st[:, 1].astype(np.float64) if reg else None,
        )
        if reg:
            # keep exact fixed-point sums alongside (value is filled by the estimator)
            order_sum = TreeArrays.from_unordered(
                feature=np.asarray(tab.feature, dtype=np.int32),
                threshold_bin=np.asarray(tab.tbin, dtype=np.int32),
                left=np.asarray(tab.left, dtype=np.int64),
                right=np.asarray(tab.right, dtype=np.int64),
                n_samples=st[:, 1],
                impurity=np.asarray(tab.term, dtype=np.float64),
            )
            ta.meta["sum_fixed"] = order_sum.n_samples.astype(np.int64)
        return ta
