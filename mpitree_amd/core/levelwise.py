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
the long tail of tiny levels. All host bookkeeping is vectorised over the
level's nodes.
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass

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

    def local_rows(self, n: int):
        """Row range of the (replicated) input this rank trains on."""
        return 0, n

    def reduce_hist(self, hist, n_slots: int):
        return None

    def combine_scan(self, res: dict) -> dict:
        return res

    def reduce_stats(self, stats: np.ndarray, reg: bool) -> np.ndarray:
        return stats

    def finish_assignment(self, m: np.ndarray) -> np.ndarray:
        """Which deferred subtrees this rank finishes (all of them locally)."""
        return np.ones(len(m), dtype=bool)

    def merge_subtrees(self, local: list, owned: np.ndarray, n_jobs: int) -> list:
        return local

    def fit_kwargs(self) -> dict:
        return {}


_DEFERRED = ("id", "start", "count", "m", "depth", "pos")


class _Table:
    """Growing node table (unordered ids; pre-ordered at the end)."""

    def __init__(self, C: int):
        self.C = C
        self.n = 0
        self.cap = 1024
        self.feature = np.full(self.cap, -1, np.int32)
        self.tbin = np.full(self.cap, -1, np.int32)
        self.left = np.full(self.cap, -1, np.int64)
        self.right = np.full(self.cap, -1, np.int64)
        self.depth = np.zeros(self.cap, np.int32)
        self.nsamp = np.zeros(self.cap, np.int64)
        self.stats = np.zeros((self.cap, C), np.int64)
        self.pos = np.zeros(self.cap, np.int64)  # pre-order position (with holes)

    def _grow(self, need):
        if need <= self.cap:
            return
        cap = max(need, 2 * self.cap)
        for name in ("feature", "tbin", "left", "right", "depth", "nsamp", "stats", "pos"):
            a = getattr(self, name)
            fill = -1 if name in ("feature", "tbin", "left", "right") else 0
            b = np.full((cap,) + a.shape[1:], fill, a.dtype)
            b[: self.n] = a[: self.n]
            setattr(self, name, b)
        self.cap = cap

    def add(self, depth, nsamp, stats, pos=None) -> np.ndarray:
        depth = np.atleast_1d(np.asarray(depth))
        k = depth.shape[0]
        self._grow(self.n + k)
        lo = self.n
        if pos is not None:
            self.pos[lo : lo + k] = pos
        self.depth[lo : lo + k] = depth
        self.nsamp[lo : lo + k] = nsamp
        self.stats[lo : lo + k] = np.asarray(stats, dtype=np.int64).reshape(k, self.C)
        self.n += k
        return np.arange(lo, lo + k)


def _node_terms(crit, stats: np.ndarray) -> np.ndarray:
    """Vectorised node terms for every node (stats: [N, C] counts or [N, 2])."""
    try:
        from ..ops import native

        return native.cpu().node_terms(np.ascontiguousarray(stats, dtype=np.int64), int(crit))
    except ImportError:
        pass
    if crit == Criterion.ENTROPY:
        return entropy_term(stats)
    if crit == Criterion.GINI:
        return gini_term(stats)
    return mse_term(stats[:, 0], stats[:, 1])


def _native_cpu():
    try:
        from ..ops import native

        return native.cpu()
    except ImportError:
        return None


def _host_threads() -> int:
    from ..ops import native

    return native.host_threads()


class LevelwiseBuilder:
    """Drive one fit through ``backend`` with communication hooks ``comm``."""

    def __init__(self, backend, params: GrowParams, comm=None, checkpoint=None):
        self.be = backend
        self.p = params
        self.comm = comm or LocalComm()
        # LevelCheckpoint (utils/level_checkpoint.py): state saved after every level
        self.ckpt = checkpoint
        if checkpoint is not None and self.comm.world_size != 1:
            raise ValueError("level checkpoints are supported for single-process fits")
        self.timings: dict = {}
        self.stats: dict = {}

    # ------------------------------------------------------------ helpers
    def _terminal(self, depth, m, stats, minmax=None) -> np.ndarray:
        p = self.p
        depth = np.asarray(depth)
        m = np.asarray(m)
        t = (m < p.min_samples_split) | (m < 2 * max(1, p.min_samples_leaf))
        if p.max_depth is not None:
            t |= depth >= p.max_depth
        if p.criterion == Criterion.SQUARED_ERROR:
            if minmax is not None:
                t |= minmax[:, 0] == minmax[:, 1]
        else:
            t |= (np.asarray(stats) > 0).sum(-1) <= 1
        return t

    def _tick(self, key, t0):
        self.be.sync()
        self.timings[key] = self.timings.get(key, 0.0) + time.perf_counter() - t0

    # ---------------------------------------------------------------- fit
    def fit(self, n_local: int, n_classes: int, n_features: int, edges=None,
            y_exp: int = 0) -> TreeArrays:
        """Grow the tree; ``edges`` ([F, B] padded bin edges) fills thresholds,
        ``y_exp`` is the regression targets' fixed-point exponent."""
        self._edges = edges
        self._y_exp = int(y_exp)
        self._fin = None
        p, be, comm = self.p, self.be, self.comm
        reg = p.criterion == Criterion.SQUARED_ERROR
        C = 2 if reg else n_classes
        f_lo, f_hi = comm.feature_range(n_features)
        F_h = f_hi - f_lo
        tab = _Table(C)
        state = self.ckpt.load() if self.ckpt is not None else None
        if state is not None:
            return self._resume(state, tab, n_local, C, F_h, f_lo, f_hi, reg)

        t0 = time.perf_counter()
        st = comm.reduce_stats(be.segment_stats(np.array([0]), np.array([n_local])), reg)
        self._tick("stats", t0)
        if reg:
            m_root, rstats, minmax = int(st[0, 0]), st[:, :2], st[:, 2:4]
        else:
            m_root, rstats, minmax = int(st[0].sum()), st, None
        root = tab.add(0, m_root, rstats, pos=0)
        # Device assembly: every node lives at its pre-order position with holes
        # (a subtree of m rows owns 2m - 1 positions: root, left, right), so the
        # backend lays the tree out on the device and compacts it in one pass.
        self._device_asm = (
            hasattr(be, "begin_positions") and comm.world_size == 1 and edges is not None
            and (os.environ.get("MPITREE_DEVICE_ASSEMBLY", "1") != "0"
                 # (the exact engine's thresholds exist only on the device)
                 or getattr(be, "thresholds_on_device", False))
            and self.ckpt is None
        )
        if self._device_asm:
            be.begin_positions(2 * m_root - 1)
        # frontier columns
        fr = dict(
            id=root,
            pos=np.zeros(1, np.int64),
            start=np.zeros(1, np.int64),
            count=np.array([n_local], np.int64),
            m=np.array([m_root], np.int64),
            depth=np.zeros(1, np.int64),
            src=np.full(1, -1, np.int64),  # parent slot in prev level if derived
            sib=np.full(1, -1, np.int64),  # frontier index of the built sibling
        )
        if self._terminal(np.zeros(1), np.array([m_root]), rstats, minmax)[0]:
            fr = {k: v[:0] for k, v in fr.items()}
        deferred = {k: [] for k in _DEFERRED}
        return self._grow(tab, fr, deferred, 0, C, F_h, f_lo, f_hi, reg)

    def _resume(self, state, tab, n_local, C, F_h, f_lo, f_hi, reg) -> TreeArrays:
        """Continue a fit from its last saved level (utils/level_checkpoint.py)."""
        self._device_asm = False
        ck = self.ckpt
        ck.restore_table(state, tab)
        self.be.set_rows(state["rows"])
        fr = ck.restore_frontier(state)
        deferred = ck.restore_deferred(state, _DEFERRED)
        self.stats["resumed_from_level"] = int(state["level"][0])
        return self._grow(tab, fr, deferred, int(state["level"][0]), C, F_h, f_lo, f_hi, reg)

    def _grow(self, tab, fr, deferred, levels, C, F_h, f_lo, f_hi, reg) -> TreeArrays:
        p, be, comm = self.p, self.be, self.comm
        prev_hist = None
        multi = comm.world_size > 1
        while fr["id"].size:
            if multi:  # failure containment: a failed peer / injected fault
                from ..parallel.failure import check_abort, fault_point

                check_abort()
                fault_point(comm, f"level:{levels}")
            levels += 1
            K = fr["id"].size
            # small subtrees go to the finisher (global row count decides)
            if p.finisher_rows > 0 and hasattr(be, "finish_subtrees"):
                small = fr["m"] <= p.finisher_rows
                if small.any():
                    for key in deferred:
                        deferred[key].append(fr[key][small])
                    if hasattr(be, "defer_segments"):
                        be.defer_segments(fr["start"][small], fr["count"][small])
                    keep = ~small
                    # derived nodes whose built sibling was deferred: build from rows
                    sib = fr["sib"]
                    lost = (fr["src"] >= 0) & small[np.maximum(sib, 0)]
                    fr["src"] = np.where(lost, -1, fr["src"])
                    new_index = np.cumsum(keep) - 1
                    fr["sib"] = np.where(fr["src"] >= 0, new_index[np.maximum(sib, 0)], -1)
                    fr = {k: v[keep] for k, v in fr.items()}
                    K = fr["id"].size
                    if K == 0:
                        break
            built = np.nonzero(fr["src"] < 0)[0]
            derived = np.nonzero(fr["src"] >= 0)[0]
            order = np.concatenate([built, derived])
            slot_of = np.empty(K, np.int64)
            slot_of[order] = np.arange(K)
            o = {k: v[order] for k, v in fr.items()}  # frontier in slot order
            nb = built.size
            hist = be.alloc_hist(K, F_h)
            t0 = time.perf_counter()
            if nb:
                be.build_hist(hist, np.arange(nb), o["start"][:nb], o["count"][:nb], f_lo, f_hi)
            self._tick("hist", t0)
            t0 = time.perf_counter()
            comm.reduce_hist(hist, nb)
            self._tick("reduce", t0)
            t0 = time.perf_counter()
            if derived.size:
                be.derive_hist(hist, prev_hist, np.arange(nb, K), o["src"][nb:],
                               slot_of[o["sib"][nb:]])
            self._tick("derive", t0)
            t0 = time.perf_counter()
            res = be.scan(hist, np.arange(K), p.min_samples_leaf, f_lo, f_hi)
            self._tick("scan", t0)
            t0 = time.perf_counter()
            res = comm.combine_scan(res)
            self._tick("combine", t0)
            split = np.nonzero(res["gain"] > -np.inf)[0]  # positions in slot order
            S = split.size
            ids = o["id"][split]
            tab.feature[ids] = res["feature"][split]
            tab.tbin[ids] = res["bin"][split]
            # partition rows of split nodes
            t0 = time.perf_counter()
            replicated = getattr(comm, "rows_replicated", True)
            nl_local = be.partition(o["start"][split], o["count"][split], res["feature"][split],
                                    res["bin"][split], need_counts=not replicated)
            if replicated:
                nl_local = np.asarray(res["n_left"])[split].astype(np.int64)
            self._tick("partition", t0)
            if S == 0:
                break
            # children (left, right interleaved: 2j, 2j+1)
            ml = np.asarray(res["n_left"])[split].astype(np.int64)
            m_par = o["m"][split]
            lstats = np.asarray(res["left"])[split].astype(np.int64)
            pstats = tab.stats[ids]
            cstats = np.stack([lstats, pstats - lstats], 1).reshape(2 * S, C)
            cm = np.stack([ml, m_par - ml], 1).reshape(-1)
            cstart = np.stack([o["start"][split], o["start"][split] + nl_local], 1).reshape(-1)
            ccount = np.stack([nl_local, o["count"][split] - nl_local], 1).reshape(-1)
            cdepth = np.repeat(o["depth"][split] + 1, 2)
            ppos = o["pos"][split]
            cpos = np.stack([ppos + 1, ppos + 2 * ml], 1).reshape(-1)
            cids = tab.add(cdepth, cm, cstats, pos=cpos)
            tab.left[ids] = cids[0::2]
            tab.right[ids] = cids[1::2]
            mm = None
            if reg:
                t0 = time.perf_counter()
                cs = comm.reduce_stats(be.segment_stats(cstart, ccount), reg)
                mm = cs[:, 2:4]
                self._tick("stats", t0)
            alive = ~self._terminal(cdepth, cm, cstats, mm)
            # the smaller child (ties: left) is built from rows, the larger is
            # derived as parent - sibling; the parent's slot is its position
            both = np.nonzero(alive[0::2] & alive[1::2])[0]
            big = np.where(ml <= (m_par - ml), 1, 0)  # offset of the larger child
            keep_idx = np.nonzero(alive)[0]
            new_pos = np.full(2 * S, -1, np.int64)
            new_pos[keep_idx] = np.arange(keep_idx.size)
            src = np.full(2 * S, -1, np.int64)
            sib = np.full(2 * S, -1, np.int64)
            if getattr(be, "derives", True):  # else every node is built from its rows
                src[2 * both + big[both]] = split[both]
                sib[2 * both + big[both]] = new_pos[2 * both + 1 - big[both]]
            fr = dict(
                id=cids[keep_idx],
                pos=cpos[keep_idx],
                start=cstart[keep_idx],
                count=ccount[keep_idx],
                m=cm[keep_idx],
                depth=cdepth[keep_idx].astype(np.int64),
                src=src[keep_idx],
                sib=sib[keep_idx],
            )
            prev_hist = hist
            if self.ckpt is not None:
                self.ckpt.save(levels, tab, fr, deferred, be.get_rows())
        self.stats["levels"] = levels
        if deferred["id"]:
            d = {k: np.concatenate(v) for k, v in deferred.items()}
            t0 = time.perf_counter()
            self._finish(tab, d)
            self._tick("finisher", t0)
            self.stats["finisher_subtrees"] = int(d["id"].size)
        t0 = time.perf_counter()
        ta = self._to_arrays(tab)
        self.timings["assemble"] = time.perf_counter() - t0
        if self.ckpt is not None:
            self.stats["checkpoint_levels_saved"] = self.ckpt.saved_levels
            self.ckpt.clear()
        return ta

    # ------------------------------------------------------------ finisher
    def _finish(self, tab: _Table, d: dict):
        """Grow each deferred subtree with the backend's subtree finisher."""
        comm = self.comm
        if self._device_asm:  # nodes stay in the device position space
            t0 = time.perf_counter()
            self.be.finish_subtrees(d["start"], d["count"], d["depth"], self.p,
                                    stats=tab.stats[d["id"]], positions=d["pos"])
            self.timings["finisher_device"] = time.perf_counter() - t0
            self._deferred_ids = np.asarray(d["id"], np.int64)
            return
        owned = comm.finish_assignment(d["m"])
        t0 = time.perf_counter()
        local = self.be.finish_subtrees(d["start"][owned], d["count"][owned], d["depth"][owned],
                                        self.p, stats=tab.stats[d["id"][owned]])
        self.timings["finisher_device"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        t = comm.merge_subtrees(local, owned, d["id"].size)
        self.timings["finisher_merge"] = time.perf_counter() - t0
        # ``t`` is one node table for all deferred subtrees (child links index
        # it, ``roots[j]`` is job j's root): append every row, link children,
        # then copy each root's split onto the deferred node it continues (the
        # appended copy of the root stays unreachable and is dropped when the
        # tree is re-numbered).
        T = len(t["feature"])
        if T == 0:
            return
        if _native_cpu() is not None:  # joined and renumbered natively in _to_arrays
            fin = t.get("i32")
            if fin is None:
                fin = np.stack([t["feature"], t["bin"], t["left"], t["right"], t["depth"],
                                t["nsamp"]], 1).astype(np.int32)
            cnt = t.get("cnt")
            if cnt is None:
                cnt = np.asarray(t["stats"], np.int64)
            self._fin = (fin, cnt, np.asarray(d["id"], np.int64),
                         np.asarray(t["roots"], np.int64))
            return
        base = tab.n
        tab.add(t["depth"], t["nsamp"], t["stats"])
        f = np.asarray(t["feature"])
        inner = f >= 0
        sl = slice(base, base + T)
        tab.feature[sl] = f
        tab.tbin[sl] = t["bin"]
        tab.left[sl] = np.where(inner, np.asarray(t["left"]) + base, -1)
        tab.right[sl] = np.where(inner, np.asarray(t["right"]) + base, -1)
        r = np.asarray(t["roots"], np.int64) + base
        did = d["id"]
        split = tab.feature[r] >= 0
        did, r = did[split], r[split]
        tab.feature[did] = tab.feature[r]
        tab.tbin[did] = tab.tbin[r]
        tab.left[did] = tab.left[r]
        tab.right[did] = tab.right[r]

    # -------------------------------------------------------------- output
    def _to_arrays_device(self, tab: _Table, reg: bool) -> TreeArrays:
        """Level-wise nodes join the finisher's in the device position space,
        which the backend compacts into finished pre-ordered columns."""
        n = tab.n
        keep = np.ones(n, bool)
        did = getattr(self, "_deferred_ids", None)
        if did is not None and did.size:
            keep[did] = False  # the finisher wrote these (with their splits)
        ids = np.nonzero(keep)[0]
        f = tab.feature[ids]
        inner = f >= 0
        lpos = np.where(inner, tab.pos[np.maximum(tab.left[ids], 0)], -1)
        rpos = np.where(inner, tab.pos[np.maximum(tab.right[ids], 0)], -1)
        self.be.put_positions(tab.pos[ids], f, tab.tbin[ids], lpos, rpos, tab.depth[ids],
                              tab.nsamp[ids], tab.stats[ids])
        # thresholds, impurity and values need no host pass (meta["final"])
        return self.be.assemble_positions(self._edges, int(self.p.criterion), self._y_exp)

    def _to_arrays(self, tab: _Table) -> TreeArrays:
        reg = self.p.criterion == Criterion.SQUARED_ERROR
        n = tab.n
        if self._device_asm:
            return self._to_arrays_device(tab, reg)
        cpu = _native_cpu()
        if cpu is not None:  # one native pass: join, pre-order, gather, thresholds, terms
            edges = self._edges
            C = tab.stats.shape[1]
            fin, cnt, did, roots = self._fin or (np.zeros((0, 6), np.int32),
                                                 np.zeros((0, C), np.int64),
                                                 np.zeros(0, np.int64), np.zeros(0, np.int64))
            a = cpu.assemble_tree(tab.feature[:n], tab.tbin[:n], tab.left[:n], tab.right[:n],
                                  tab.nsamp[:n], tab.stats[:n], fin, cnt, did, roots,
                                  np.empty((0, 0)) if edges is None else edges,
                                  int(self.p.criterion), _host_threads())
            st = a["stats"]
            ta = TreeArrays(
                feature=a["feature"], threshold=a.get("threshold", np.full(len(st), np.nan)),
                threshold_bin=a["bin"], left=a["left"], right=a["right"], depth=a["depth"],
                n_samples=a["nsamp"], impurity=a["term"],
                count=None if reg else st,
                value=st[:, 1].astype(np.float64) if reg else None,
            )
            ta.meta["thresholds_set"] = edges is not None
            if reg:
                ta.meta["sum_fixed"] = st[:, 1].copy()
            return ta
        st = tab.stats[:n]
        term = _node_terms(self.p.criterion, st)
        ta = TreeArrays.from_unordered(
            feature=tab.feature[:n],
            threshold_bin=tab.tbin[:n],
            left=tab.left[:n],
            right=tab.right[:n],
            n_samples=tab.nsamp[:n],
            impurity=term,
            count=None if reg else st,
            value=st[:, 1].astype(np.float64) if reg else None,
        )
        if reg:
            ta.meta["sum_fixed"] = ta.value.astype(np.int64)
            ta.meta["sum_fixed"] = TreeArrays.from_unordered(
                feature=tab.feature[:n], threshold_bin=tab.tbin[:n], left=tab.left[:n],
                right=tab.right[:n], n_samples=st[:, 1], impurity=term,
            ).n_samples.astype(np.int64)
        return ta
