"""Flat structure-of-arrays tree: the framework's canonical fitted-tree format.

Every builder (native CPU, level-wise CPU, gfx950 level-wise, distributed)
emits a :class:`TreeArrays`. Nodes are stored in depth-first pre-order (root
0, then the whole left subtree, then the right subtree), so two builders that
grow the same tree produce byte-identical arrays regardless of their growth
order; ``tests`` compare fits through :meth:`TreeArrays.equal`.

Conversions to and from the reference's linked ``Node`` graph
(reference: ``mpitree/tree/_base.py:22-101``) live here, as does the text
renderer (reference: ``mpitree/tree/decision_tree.py:250-307``).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from .node import BranchType, Node

__all__ = ["TreeArrays"]


@dataclass
class TreeArrays:
    feature: np.ndarray  # int32 [N], -1 for leaves
    threshold: np.ndarray  # float64 [N], nan for leaves
    threshold_bin: np.ndarray  # int32 [N], -1 for leaves
    left: np.ndarray  # int32 [N], -1 for leaves
    right: np.ndarray  # int32 [N], -1 for leaves
    depth: np.ndarray  # int32 [N]
    n_samples: np.ndarray  # int64 [N]
    impurity: np.ndarray  # float64 [N]
    count: Optional[np.ndarray] = None  # [N, C] class counts: int32 (GPU), int64 (host)
    value: Optional[np.ndarray] = None  # float64 [N] (regression leaf mean)
    meta: dict = field(default_factory=dict)

    @classmethod
    def from_packed(cls, buf: np.ndarray, N: int, C: int, regression: bool,
                    max_depth: int | None = None) -> "TreeArrays":
        """Views of the device assembly's packed columns (``ops/csrc/assemble.hip``
        ``asm_cols``): n_samples i64 | threshold f64 | impurity f64 + counts i32
        [N, C] (or the leaf value f64: a regression tree's impurity is NaN at every
        node, a read-only broadcast view here) | feature, threshold_bin, left,
        right, depth i32. Every column is final: no host pass follows."""
        o = 0

        def take(dtype, count):
            nonlocal o
            a = buf[o : o + count * np.dtype(dtype).itemsize].view(dtype)
            o += count * np.dtype(dtype).itemsize
            return a

        n_samples = take(np.int64, N)
        threshold = take(np.float64, N)
        count = value = None
        if regression:  # (impurity: NaN at every node of a regression tree)
            impurity = np.broadcast_to(np.float64(np.nan), (N,))
            value = take(np.float64, N)
        else:
            impurity = take(np.float64, N)
            count = take(np.int32, N * C).reshape(N, C)
        feature = take(np.int32, N)
        threshold_bin = take(np.int32, N)
        left = take(np.int32, N)
        right = take(np.int32, N)
        depth = take(np.int32, N)
        ta = cls(feature=feature, threshold=threshold, threshold_bin=threshold_bin, left=left,
                 right=right, depth=depth, n_samples=n_samples, impurity=impurity, count=count,
                 value=value)
        ta.meta["final"] = True  # thresholds, impurities and values need no host pass
        if max_depth is not None:
            ta.meta["max_depth"] = int(max_depth)
        return ta

    # ------------------------------------------------------------------ basics
    @property
    def node_count(self) -> int:
        return int(self.right.shape[0])

    @property
    def is_classifier(self) -> bool:
        return self.count is not None

    @property
    def max_depth(self) -> int:
        if "max_depth" in self.meta:
            return int(self.meta["max_depth"])  # device-assembled: reduced on the device
        return int(self.depth.max()) if self.node_count else 0

    @property
    def n_leaves(self) -> int:
        # every internal node has two children, so N = 2 L - 1 (O(1); a
        # (feature < 0).sum() over a 187k-node flagship tree costs ~130 us)
        return (self.node_count + 1) // 2 if self.node_count else 0

    def equal(self, other: "TreeArrays", *, check_impurity: bool = True) -> bool:
        names = ["feature", "threshold_bin", "left", "right", "depth", "n_samples"]
        for n in names:
            if not np.array_equal(getattr(self, n), getattr(other, n)):
                return False
        if not np.array_equal(self.threshold, other.threshold, equal_nan=True):
            return False
        if (self.count is None) != (other.count is None):
            return False
        if self.count is not None and not np.array_equal(self.count, other.count):
            return False
        if (self.value is None) != (other.value is None):
            return False
        if self.value is not None and not np.array_equal(self.value, other.value, equal_nan=True):
            return False
        if check_impurity and not np.array_equal(self.impurity, other.impurity, equal_nan=True):
            return False
        return True

    def leaf_label_index(self) -> np.ndarray:
        """argmax of per-class counts, ties to the lowest class (reference :125)."""
        return np.argmax(self.count, axis=1)

    # -------------------------------------------------------------- ordering
    @staticmethod
    def from_unordered(
        feature,
        threshold_bin,
        left,
        right,
        n_samples,
        impurity,
        *,
        count=None,
        value=None,
        root: int = 0,
        threshold=None,
    ) -> "TreeArrays":
        """Re-number an arbitrary node table into depth-first pre-order."""
        feature = np.asarray(feature)
        left = np.asarray(left, dtype=np.int64)
        right = np.asarray(right, dtype=np.int64)
        n = feature.shape[0]
        try:
            from ..ops import native

            cpu = native.cpu()
        except ImportError:
            cpu = None
        if cpu is not None:
            order, depth_old = cpu.preorder(feature.astype(np.int32), left, right, int(root))
            k = order.shape[0]
            new_id = np.full(n, -1, dtype=np.int64)
            new_id[order] = np.arange(k)
            return TreeArrays._reindex(order, new_id, depth_old, feature, left, right,
                                       threshold_bin, n_samples, impurity, count, value,
                                       threshold)
        # level-synchronous passes (vectorised over each depth):
        # 1) nodes per depth from the root, 2) subtree sizes bottom-up,
        # 3) pre-order index top-down: left = parent + 1, right = left + |left subtree|
        depth_old = np.zeros(n, dtype=np.int32)
        levels = [np.array([root], dtype=np.int64)]
        while True:
            cur = levels[-1]
            inner = cur[feature[cur] >= 0]
            if inner.size == 0:
                break
            nxt = np.concatenate([left[inner], right[inner]])
            depth_old[nxt] = len(levels)
            levels.append(nxt)
        size = np.ones(n, dtype=np.int64)
        for cur in reversed(levels):
            inner = cur[feature[cur] >= 0]
            size[inner] = 1 + size[left[inner]] + size[right[inner]]
        new_id = np.full(n, -1, dtype=np.int64)
        new_id[root] = 0
        for cur in levels:
            inner = cur[feature[cur] >= 0]
            new_id[left[inner]] = new_id[inner] + 1
            new_id[right[inner]] = new_id[inner] + 1 + size[left[inner]]
        k = int(size[root])
        order = np.empty(k, dtype=np.int64)
        reach = new_id >= 0
        order[new_id[reach]] = np.nonzero(reach)[0]
        return TreeArrays._reindex(order, new_id, depth_old, feature, left, right, threshold_bin,
                                   n_samples, impurity, count, value, threshold)

    @staticmethod
    def _reindex(order, new_id, depth_old, feature, left, right, threshold_bin, n_samples,
                 impurity, count, value, threshold) -> "TreeArrays":
        k = order.shape[0]
        f = feature[order].astype(np.int32)
        lm = left[order]
        rm = right[order]
        inner = f >= 0
        new_left = np.where(inner, new_id[np.where(inner, lm, 0)], -1).astype(np.int32)
        new_right = np.where(inner, new_id[np.where(inner, rm, 0)], -1).astype(np.int32)
        tb = np.where(inner, np.asarray(threshold_bin)[order], -1).astype(np.int32)
        thr = (
            np.where(inner, np.asarray(threshold, dtype=np.float64)[order], np.nan)
            if threshold is not None
            else np.full(k, np.nan)
        )
        return TreeArrays(
            feature=f,
            threshold=thr,
            threshold_bin=tb,
            left=new_left,
            right=new_right,
            depth=depth_old[order],
            n_samples=np.asarray(n_samples, dtype=np.int64)[order],
            impurity=np.asarray(impurity, dtype=np.float64)[order],
            count=None if count is None else np.asarray(count, dtype=np.int64)[order],
            value=None if value is None else np.asarray(value, dtype=np.float64)[order],
        )

    def with_thresholds(self, edges: list) -> "TreeArrays":
        """Fill ``threshold`` from per-feature bin edges (edge value of the bin)."""
        thr = np.full(self.node_count, np.nan)
        inner = np.nonzero(self.feature >= 0)[0]
        if inner.size:
            bmax = max(len(e) for e in edges)
            table = np.full((len(edges), bmax), np.nan)
            for f, e in enumerate(edges):
                table[f, : len(e)] = e
            thr[inner] = table[self.feature[inner], self.threshold_bin[inner]]
        self.threshold = thr
        return self

    # ------------------------------------------------------------- inference
    def apply(self, X: np.ndarray) -> np.ndarray:
        """Leaf index reached by each row (vectorised level-synchronous walk)."""
        X = np.asarray(X)
        n = X.shape[0]
        node = np.zeros(n, dtype=np.int64)
        if self.node_count == 0:
            return node
        active = np.nonzero(self.feature[node] >= 0)[0]
        while active.size:
            cur = node[active]
            f = self.feature[cur]
            go_left = X[active, f] <= self.threshold[cur]
            node[active] = np.where(go_left, self.left[cur], self.right[cur])
            active = active[self.feature[node[active]] >= 0]
        return node

    # ------------------------------------------------------------ Node graph
    def to_nodes(self, classes=None, *, regression: bool = False) -> Node:
        """Materialise the reference-style linked ``Node`` graph."""
        n = self.node_count
        nodes: list = [None] * n
        feature = self.feature
        for i in range(n):  # pre-order: parents come before children
            nodes[i] = None
        parent_of = np.full(n, -1, dtype=np.int64)
        inner = np.nonzero(feature >= 0)[0]
        parent_of[self.left[inner]] = inner
        parent_of[self.right[inner]] = inner
        labels = None
        if not regression:
            argm = self.leaf_label_index()
            labels = np.asarray(classes)[argm] if classes is not None else argm
        for i in range(n):
            p = parent_of[i]
            parent = nodes[p] if p >= 0 else None
            if regression:
                cnt = np.int64(self.n_samples[i])
            else:
                cnt = self.count[i].astype(np.int64)
            if feature[i] >= 0:
                node = Node(
                    value=np.int64(feature[i]),
                    threshold=float(self.threshold[i]),
                    count=cnt,
                    parent=parent,
                )
            else:
                val = float(self.value[i]) if regression else labels[i]
                if not regression and isinstance(val, (np.integer, int)):
                    val = np.int64(val)
                node = Node(value=val, count=cnt, parent=parent)
            nodes[i] = node
            if parent is not None:
                if self.left[p] == i:
                    parent.left = node
                else:
                    parent.right = node
        for i in range(n):  # glyph state as the reference renderer leaves it
            if feature[i] >= 0:
                lnode, rnode = nodes[self.left[i]], nodes[self.right[i]]
                if rnode.is_leaf:
                    lnode._btype, rnode._btype = BranchType.INTERIOR_LIKE, BranchType.LEAF_LIKE
                else:
                    rnode._btype, lnode._btype = BranchType.INTERIOR_LIKE, BranchType.LEAF_LIKE
        return nodes[0] if n else None

    @staticmethod
    def from_nodes(root: Node, classes=None, *, regression: bool = False) -> "TreeArrays":
        """Inverse of :meth:`to_nodes` (accepts reference-written pickles)."""
        feats, thr, left, right, depth, nsamp, cnts, vals = [], [], [], [], [], [], [], []
        stack = [(root, -1, 0, 0)]
        class_index = None
        if classes is not None and not regression:
            class_index = {c.item() if hasattr(c, "item") else c: i for i, c in enumerate(classes)}
        while stack:
            node, parent, side, d = stack.pop()
            i = len(feats)
            if parent >= 0:
                (left if side == 0 else right)[parent] = i
            leaf = node.is_leaf
            feats.append(-1 if leaf else int(node.value))
            thr.append(np.nan if leaf else float(node.threshold))
            left.append(-1)
            right.append(-1)
            depth.append(d)
            if regression:
                nsamp.append(int(np.asarray(node.count).sum()))
                vals.append(float(node.value) if leaf else np.nan)
            else:
                c = np.asarray(node.count, dtype=np.int64)
                cnts.append(c)
                nsamp.append(int(c.sum()))
            if not leaf:
                stack.append((node.right, i, 1, d + 1))
                stack.append((node.left, i, 0, d + 1))
        n = len(feats)
        ta = TreeArrays(
            feature=np.asarray(feats, dtype=np.int32),
            threshold=np.asarray(thr, dtype=np.float64),
            threshold_bin=np.full(n, -1, dtype=np.int32),
            left=np.asarray(left, dtype=np.int32),
            right=np.asarray(right, dtype=np.int32),
            depth=np.asarray(depth, dtype=np.int32),
            n_samples=np.asarray(nsamp, dtype=np.int64),
            impurity=np.full(n, np.nan),
            count=None if regression else np.stack(cnts).astype(np.int64),
            value=np.asarray(vals, dtype=np.float64) if regression else None,
        )
        if regression:
            # interior means from children (weighted), bottom-up over pre-order
            for i in range(n - 1, -1, -1):
                if ta.feature[i] >= 0:
                    lo, hi = ta.left[i], ta.right[i]
                    ta.value[i] = (
                        ta.value[lo] * ta.n_samples[lo] + ta.value[hi] * ta.n_samples[hi]
                    ) / max(ta.n_samples[i], 1)
        del class_index
        return ta

    # ------------------------------------------------------------ rendering
    def export_text(
        self,
        *,
        feature_names=None,
        class_names=None,
        precision: int = 2,
        classes=None,
        regression: bool = False,
    ) -> str:
        """Box-drawing render with the reference's exact layout rules.

        Interior nodes print their feature name, leaves their class name (or
        ``class: <label>``). Non-root nodes carry ``[<= t]``/``[> t]`` with the
        parent's threshold. An interior right child is printed before its
        sibling and drawn ``├──``; a child's prefix grows by ``"   "`` when its
        parent was drawn ``└──`` and by ``"│  "`` otherwise (the root included).
        """
        if self.node_count == 0:
            return ""
        lines: list[str] = []
        feature = self.feature
        labels = None
        if not regression:
            argm = self.leaf_label_index()
            labels = np.asarray(classes)[argm] if classes is not None else argm

        def label_of(i: int) -> str:
            if feature[i] >= 0:
                f = int(feature[i])
                return str(feature_names[f]) if feature_names is not None else f"feature_{f}"
            if regression:
                return f"value: {self.value[i]:.{precision}f}"
            lab = labels[i]
            if class_names is not None:
                return str(class_names[int(argm[i]) if classes is not None else int(lab)])
            return f"class: {lab}"

        # iterative DFS: (node, glyph, prefix, sign, parent_threshold)
        stack = [(0, BranchType.ROOT, "", None, None)]
        while stack:
            i, glyph, prefix, sign, pthr = stack.pop()
            text = f"{glyph.value} {label_of(i)}"
            if sign is not None:
                text = f"{text} [{sign} {pthr:.{precision}f}]"
            lines.append(prefix + text)
            if feature[i] < 0:
                continue
            lc, rc = int(self.left[i]), int(self.right[i])
            child_prefix = prefix + ("   " if glyph is BranchType.LEAF_LIKE else "│  ")
            thr = self.threshold[i]
            if feature[rc] >= 0:  # interior right child is drawn first
                order = [(rc, BranchType.INTERIOR_LIKE, ">"), (lc, BranchType.LEAF_LIKE, "<=")]
            else:
                order = [(lc, BranchType.INTERIOR_LIKE, "<="), (rc, BranchType.LEAF_LIKE, ">")]
            for child, g, s in reversed(order):
                stack.append((child, g, child_prefix, s, thr))
        return "\n".join(lines)

    # ---------------------------------------------------------- persistence
    def to_dict(self) -> dict:
        d = {
            k: getattr(self, k)
            for k in (
                "feature",
                "threshold",
                "threshold_bin",
                "left",
                "right",
                "depth",
                "n_samples",
                "impurity",
            )
        }
        if self.count is not None:
            d["count"] = self.count
        if self.value is not None:
            d["value"] = self.value
        return d

    @staticmethod
    def from_dict(d: dict) -> "TreeArrays":
        return TreeArrays(
            **{k: np.asarray(v) for k, v in d.items() if k not in ("count", "value", "meta")},
            count=None if d.get("count") is None else np.asarray(d["count"]),
            value=None if d.get("value") is None else np.asarray(d["value"]),
        )
