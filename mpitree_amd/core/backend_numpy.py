"""Host (numpy/torch-CPU) implementation of the level-wise engine's device ops.

This backend runs the exact same level-wise algorithm as the gfx950 backend
(:mod:`mpitree_amd.ops.hip_backend`) with plain numpy arithmetic. It serves the
CPU-only test environment, the multi-process ``gloo`` distributed tests
(histograms are torch CPU tensors so they can be handed to
``torch.distributed``), and as a readable specification of each kernel.
"""

from __future__ import annotations

import numpy as np
import torch

from .criterion import Criterion, entropy_term, gini_term, mse_term, tie_round

__all__ = ["NumpyBackend"]


class NumpyBackend:
    name = "numpy"
    device = torch.device("cpu")

    def __init__(self):
        self.codes = None

    # ------------------------------------------------------------- setup
    def setup(self, codes, y, *, n_bins: int, n_classes: int, criterion: Criterion):
        self.codes = np.ascontiguousarray(codes)
        self.n, self.F = self.codes.shape
        self.y = np.ascontiguousarray(y)
        self.B = int(n_bins)
        self.C = int(n_classes)
        self.crit = criterion
        self.reg = criterion == Criterion.SQUARED_ERROR
        self.idx = np.arange(self.n, dtype=np.int64)

    def alloc_hist(self, slots: int, F_h: int | None = None) -> torch.Tensor:
        # [slots, F_h, B, C] class counts; regression payload [..., 2] = {count, fixed sum}
        F_h = self.F if F_h is None else F_h
        last = 2 if self.reg else self.C
        return torch.zeros((max(slots, 1), F_h, self.B, last), dtype=torch.int64)

    # ------------------------------------------------------ histogram ops
    def build_hist(self, hist, slots, starts, counts, f_lo=0, f_hi=None):
        f_hi = self.F if f_hi is None else f_hi
        h = hist.numpy()
        for s, st, ct in zip(slots, starts, counts):
            rows = self.idx[st : st + ct]
            cn = self.codes[rows, f_lo:f_hi].astype(np.int64)
            fi = np.broadcast_to(np.arange(f_hi - f_lo), cn.shape)
            yn = self.y[rows]
            out = np.zeros(h.shape[1:], dtype=np.int64)
            if self.reg:
                np.add.at(out, (fi, cn, 0), 1)
                np.add.at(out, (fi, cn, 1), np.broadcast_to(yn[:, None], cn.shape))
            else:
                np.add.at(out, (fi, cn, np.broadcast_to(yn[:, None], cn.shape)), 1)
            h[s] = out

    def derive_hist(self, hist, prev_hist, slots, parent_slots, sibling_slots):
        h = hist.numpy()
        p = prev_hist.numpy()
        for s, ps, ss in zip(slots, parent_slots, sibling_slots):
            h[s] = p[ps] - h[ss]

    # ----------------------------------------------------------- split scan
    def scan(self, hist, slots, min_samples_leaf=1, f_lo=0, f_hi=None):
        """Best split per node over features ``[f_lo, f_hi)``.

        Returns a dict of per-node numpy arrays: ``gain`` (-inf if none),
        ``feature``, ``bin``, ``n_left`` and ``left`` (left class counts, or
        ``[count, sum]`` for regression).
        """
        f_hi = self.F if f_hi is None else f_hi
        h = hist.numpy()
        k = len(slots)
        C = 2 if self.reg else self.C
        out = {
            "gain": np.full(k, -np.inf),
            "feature": np.full(k, -1, dtype=np.int32),
            "bin": np.full(k, -1, dtype=np.int32),
            "n_left": np.zeros(k, dtype=np.int64),
            "left": np.zeros((k, C), dtype=np.int64),
        }
        msl = max(1, int(min_samples_leaf))
        for j, s in enumerate(slots):
            hs = h[s]
            if hs.shape[0] == 0:
                continue
            if self.reg:
                cnt = hs[..., 0]
                L = np.cumsum(cnt, axis=1)
                SL = np.cumsum(hs[..., 1], axis=1)
                m = int(L[0, -1])
                S = SL[:, -1:]
                cost = mse_term(L, SL) + mse_term(m - L, S - SL)
                pt = float(mse_term(m, int(S[0, 0])))
                mL = L
                nonempty = cnt > 0
            else:
                L = np.cumsum(hs, axis=1)
                tot = L[:, -1:, :]
                m = int(tot[0].sum())
                mL = L.sum(-1)
                if self.crit == Criterion.ENTROPY:
                    cost = entropy_term(L) + entropy_term(tot - L)
                    pt = float(entropy_term(tot[0, 0]))
                else:
                    cost = gini_term(L) + gini_term(tot - L)
                    pt = float(gini_term(tot[0, 0]))
                cost = tie_round(cost, m)
                nonempty = hs.sum(-1) > 0
            valid = nonempty & (mL >= msl) & (m - mL >= msl)
            cost = np.where(valid, cost, np.inf)
            b = np.argmin(cost, axis=1)
            fr = np.arange(cost.shape[0])
            bc = cost[fr, b]
            ok = np.isfinite(bc)
            if not ok.any():
                continue
            gain = np.where(ok, pt - bc, -np.inf)
            f = int(np.argmax(gain))
            out["gain"][j] = gain[f]
            out["feature"][j] = f + f_lo
            out["bin"][j] = b[f]
            out["n_left"][j] = mL[f, b[f]]
            if self.reg:
                out["left"][j] = (L[f, b[f]], SL[f, b[f]])
            else:
                out["left"][j] = L[f, b[f]]
        return out

    # ------------------------------------------------------------ partition
    # row permutation (level checkpoints, utils/level_checkpoint.py)
    def get_rows(self) -> np.ndarray:
        return self.idx.copy()

    def set_rows(self, rows) -> None:
        self.idx[:] = np.asarray(rows, dtype=self.idx.dtype)

    def partition(self, starts, counts, features, bins, need_counts=True):
        """Move each split node's rows so left rows come first; return local left counts."""
        nl = np.zeros(len(starts), dtype=np.int64)
        for j, (st, ct, f, b) in enumerate(zip(starts, counts, features, bins)):
            seg = self.idx[st : st + ct]
            go = self.codes[seg, f] <= b
            self.idx[st : st + ct] = np.concatenate([seg[go], seg[~go]])
            nl[j] = int(go.sum())
        return nl

    def segment_stats(self, starts, counts):
        """Per-segment class counts (or [count, sum, min, max] for regression)."""
        k = len(starts)
        if self.reg:
            out = np.zeros((k, 4), dtype=np.int64)
            # an empty (row-shard) segment must not pull the cross-rank min / max
            out[:, 2] = np.iinfo(np.int64).max
            out[:, 3] = np.iinfo(np.int64).min
            for j, (st, ct) in enumerate(zip(starts, counts)):
                yn = self.y[self.idx[st : st + ct]]
                if ct:
                    out[j] = (ct, yn.sum(), yn.min(), yn.max())
            return out
        out = np.zeros((k, self.C), dtype=np.int64)
        for j, (st, ct) in enumerate(zip(starts, counts)):
            out[j] = np.bincount(self.y[self.idx[st : st + ct]], minlength=self.C)
        return out

    # ------------------------------------------------------------- finisher
    def finisher_supported(self) -> bool:
        return True

    def finish_subtrees(self, starts, counts, depths, params, stats=None):
        """Reference (depth-first) growth of each deferred subtree.

        Same contract as the gfx950 finisher: one node table for all jobs,
        child links indexing it, ``roots[j]`` the row of job j's root.
        """
        from .reference import fit_reference

        parts = []
        for st, ct, d in zip(starts, counts, depths):
            rows = self.idx[st : st + ct]
            md = None if params.max_depth is None else int(params.max_depth) - int(d)
            ta = fit_reference(
                self.codes[rows], self.y[rows], n_classes=self.C, n_bins=self.B,
                criterion=self.crit, max_depth=md, min_samples_split=params.min_samples_split,
                min_samples_leaf=params.min_samples_leaf,
            )
            stats = (np.stack([ta.n_samples, ta.meta["sum_fixed"]], 1) if self.reg
                     else ta.count)
            parts.append(dict(feature=ta.feature, bin=ta.threshold_bin,
                              left=ta.left.astype(np.int64), right=ta.right.astype(np.int64),
                              depth=ta.depth + int(d), nsamp=ta.n_samples, stats=stats))
        lens = np.array([len(p["feature"]) for p in parts], dtype=np.int64)
        offsets = np.concatenate([[0], np.cumsum(lens)])
        for p, o in zip(parts, offsets[:-1]):
            inner = p["feature"] >= 0
            p["left"] = np.where(inner, p["left"] + o, -1)
            p["right"] = np.where(inner, p["right"] + o, -1)
        out = {k: (np.concatenate([p[k] for p in parts]) if parts else np.zeros(0, np.int64))
               for k in ("feature", "bin", "left", "right", "depth", "nsamp")}
        C = 2 if self.reg else self.C
        out["stats"] = (np.concatenate([p["stats"] for p in parts]) if parts
                        else np.zeros((0, C), np.int64))
        out["roots"] = offsets[:-1].copy()
        return out

    def sync(self):
        pass
