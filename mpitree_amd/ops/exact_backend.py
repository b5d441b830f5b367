"""Exact-threshold GPU backend for continuous features (``ops/csrc/exact.hip``).

The histogram engines are exact only while a feature has at most 256 unique
values. The reference's search (``mpitree/tree/decision_tree.py:73-90``) takes
*every* unique value as a candidate, and with ``max_bins=None`` (the default)
so does this framework: when some feature has more than 256 values the GPU
fit runs this backend under the level-wise grower
(:class:`~mpitree_amd.core.levelwise.LevelwiseBuilder`).

Layout: every feature keeps its rows sorted by value, grouped by frontier
node (``E[f][p] = rank << 32 | label << 24 | row``, uint64). A level scans
the frontier's segments -- class prefix counts at every position, the shared
integer-form cost at every value boundary -- and stably partitions the split
nodes' segments of every feature into the other list buffer. Rows that reach
a leaf are never touched again. Thresholds are the sorted unique values
(``uniq[f][rank]``), i.e. data values, exactly like ``np.unique``.

Limits: classification, fewer than 2^24 rows, at most 256 classes (the label
lives in 8 bits of each entry).
"""

from __future__ import annotations

import numpy as np
import torch

from ..core.criterion import Criterion
from . import hip_backend as hb
from .hip_backend import HipBackend, XTAB_N, unpack_records

__all__ = ["ExactHipBackend", "exact_supported", "needs_exact"]

MAX_ROWS = 1 << 24
MAX_CLASSES = 256


def exact_supported(n: int, C: int, regression: bool) -> bool:
    return (not regression) and n < MAX_ROWS and 1 <= C <= MAX_CLASSES


def needs_exact(mapper) -> bool:
    """A binned fit cannot be exact: some feature kept quantile edges."""
    ex = np.asarray(getattr(mapper, "exact", []), dtype=bool)
    return bool(ex.size) and not bool(ex.all())


class _Frontier:
    """What the grower's ``alloc_hist`` / ``build_hist`` hand to ``scan``: the
    list segments of the level's frontier slots (no histogram is stored)."""

    def __init__(self, K: int):
        self.starts = np.zeros(K, np.int64)
        self.counts = np.zeros(K, np.int64)


class ExactHipBackend(HipBackend):
    """Level-wise backend over presorted feature lists (no histograms)."""

    thresholds_on_device = True  # the unique values never leave the GPU: device assembly always

    name = "hip-exact"
    derives = False  # every frontier node is scanned from its own segment

    def setup_exact(self, X: torch.Tensor, y_codes: torch.Tensor, n_classes: int,
                    criterion: Criterion):
        n, F = X.shape
        if not exact_supported(n, n_classes, criterion == Criterion.SQUARED_ERROR):
            raise ValueError("exact GPU engine: classification with < 2^24 rows and "
                             "<= 256 classes")
        dev = self.device
        self.n, self.F, self.C = int(n), int(F), int(n_classes)
        self.crit = criterion
        self.reg = False
        self.chunk = int(self.hip.ex_chunk())
        if X.dtype == torch.float32:
            self._setup_native(X.contiguous(), y_codes)
            return
        # per feature: values sorted (stable), dense ranks, unique-value table.
        # One 1-D radix sort of 64-bit keys {feature : 32, order-preserving value
        # bits : 32} (radix sorts are stable) instead of a segmented merge sort
        # of the [F, n] matrix (12.5 -> ~3 ms for 1M x 64).
        xt = X.t().contiguous()
        if xt.dtype == torch.float32:
            xt = xt + 0.0  # -0.0 -> +0.0: equal values share one key (stable by row)
            bits = xt.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
            neg = (bits >> 31) == 1
            # IEEE order: negatives flip every bit, positives flip the sign bit
            key = torch.where(neg, bits ^ 0xFFFFFFFF, bits | 0x80000000)
            key = key | (torch.arange(F, device=dev, dtype=torch.int64)[:, None] << 32)
            _, perm = torch.sort(key.view(-1), stable=True)
            del bits, neg, key
            order = (perm.view(F, n) - torch.arange(F, device=dev, dtype=torch.int64)[:, None] * n)
            vals = torch.gather(xt, 1, order)
            del perm
        else:
            vals, order = torch.sort(xt, dim=1, stable=True)
        del xt
        new = torch.ones_like(vals, dtype=torch.bool)
        new[:, 1:] = vals[:, 1:] != vals[:, :-1]
        rank = torch.cumsum(new, 1, dtype=torch.int64) - 1
        nb = rank[:, -1] + 1
        self.B = int(nb.max())
        uniq = torch.full((F, self.B), float("inf"), dtype=torch.float64, device=dev)
        uniq.scatter_(1, rank, vals.double())
        self.uniq = uniq + 0.0  # -0.0 -> +0.0, as np.unique prints it
        self.nbins = nb.to(torch.int32)
        lab = y_codes.to(torch.int64)[order]
        e = (rank << 32) | (lab << 24) | order.to(torch.int64)
        del vals, order, rank, new, lab
        self.E = [e.contiguous(), torch.empty_like(e)]
        self.cur = 0
        self.flag = torch.empty(n, dtype=torch.uint8, device=dev)
        self.xtab = hb.xlog2x_table(dev)
        self.xtabf = hb.xlog2x_table_f32(dev)
        self.y = y_codes
        self._deferred = []
        self._loc = None

    def _setup_native(self, X: torch.Tensor, y_codes: torch.Tensor):
        """float32 input (``ops/csrc/exact_setup.hip``): feature-major keys from
        an LDS-transposed pass over X, one stable radix sort of {feature, value
        bits} keys with 32-bit row ids, then per-chunk value-change counts, a
        per-feature scan, and one pass writing the list entries and the unique
        values. The two key buffers become the two list buffers."""
        n, F, dev = self.n, self.F, self.device
        s = hb._stream()
        keys = [torch.empty((F, n), dtype=torch.int64, device=dev) for _ in range(2)]
        rows = [torch.empty((F, n), dtype=torch.int32, device=dev) for _ in range(2)]
        tb = int(self.hip.exact_setup_temp_bytes(n, F))
        temp = torch.empty(max(tb, 1), dtype=torch.uint8, device=dev)
        nc = -(-n // int(self.hip.exact_setup_chunk()))
        cnt = torch.empty((F, nc), dtype=torch.int32, device=dev)
        nuniq = torch.empty(F, dtype=torch.int32, device=dev)
        self.hip.exact_setup_sort(s, X.data_ptr(), n, F, keys[0].data_ptr(), keys[1].data_ptr(),
                                  rows[0].data_ptr(), rows[1].data_ptr(), temp.data_ptr(), tb,
                                  cnt.data_ptr(), nuniq.data_ptr())
        del temp
        self.nbins = nuniq
        self.B = int(nuniq.max())  # (one small sync: the table width)
        self.uniq = torch.full((F, self.B), float("inf"), dtype=torch.float64, device=dev)
        y32 = y_codes.to(torch.int32).contiguous()
        # entries go to keys[0] (the keys the sort consumed); keys[1] is the second list
        self.hip.exact_setup_emit(s, keys[1].data_ptr(), rows[1].data_ptr(), n, F,
                                  cnt.data_ptr(), y32.data_ptr(), self.B, keys[0].data_ptr(),
                                  self.uniq.data_ptr())
        self.E = [keys[0], keys[1]]
        del rows, cnt, y32  # (stream-ordered frees: the kernels above run first)
        self.cur = 0
        self.flag = torch.empty(n, dtype=torch.uint8, device=dev)
        self.xtab = hb.xlog2x_table(dev)
        self.xtabf = hb.xlog2x_table_f32(dev)
        self.y = y_codes
        self._deferred = []
        self._loc = None

    # the level-wise grower's histogram hooks: only the segments matter here
    def alloc_hist(self, slots: int, F_h: int | None = None):
        return _Frontier(max(int(slots), 1))

    def build_hist(self, hist, slots, starts, counts, f_lo=0, f_hi=None):
        hist.starts[np.asarray(slots)] = starts
        hist.counts[np.asarray(slots)] = counts

    def derive_hist(self, hist, prev_hist, slots, parent_slots, sibling_slots):
        raise RuntimeError("exact backend builds every node from its segment")

    def finisher_supported(self) -> bool:
        """Subtrees of <= ``max_finisher_rows`` rows continue in the histogram
        finisher on subtree-local codes (see :meth:`defer_segments`)."""
        return self.F <= 256 and self.hip.finish_feature_tile(self.F, 256, self.C) > 0

    @property
    def max_finisher_rows(self) -> int:
        return int(self.hip.ex_local_max())  # local codes are offsets < 256: one byte

    def defer_segments(self, starts, counts):
        """The level-wise grower defers these frontier segments to the finisher:
        note the list buffer holding them now (later levels only write the
        other buffer at split segments, never these positions)."""
        starts = np.asarray(starts, np.int64)
        self._deferred.append(np.stack([starts, np.asarray(counts, np.int64),
                                        np.full(starts.size, self.cur, np.int64)], 1))

    def finish_subtrees(self, starts, counts, depths, params, stats=None, positions=None):
        """Grow the deferred subtrees with the histogram finisher: per segment,
        8-bit local codes (offset of the first list entry of the row's value)
        as the finisher's row-major / feature-major code matrices over virtual
        rows (positions of feature 0's list), packed label entries as its row
        buffer; afterwards the split codes become value ranks again."""
        segs = np.concatenate(self._deferred) if self._deferred else np.zeros((0, 3), np.int64)
        self._deferred = []
        starts = np.asarray(starts, np.int64)
        if segs.shape[0] != starts.size or not np.array_equal(segs[:, 0], starts):
            raise RuntimeError("exact finisher: deferred segments out of sync with the grower")
        J = starts.size
        if J == 0:
            return None
        dev, n, F = self.device, self.n, self.F
        rb = (F + 15) // 16 * 16
        if getattr(self, "_loc", None) is None:
            self._loc = dict(
                rm=torch.empty((n, rb), dtype=torch.uint8, device=dev),
                fm=torch.empty((F, n), dtype=torch.uint8, device=dev),
                ent=torch.empty(n, dtype=torch.int32, device=dev),
                tmp=torch.empty(n, dtype=torch.int32, device=dev),
                inv=torch.empty(n, dtype=torch.int32, device=dev),
                nbins=torch.full((F,), 256, dtype=torch.int32, device=dev),
            )
        L = self._loc
        (d_seg,) = self.up(segs)
        E0, E1 = self.E[0].data_ptr(), self.E[1].data_ptr()
        self.hip.ex_local_codes(hb._stream(), E0, E1, n, d_seg.data_ptr(), J, F, rb,
                                L["rm"].data_ptr(), L["fm"].data_ptr(), L["ent"].data_ptr(),
                                L["inv"].data_ptr())
        self._seg_buf = segs[:, 2]
        # the finisher reads the binned engine's fields: point them at the local codes
        saved = {k: getattr(self, k, None) for k in
                 ("codes_rm", "codes_fm", "idx", "tmp", "lab_shift", "nbins", "B", "row_elems",
                  "cb", "y")}
        self.codes_rm, self.codes_fm = L["rm"], L["fm"]
        self.idx, self.tmp = L["ent"], L["tmp"]
        self.lab_shift, self.nbins, self.B, self.row_elems, self.cb = 24, L["nbins"], 256, rb, 1
        try:
            return self._finish_subtrees(starts, counts, depths, params, stats, positions)
        finally:
            for k, v in saved.items():
                setattr(self, k, v)

    def _after_finisher(self, rec, starts, counts, positions):
        jobs = np.stack([np.asarray(positions, np.int64), np.asarray(counts, np.int64),
                         np.asarray(starts, np.int64), self._seg_buf], 1)
        (d_jobs,) = self.up(jobs)
        self.hip.ex_local_fix(hb._stream(), self.E[0].data_ptr(), self.E[1].data_ptr(), self.n,
                              d_jobs.data_ptr(), jobs.shape[0], rec.data_ptr())
        self._keep_fix = d_jobs

    def _chunks(self, starts, counts):
        """Chunk items {id, segment start, chunk start, chunk count} + first item per id."""
        ch = self.chunk
        k = np.maximum(1, -(-counts // ch))
        ids = np.repeat(np.arange(counts.size), k)
        first = np.concatenate([[0], np.cumsum(k)])
        off = (np.arange(ids.size) - first[:-1][ids]) * ch
        items = np.stack([ids, starts[ids], starts[ids] + off,
                          np.maximum(0, np.minimum(ch, counts[ids] - off))], 1)
        return items, first

    def scan(self, hist, slots, min_samples_leaf=1, f_lo=0, f_hi=None):
        slots = np.asarray(slots, np.int64)
        K = slots.size
        starts, counts = hist.starts[slots], hist.counts[slots]
        items, first = self._chunks(starts, counts)
        NI = items.shape[0]
        F, C = self.F, self.C
        d_items, d_first, d_seg = self.up(items, first, np.stack([starts, counts], 1))
        dev = self.device
        tot = torch.empty((NI, F, C), dtype=torch.int32, device=dev)
        carry = torch.empty_like(tot)
        slot_tot = torch.empty((K, C), dtype=torch.int32, device=dev)
        best = torch.empty((K, F), dtype=torch.int64, device=dev)
        rec = torch.empty((K, 5 + 2 * C), dtype=torch.int64, device=dev)
        self.hip.ex_scan_level(hb._stream(), self.E[self.cur].data_ptr(), self.n,
                               d_items.data_ptr(), NI, d_first.data_ptr(), d_seg.data_ptr(), K,
                               F, C, int(self.crit), int(max(1, min_samples_leaf)),
                               self.xtab.data_ptr(), XTAB_N, tot.data_ptr(), carry.data_ptr(),
                               slot_tot.data_ptr(), best.data_ptr(), rec.data_ptr())
        self.last_rec = rec
        return unpack_records(rec.cpu().numpy(), C, False)

    def partition(self, starts, counts, features, bins, need_counts=True):
        S = len(starts)
        if S == 0:
            return np.zeros(0, dtype=np.int64)
        starts = np.asarray(starts, np.int64)
        counts = np.asarray(counts, np.int64)
        split = np.stack([starts, counts, np.asarray(features, np.int64),
                          np.asarray(bins, np.int64)], 1)
        pitems, pfirst = self._chunks(starts, counts)
        NP = pitems.shape[0]
        d_items, d_first, d_split = self.up(pitems, pfirst, split)
        dev = self.device
        lc = torch.empty((NP, self.F), dtype=torch.int32, device=dev)
        lcar = torch.empty_like(lc)
        nl = torch.empty(S, dtype=torch.int32, device=dev)
        # the scatter's left flags, one ballot word per 64 entries (pcount -> pscatter)
        bits = torch.empty((NP, self.F, int(self.hip.ex_part_bits_words())), dtype=torch.int64,
                           device=dev)
        src, dst = self.E[self.cur], self.E[1 - self.cur]
        self.hip.ex_partition_level(hb._stream(), src.data_ptr(), dst.data_ptr(), self.n,
                                    d_items.data_ptr(), NP, d_first.data_ptr(),
                                    d_split.data_ptr(), S, self.F, self.flag.data_ptr(),
                                    lc.data_ptr(), lcar.data_ptr(), nl.data_ptr(),
                                    bits.data_ptr())
        self.cur = 1 - self.cur  # every next-level node lives in the list just written
        self._keep_p = (d_items, d_first, d_split, lc, lcar, bits)
        if not need_counts:
            self._keep_nl = nl
            return None
        return nl.cpu().numpy().astype(np.int64)

    def segment_stats(self, starts, counts):
        e0 = self.E[self.cur][0]
        out = np.zeros((len(starts), self.C), dtype=np.int64)
        for j, (s, c) in enumerate(zip(np.asarray(starts), np.asarray(counts))):
            lab = ((e0[int(s): int(s) + int(c)] >> 24) & 0xFF)
            out[j] = torch.bincount(lab, minlength=self.C).cpu().numpy()[: self.C]
        return out

    def get_rows(self):  # pragma: no cover - level checkpoints use the binned engines
        raise RuntimeError("level checkpoints are not supported by the exact engine")

    def assemble_positions(self, edges, crit: int, y_exp: int = 0, d_edges=None) -> dict:
        # thresholds straight from the device unique-value table (rank -> value)
        return super().assemble_positions(None, crit, y_exp, d_edges=self.uniq)
