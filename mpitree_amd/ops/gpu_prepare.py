"""Device-side fit preparation: binning plus label / target encoding.

The reference prepares a fit on the host of every rank (``np.unique`` class
discovery, ``mpitree/tree/decision_tree.py:418-421``; no binning -- it scans
raw values). Here a fit on the GPU needs, before the first tree level:

* the feature bin edges, codes and verification flags (``DeviceBinning``),
* the class list and int32 label codes (or the fixed-point regression
  targets and their exponent),
* the root node's statistics (class counts, or {count, sum, min, max}).

Every host decision among these needs a small device read; issued one by one
they cost ~6 synchronisations with host work in between, during which the
GPU idles. :func:`prepare` batches them: with at most 256 bins the bin
kernel is enqueued right behind the edges kernel (it reads the bin counts on
the device), and the class counts are taken speculatively over [0, 8192) with
an out-of-range tally, so a classification fit on integer labels needs ONE
synchronisation (edge table, bin flags and class counts in one wait). Labels
outside the guess, more than 256 bins and regression targets (whose
fixed-point exponent depends on max |y|) take a second one. The root
statistics come for free and the device level loop starts without another
round trip.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import native
from .hip_backend import (DeviceBinning, _d2h, _event, _pinned_copy, _pinned_host, _stream,
                          _uploader, _ws_tensor)

__all__ = ["Prepared", "prepare"]

_LUT_MAX = 1 << 22  # label ranges beyond this fall back to torch.unique
_SPEC_R = 8192  # guessed label range [0, _SPEC_R) (the count kernel's LDS histogram)


@dataclass
class Prepared:
    mapper: object
    codes_rm: torch.Tensor
    codes_fm: torch.Tensor
    nbins: torch.Tensor
    y: torch.Tensor  # int32 class codes or int64 fixed-point targets (device)
    classes: np.ndarray | None
    y_exp: int
    root: np.ndarray | None  # root statistics when known without another sync
    d_edges64: torch.Tensor | None  # device fp64 edge table [F, W] (None: use host edges)
    # deferred bin verification (None: already checked): call once the stream has
    # passed the bin kernel; False means the fit must be redone with sync=True
    verify: object = None
    # prepare(split=True): the labels are ready, the edge table is not -- call
    # once before reading mapper / d_edges64 / verify (waits for the edges kernel)
    resolve: object = None


_NP_DT: dict = {}


def _np_dtype(dt: torch.dtype):
    v = _NP_DT.get(dt)
    if v is None:
        v = _NP_DT[dt] = torch.empty(0, dtype=dt).numpy().dtype
    return v


class _Labels:
    """Classification labels: device int tensors take the two-sync path."""

    def __init__(self, y, n, dev, encode_fallback):
        self.y, self.n, self.dev = y, n, dev
        self.fallback = encode_fallback
        self.dev_path = (
            torch.is_tensor(y) and y.is_cuda and y.dim() == 1 and y.shape[0] == n and n > 0
            and not torch.is_floating_point(y) and y.dtype != torch.bool
        )
        self._counts = None
        if self.dev_path:
            self.yl = y if (y.dtype == torch.int64 and y.is_contiguous()) else \
                y.long().contiguous()
            # speculate that the labels lie in [0, _SPEC_R): the counts (and an
            # out-of-range tally) then arrive with the fit's first sync; the same
            # pass writes the int32 codes, valid when the labels are 0..C-1
            self.spec = _ws_tensor(dev, "lab.spec", (_SPEC_R + 1,), torch.int32)
            self.enc0 = _ws_tensor(dev, "lab.enc", (n,), torch.int32)
            native.hip().label_count(_stream(), self.yl.data_ptr(), n, 0, _SPEC_R,
                                     self.spec.data_ptr(), True, self.enc0.data_ptr())
            self._spec, hp = _pinned_host("prep.lab.spec", _SPEC_R + 1, np.int32)
            _d2h(hp, self.spec)

    def after_first_sync(self) -> bool:
        """True when the labels need another device round (outside the guess)."""
        if not self.dev_path:
            return False
        if int(self._spec[_SPEC_R]) == 0:
            self.lo, self.R = 0, _SPEC_R
            self._counts = self._spec[:_SPEC_R]
            return False
        self.enc0 = None
        mm = torch.stack(torch.aminmax(self.yl)).cpu().numpy()  # one extra sync
        lo, hi = int(mm[0]), int(mm[1])
        R = hi - lo + 1
        if R > _LUT_MAX:
            self.dev_path = False
            return False
        self.lo, self.R = lo, R
        self.counts = torch.empty(R, dtype=torch.int32, device=self.dev)
        native.hip().label_count(_stream(), self.yl.data_ptr(), self.n, lo, R,
                                 self.counts.data_ptr())
        self._counts = _pinned_copy(self.counts, "prep.lab.counts")
        return True

    def finish(self):
        """(classes, int32 device codes, root class counts)."""
        if not self.dev_path:
            classes, enc = self.fallback(self.y, self.n)
            if torch.is_tensor(enc):
                return classes, enc.to(self.dev).to(torch.int32).contiguous(), None
            root = np.bincount(enc, minlength=len(classes)).astype(np.int64)
            d = torch.from_numpy(np.ascontiguousarray(enc, np.int32)).to(self.dev)
            return classes, d, root
        counts = self._counts
        idx = np.flatnonzero(counts)
        classes = (idx + self.lo).astype(_np_dtype(self.y.dtype))
        last = int(idx[-1]) if idx.size else -1
        if self.lo == 0 and last + 1 == idx.size and self.enc0 is not None:
            enc = self.enc0
        elif self.lo == 0 and idx.size == counts.size:
            enc = self.yl.to(torch.int32)
        else:
            present = counts > 0
            (d_lut,) = _uploader(self.dev)(np.cumsum(present) - 1)
            enc = torch.empty(self.n, dtype=torch.int32, device=self.dev)
            native.hip().label_encode(_stream(), self.yl.data_ptr(), self.n, self.lo,
                                      d_lut.data_ptr(), enc.data_ptr())
        return classes, enc, counts[idx].astype(np.int64)


class _Targets:
    """Regression targets as fixed-point int64 (exponent chosen from max |y|).

    fp32 / fp64 device targets: two kernels (``misc.hip`` target_stats /
    target_encode) find max |y|, pick the exponent on the device, encode and
    reduce the root {sum, min, max}, all enqueued ahead of the binning -- the
    host reads the result with the binning's first wait (no second sync)."""

    def __init__(self, y, n, dev, encode_fallback, exponent):
        self.y, self.n, self.dev = y, n, dev
        self.fallback, self.exponent = encode_fallback, exponent
        self.dev_path = torch.is_tensor(y) and y.is_cuda and y.dim() == 1 and y.shape[0] == n
        self.fused = False
        if self.dev_path and n > 0:
            if y.dtype in (torch.float32, torch.float64) and y.is_contiguous():
                self.fused = True
                st = torch.empty(8, dtype=torch.int64, device=dev)
                self.yi = torch.empty(n, dtype=torch.int64, device=dev)
                native.hip().targets(_stream(), y.data_ptr(), y.dtype == torch.float64, n,
                                     st.data_ptr(), self.yi.data_ptr())
                self._st = _pinned_copy(st, "prep.reg.fused")
                return
            self.yd = y.double()
            st = torch.stack([self.yd.abs().max(), torch.isfinite(self.yd).all().double()])
            self._st = _pinned_copy(st, "prep.reg.st")
        elif self.dev_path:
            self.dev_path = False

    def after_first_sync(self) -> bool:
        """True: the fixed-point targets need another sync (the unfused device path)."""
        if not self.dev_path:
            return False
        if self.fused:
            st = np.array(self._st, dtype=np.int64)
            if st[1]:
                raise ValueError("Input y contains NaN or infinity.")
            self.e = int(st[2])
            self._root = st[3:6].copy()
            return False
        if not self._st[1]:
            raise ValueError("Input y contains NaN or infinity.")
        self.e = self.exponent(float(self._st[0]), self.n)
        scale = torch.tensor(float(self.e), dtype=torch.float64, device=self.dev)
        self.yi = torch.round(torch.ldexp(self.yd, scale)).long()
        mn, mx = torch.aminmax(self.yi)
        self._root = _pinned_copy(torch.stack([self.yi.sum(), mn, mx]), "prep.reg.root")
        return True

    def finish(self):
        """(int64 device targets, exponent, root {count, sum, min, max})."""
        if not self.dev_path:
            yi, e = self.fallback(self.y, self.n)
            if torch.is_tensor(yi):
                return yi.to(self.dev).contiguous(), e, None
            root = None
            if yi.size:
                root = np.array([yi.size, int(yi.sum()), int(yi.min()), int(yi.max())], np.int64)
            return torch.from_numpy(np.ascontiguousarray(yi)).to(self.dev), e, root
        r = np.array(self._root, dtype=np.int64)
        return self.yi.contiguous(), self.e, np.array([self.n, r[0], r[1], r[2]], np.int64)


def prepare(Xd: torch.Tensor, y, *, regression: bool, max_bins, encode_labels,
            encode_targets, exponent, sync: bool = False, exact_probe: bool = False,
            rows=None, agree=None, split: bool = False) -> Prepared:
    """Bin ``Xd`` (device, fp32/fp64) and encode ``y`` with two host syncs.

    ``encode_labels`` / ``encode_targets`` are the host encoders of
    ``core/fit.py``, used for host arrays and unusual label dtypes.

    With at most 256 bins the first sync waits only for the edge table and the
    label counts: the bin kernel (~0.1 ms on 1M x 64) keeps running while the
    host builds its tables and enqueues the level loop. Its codes are always
    valid bins (clamped), so nothing downstream depends on its verification
    flags until the tree is assembled; ``Prepared.verify`` checks them then
    (non-finite input raises, an exact-mode sample that missed a value asks
    for a redo with ``sync=True``, which checks before growing).

    ``exact_probe`` (exact-threshold requests): features past ``max_bins`` values
    get no quantile edges and, when any feature has them, the bin pass writes no
    codes (``DeviceBinning``); such a result is only for the presorted-list engine.

    ``rows`` = (lo, hi): codes for that row range only (a data-parallel rank's
    shard of a replicated input; edges, labels and targets still cover every
    row, so every rank derives the same tables). ``agree``: combines the bin
    flags over the ranks (checked before growth, as with ``sync``).

    ``split`` (<= 256 bins, no ``sync``): the label / target pass runs first and
    the host waits for it alone; the returned ``Prepared`` has no mapper yet and
    ``resolve()`` waits for the edge table later -- so the caller's label-dependent
    setup (buffers, the row permutation) overlaps the edges and bin kernels
    instead of following them.
    """
    n = Xd.shape[0]
    dev = Xd.device
    stream = torch.cuda.current_stream(dev)
    if split and agree is None and not sync and (max_bins or 0) <= 256:
        return _prepare_split(Xd, y, regression, max_bins, encode_labels, encode_targets,
                              exponent, exact_probe, rows, stream)
    # the edges kernel first: the label / target kernels and their host-side
    # setup (~40 us of host time) then overlap it instead of delaying it. (A side
    # stream for the label pass, so the bin kernel could follow the edges at
    # once, measured 0.35 ms slower per flagship fit.)
    if agree is not None:
        sync = True  # the ranks' flags are combined before any rank grows
    binning = DeviceBinning(Xd, max_bins, probe=exact_probe, rows=rows, agree=agree)
    lab = (_Targets(y, n, dev, encode_targets, exponent) if regression
           else _Labels(y, n, dev, encode_labels))
    early = binning.early
    if early:  # <= 256 bins: the bin kernel reads the bin counts on the device
        tables = _event(dev, "prep.tables")
        tables.record(stream)  # edge table + label count copies are enqueued before it
        binning.launch_bin_early()
        if sync:
            stream.synchronize()  # sync 1 covers the bin flags too
        else:
            tables.synchronize()  # sync 1: edge table + label counts / target scale
    else:
        stream.synchronize()  # sync 1: edge table + label counts / target scale
    need2 = lab.after_first_sync()
    binning.launch_bin()  # host tables; enqueues the bin kernel unless already done
    deferred = early and not sync
    if need2 or not early:
        stream.synchronize()  # sync 2: bin flags / class counts / target root stats
        deferred = False
    mapper, codes_rm, codes_fm, nb = binning.finish(check=not deferred)
    if regression:
        yenc, y_exp, root = lab.finish()
        classes = None
    else:
        classes, yenc, root = lab.finish()
        y_exp = 0
    return Prepared(mapper=mapper, codes_rm=codes_rm, codes_fm=codes_fm, nbins=nb, y=yenc,
                    classes=classes, y_exp=y_exp, root=root, d_edges64=binning.d_edges64,
                    verify=binning.verify if deferred else None)


def _prepare_split(Xd, y, regression, max_bins, encode_labels, encode_targets, exponent,
                   exact_probe, rows, stream) -> Prepared:
    """``prepare(split=True)``: labels -> edges -> bin on the stream, one host
    wait for the labels; the edge table is read in ``Prepared.resolve``."""
    n = Xd.shape[0]
    dev = Xd.device
    lab = (_Targets(y, n, dev, encode_targets, exponent) if regression
           else _Labels(y, n, dev, encode_labels))
    lab_ev = _event(dev, "prep.labels")
    lab_ev.record(stream)
    binning = DeviceBinning(Xd, max_bins, probe=exact_probe, rows=rows)
    tables = _event(dev, "prep.tables")
    tables.record(stream)
    binning.launch_bin_early()
    lab_ev.synchronize()  # the one early wait: label counts / target scale
    if lab.after_first_sync():  # (labels outside the guess: another device round)
        stream.synchronize()
    if regression:
        yenc, y_exp, root = lab.finish()
        classes = None
    else:
        classes, yenc, root = lab.finish()
        y_exp = 0
    prep = Prepared(mapper=None, codes_rm=binning.codes_rm, codes_fm=binning.codes_fm,
                    nbins=binning.nb, y=yenc, classes=classes, y_exp=y_exp, root=root,
                    d_edges64=None)

    def resolve():
        tables.synchronize()  # (the edges kernel ran while the caller set up)
        binning.launch_bin()  # host tables (the bin kernel is enqueued already)
        prep.mapper = binning.finish(check=False)[0]
        prep.d_edges64 = binning.d_edges64
        prep.verify = binning.verify
        prep.resolve = None

    prep.resolve = resolve
    return prep


def prepare_with_mapper(Xd: torch.Tensor, y_enc, mapper, classes, y_exp: int) -> Prepared:
    """Bin ``Xd`` with a given (globally agreed) ``BinMapper`` and upload the
    already-encoded targets ``y_enc`` (int32 class codes / int64 fixed-point).
    Used by row-sharded data-parallel fits (``parallel/agreement.py``)."""
    dev = Xd.device
    hip = native.hip()
    F = Xd.shape[1]
    table = mapper.padded_edges(np.float64)
    W = table.shape[1]
    edges = torch.from_numpy(table).to(dev)
    edges_x = edges.to(Xd.dtype).contiguous()
    nb = torch.from_numpy(mapper.n_bins.astype(np.int32)).to(dev)
    exact = torch.from_numpy(np.asarray(mapper.exact, np.uint8)).to(dev)
    job = DeviceBinning.__new__(DeviceBinning)  # the bin pass alone (no edges kernel)
    job.hip, job.X, job.dev = hip, Xd, dev
    job.n, job.F = Xd.shape
    job.lo, job.hi = 0, job.n  # (every row of this rank's shard)
    job.x64 = Xd.dtype == torch.float64
    job._codes = None
    codes_rm, codes_fm, flags = job._run_bin(edges_x, nb, exact, max(1, W))
    if (flags.cpu().numpy() & 2).any():
        raise ValueError("Input X contains NaN or infinity.")
    yd = torch.as_tensor(np.ascontiguousarray(y_enc)).to(dev)
    del F
    return Prepared(mapper=mapper, codes_rm=codes_rm, codes_fm=codes_fm, nbins=nb, y=yd,
                    classes=classes, y_exp=int(y_exp), root=None, d_edges64=edges)
