"""gfx950 backend of the level-wise engine: device buffers + kernel launches.

Implements the same operations as :class:`mpitree_amd.core.backend_numpy.NumpyBackend`
with the HIP kernels in ``ops/csrc``. Device data (row-major and
feature-major codes, labels, the row permutation) stays resident in HBM for
the whole fit; per level the host only uploads a small work plan and reads
back one record per frontier node.
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

from ..core.binning import MAX_BINS_LIMIT, BinMapper, TableBinMapper
from ..core.criterion import Criterion
from ..models.tree_arrays import TreeArrays
from . import native

__all__ = ["HipBackend", "gpu_bin_features"]

LDS_BUDGET = int(os.environ.get("MPITREE_HIST_LDS", 80 * 1024))
MAX_ITEM_ROWS = 65535  # 16-bit packed LDS counters
N_CU = 256  # MI355X compute units


def _tiny_batch(hip) -> int:
    """Tiny-subtree records a finisher workgroup reserves at a time (grow.h
    kFinTinyBatch; 1 for an extension built before the batched reservation)."""
    f = getattr(hip, "fin_tiny_batch", None)
    return int(f()) if f is not None else 1


_EDGE_ROWS: dict = {}  # x64 -> rows the edges kernel samples (asked once)
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_dev = getattr(torch._C, "_cuda_getDevice", None)


def _stream() -> int:
    """The current HIP stream handle (every launch passes it). The raw
    accessors skip ``torch.cuda.current_stream``'s device-index resolution,
    ~3 us of host time per call x ~90 launches per fit."""
    if _raw_stream is not None and _cur_dev is not None:
        return _raw_stream(_cur_dev())
    return torch.cuda.current_stream().cuda_stream


class _Uploader:
    """Pack several small int64 host arrays into one asynchronous pinned H2D copy.

    A ring of pinned staging buffers, each guarded by the event recorded after
    its copy, lets the host prepare the next plan while earlier copies are in
    flight without ever overwriting a buffer the DMA engine still reads.
    """

    RING = 8

    def __init__(self, device):
        self.device = device
        self._bufs = [torch.empty(256, dtype=torch.int64).pin_memory() for _ in range(self.RING)]
        self._events = [None] * self.RING
        self._i = 0

    def __call__(self, *arrays):
        arrays = [np.asarray(a, dtype=np.int64).ravel() for a in arrays]
        sizes = [a.size for a in arrays]
        total = max(1, sum(sizes))
        i = self._i
        self._i = (i + 1) % self.RING
        if self._events[i] is not None:
            self._events[i].synchronize()
        if self._bufs[i].numel() < total:
            self._bufs[i] = torch.empty(max(total, 2 * self._bufs[i].numel()),
                                        dtype=torch.int64).pin_memory()
        buf = self._bufs[i].numpy()
        o = 0
        for a, s in zip(arrays, sizes):
            buf[o : o + s] = a
            o += s
        dev = self._bufs[i][:total].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._events[i] = ev
        outs, o = [], 0
        for s in sizes:
            outs.append(dev[o : o + s])
            o += s
        return outs


_workspaces: dict = {}


def _workspace(device, name: str, nbytes: int) -> torch.Tensor:
    """A reusable uint8 device scratch buffer per (device, name), grown
    geometrically: steady-state fits of one shape allocate nothing. Reuse is
    safe because every user enqueues on the one current stream."""
    key = (str(device), name)
    buf = _workspaces.get(key)
    if buf is None or buf.numel() < nbytes:
        cap = max(int(nbytes), int(1.25 * buf.numel()) if buf is not None else 0, 256)
        cap = (cap + 255) // 256 * 256  # (any typed view of a full buffer stays aligned)
        buf = _workspaces[key] = torch.empty(cap, dtype=torch.uint8, device=device)
    return buf


def _i64_scratch(device, name: str, rows: int, cols: int) -> torch.Tensor:
    """An int64 [rows, cols] view of a reused scratch buffer (uninitialised; the
    finisher's record lists: allocating them per launch cost host time right
    where the GPU waits for the finisher's launch)."""
    nb = int(rows) * int(cols) * 8
    return _workspace(device, name, nb)[:nb].view(torch.int64).view(int(rows), int(cols))


_uploaders: dict = {}


def _uploader(device) -> _Uploader:
    """One staging ring per device, shared by every fit (pinned allocations
    are expensive; the ring's events keep reuse safe)."""
    key = str(device)
    u = _uploaders.get(key)
    if u is None:
        u = _uploaders[key] = _Uploader(device)
    return u


class DeviceBinning:
    """Bin a device feature matrix in three host steps around two syncs.

    ``__init__`` enqueues the edges kernel (binning.hip ``edges_kernel``: a
    deterministic strided row sample per feature, exact mode when the sample
    has at most ``max_bins`` distinct values) and one D2H of the packed edge
    table. After the caller synchronises, :meth:`launch_bin` enqueues the bin
    kernel and the D2H of its flags, and builds the host ``BinMapper`` while
    the kernel runs. After the next sync :meth:`finish` rejects non-finite
    input and, when an exact-mode sample missed a value, re-bins the affected
    features from their full columns. Callers batch their own small reads
    into the same two syncs (``core/fit.py``); :func:`gpu_bin_features` is
    the stand-alone form.
    """

    def __init__(self, X: torch.Tensor, max_bins=256, sample_rows: int | None = None,
                 probe: bool = False, rows=None, agree=None):
        hip = self.hip = native.hip()
        # rows = (lo, hi): the edges come from every row of X (a replicated input:
        # every rank derives the same table), the codes only for rows [lo, hi) --
        # a data-parallel rank bins its own shard. agree(flags) -> the flags of
        # every rank combined (max), so all ranks take the same refit / error path.
        self.lo, self.hi = (0, int(X.shape[0])) if rows is None else (int(rows[0]), int(rows[1]))
        self.agree = agree
        # probe (exact-threshold requests): a feature whose sample exceeds the limit
        # is only marked inexact (no quantile edges), and the early bin pass then
        # only checks for non-finite values -- the fit goes to the presorted-list
        # engine, which reads neither
        self.probe = bool(probe)
        self.X = X
        n, F = self.n, self.F = X.shape
        dev = self.dev = X.device
        self.x64 = X.dtype == torch.float64
        self.limit = MAX_BINS_LIMIT if max_bins is None else int(max_bins)
        er = _EDGE_ROWS.get(self.x64)
        if er is None:
            er = _EDGE_ROWS[self.x64] = int(hip.edges_sample_rows(self.x64))
        s = min(n, int(sample_rows or er))
        L = self.limit
        # (setup buffers reused across fits of one shape: see _ws_tensor)
        self.edges = _ws_tensor(dev, "bin.edges", (F, L), X.dtype)
        self.nb = _ws_tensor(dev, "bin.nb", (F,), torch.int32)
        self.exact = _ws_tensor(dev, "bin.exact", (F,), torch.uint8)
        # fp64 [F*L edges | F counts | F exact flags]: the host's copy in one D2H
        self.pack = _ws_tensor(dev, "bin.pack", (F * L + 2 * F,), torch.float64)
        hip.edges(_stream(), X.data_ptr(), self.x64, n, F, s, L, self.edges.data_ptr(),
                  self.nb.data_ptr(), self.exact.data_ptr(), self.pack.data_ptr(), self.probe)
        self._host_pack, hp = _pinned_host("bin.pack", F * L + 2 * F, np.float64)
        _d2h(hp, self.pack)
        # the code buffers' shapes are known up front for <= 256 bins
        self._codes = self._alloc_codes(1) if L <= 256 else None

    def _alloc_codes(self, cb):
        n, F = self.hi - self.lo, self.F
        ctype = torch.uint8 if cb == 1 else torch.int16
        row_elems = ((F * cb + 3) // 4) * 4 // cb
        codes_rm = _ws_tensor(self.dev, "bin.codes_rm", (n, row_elems), ctype)
        codes_fm = _ws_tensor(self.dev, "bin.codes_fm", (F, n), ctype)
        flags = _ws_tensor(self.dev, "bin.flags", (self.F,), torch.int32)
        flags.zero_()
        return cb, row_elems, codes_rm, codes_fm, flags

    def _run_bin(self, edges_t, nb_t, exact_t, bmax, skip_inexact=False):
        cb = 1 if bmax <= 256 else 2
        if self._codes is None or self._codes[0] != cb:
            self._codes = self._alloc_codes(cb)
        cb, row_elems, codes_rm, codes_fm, flags = self._codes
        self._codes = None  # buffers belong to this pass
        # (a row range of the contiguous row-major input is contiguous too)
        x_ptr = self.X.data_ptr() + self.lo * self.F * self.X.element_size()
        self.hip.bin(_stream(), x_ptr, self.x64, self.hi - self.lo, self.F, edges_t.data_ptr(),
                     bmax, nb_t.data_ptr(), exact_t.data_ptr(), codes_rm.data_ptr(), row_elems,
                     codes_fm.data_ptr(), cb, flags.data_ptr(), estride=int(edges_t.stride(0)),
                     skip_inexact=skip_inexact)
        return codes_rm, codes_fm, flags

    @property
    def early(self) -> bool:
        """At most 256 bins: one code byte whatever the per-feature counts, so
        the bin kernel can be enqueued before the edge table reaches the host."""
        return self.limit <= 256

    def launch_bin_early(self):
        """Enqueue the bin kernel straight after the edges kernel (``early``):
        it reads the bin counts from the device, so the fit's first sync covers
        edges, codes and flags together."""
        self.codes_rm, self.codes_fm, flags = self._run_bin(self.edges, self.nb, self.exact,
                                                            self.limit, skip_inexact=self.probe)
        self._host_flags, hp = _pinned_host("bin.flags", self.F, np.int32)
        _d2h(hp, flags)
        self._flags_ready = _event(self.dev, "bin.flags")
        self._flags_ready.record(torch.cuda.current_stream(self.dev))
        self._launched = True

    def host_tables(self):
        """Host edge table and ``BinMapper`` (after a sync covering ``__init__``'s copy).
        The table stays a view of the pinned buffer until the level loop runs (its
        private copy is deferred work: the next fit reuses the buffer)."""
        F, L = self.F, self.limit
        host = self._host_pack
        self.host_edges = host[: F * L].reshape(F, L)
        self.host_nb = host[F * L : F * L + F].astype(np.int64)
        self.host_exact = host[F * L + F :].astype(bool)
        self.bmax = int(max(1, self.host_nb.max())) if F else 1
        self.mapper = TableBinMapper(self.host_edges, self.host_nb, self.host_exact.copy(), L)
        defer(self.mapper.own_table)

    def launch_bin(self):
        """Enqueue the bin kernel (after a sync covering ``__init__``'s copy)."""
        self.host_tables()
        if not getattr(self, "_launched", False):
            self.codes_rm, self.codes_fm, flags = self._run_bin(self.edges, self.nb, self.exact,
                                                                self.bmax, skip_inexact=self.probe)
            self._host_flags = _pinned_copy(flags, "bin.flags")
            self._launched = True

    def finish(self, check: bool = True):
        """(mapper, codes_rm, codes_fm, nbins_dev) after a sync covering the flags copy
        (``check=False``: before it; :meth:`verify` then checks the flags later)."""
        missed = False
        if check:
            fl = np.array(self._host_flags)
            if self.agree is not None:
                fl = np.asarray(self.agree(fl.astype(np.int64)), dtype=np.int64)
            if (fl & 2).any():
                raise ValueError("Input X contains NaN or infinity.")
            missed = bool((fl & 1).any())
            if missed:
                self._refit_missed(np.nonzero(fl & 1)[0])
        self.d_edges64 = None if missed else self.pack[: self.F * self.limit].view(
            self.F, self.limit)
        return self.mapper, self.codes_rm, self.codes_fm, self.nb

    def verify(self) -> bool:
        """Deferred flag check of an early bin pass whose result is already in use:
        raises on non-finite input; False when an exact-mode sample missed a value
        (the codes were clamped to the sampled edges: the fit must be redone)."""
        self._flags_ready.synchronize()
        fl = np.array(self._host_flags)
        if self.agree is not None:
            fl = np.asarray(self.agree(fl.astype(np.int64)), dtype=np.int64)
        if (fl & 2).any():
            raise ValueError("Input X contains NaN or infinity.")
        return not bool((fl & 1).any())

    def _refit_missed(self, feats):
        """The sample missed values of an "exact" feature: use the full column."""
        X, dev, n, limit = self.X, self.dev, self.n, self.limit
        edges, host_edges = self.edges, self.host_edges
        host_nb, host_exact = self.host_nb, self.host_exact
        for f in feats:
            col = X[:, f]
            u = torch.unique(torch.where(col == 0, torch.zeros_like(col), col))
            if u.numel() <= limit:
                e = u
                host_exact[f] = True
            else:
                srtc = torch.sort(col).values
                k = torch.arange(1, limit + 1, device=dev, dtype=torch.int64)
                qi = torch.clamp((k * n + limit - 1) // limit - 1, max=n - 1)
                e = torch.unique(srtc[qi])
                host_exact[f] = False
            if e.numel() > edges.shape[1]:
                wider = torch.full((self.F, e.numel()), float("inf"), dtype=X.dtype, device=dev)
                wider[:, : edges.shape[1]] = edges
                edges = wider
                host_edges = np.concatenate(
                    [host_edges, np.full((self.F, e.numel() - host_edges.shape[1]), np.inf)], 1)
            edges[f].fill_(float("inf"))
            edges[f, : e.numel()] = e
            host_edges[f] = np.inf
            host_edges[f, : e.numel()] = e.double().cpu().numpy()
            host_nb[f] = e.numel()
        self.nb = torch.from_numpy(host_nb.astype(np.int32)).to(dev)
        exact = torch.from_numpy(host_exact.astype(np.uint8)).to(dev)
        bmax = int(max(1, host_nb.max()))
        self.codes_rm, self.codes_fm, flags = self._run_bin(edges, self.nb, exact, bmax)
        if (flags.cpu().numpy() & 2).any():  # pragma: no cover - caught by the first pass
            raise ValueError("Input X contains NaN or infinity.")
        self.mapper = BinMapper(
            edges=[host_edges[f, : host_nb[f]].copy() for f in range(self.F)],
            exact=host_exact.astype(bool),
            max_bins=limit,
        )


def gpu_bin_features(X: torch.Tensor, max_bins=256, sample_rows: int | None = None):
    """Bin a device feature matrix; returns (BinMapper, codes_rm, codes_fm, nbins_dev).

    Stand-alone form of :class:`DeviceBinning` (two host synchronisations:
    the packed edge table and the bin kernel's verification flags).
    """
    job = DeviceBinning(X, max_bins, sample_rows)
    torch.cuda.current_stream(X.device).synchronize()
    job.launch_bin()
    torch.cuda.current_stream(X.device).synchronize()
    return job.finish()


XTAB_N = 1 << 16
_xtab_cache: dict = {}


def xlog2x_table(device, min_n: int = XTAB_N) -> torch.Tensor:
    """Device table of x*log2(x) for x < max(2^16, min_n), built by the same
    device function the kernels would otherwise evaluate (identical bits) and
    kept per device; a request for more entries rebuilds it larger (powers of
    two). Kernels bound their lookups by the xtab_n they are given, so a larger
    table serves every caller (the exact engine asks for n + 1 entries: every
    count of a node is a table read)."""
    key = str(device)
    t = _xtab_cache.get(key)
    if t is None or t.numel() < min_n:
        size = XTAB_N
        while size < min_n:
            size *= 2
        t = torch.empty(size, dtype=torch.float64, device=device)
        native.hip().xlog2x_device(_stream(), t.data_ptr(), size)
        _xtab_cache[key] = t
        _xtab_cache.pop("f32:" + key, None)
    return t


_pinned: dict = {}
_ASM_HINT: dict = {}  # (device, positions, C, reg, thresholds) -> last assembled node count


_TASK_FLAGS: dict = {}  # device -> [int32 flag tensor, epoch]
_REG_PER_CU: dict = {}  # (bins, code bytes) -> regression finisher workgroups per CU
_FIN_WATCH: list = []  # pinned views of finisher watchdog words, checked at assembly


def _tiny_order(device, cap: int, on: bool) -> int:
    """Scratch for the tiny-subtree kernels' largest-first order ([2 * 65] bucket
    counts, then ``cap`` record indices), or 0: the records in discovery order.
    ``on``: regression and many classes by default (``MPITREE_TINY_LPT`` = 1 / 0
    forces it): their subtrees keep splitting to (nearly) single rows, so a
    subtree's chain grows with its rows and a late large one idles the other
    waves -- 1M x 64 regression 8.90 -> 8.51 ms; two-class subtrees stop at pure
    nodes and the ordering's two launches cost more than they balance (3.087 vs
    3.098 ms; P = 8 rank 1.910 vs 1.915, ``profiles/r6/ab_lpt_*.log``)."""
    env = os.environ.get("MPITREE_TINY_LPT")
    if (env == "0") if env is not None else not on:
        return 0
    nb = (2 * 65 + int(cap)) * 4
    return _workspace(device, "fin.tiny_order", nb).data_ptr()


def _task_flags(device, n: int, slot: int = 0):
    """Epoch-tagged publish flags of the finisher's hand-off queue: a flag is
    set when it equals this launch's epoch, so the buffer is never cleared
    between launches (zeroed once when it grows). Launches that can run at the
    same time (``slot``: the early finisher batch on a side stream) own
    separate buffers."""
    key = f"{device}/{slot}"
    ent = _TASK_FLAGS.get(key)
    if ent is None or ent[0].numel() < n:
        ent = _TASK_FLAGS[key] = [torch.zeros(max(n, 4096), dtype=torch.int32, device=device), 0]
    ent[1] = ent[1] % 0x7FFFFFFE + 1
    return ent[0], ent[1]


_ws_tensors: dict = {}


def _ws_tensor(device, name: str, shape: tuple, dtype) -> torch.Tensor:
    """A device tensor reused by consecutive fits of one shape (one dict lookup:
    each fresh allocation costs host time on the path to the first level). The
    fit's setup buffers only: nothing holds them once a fit returns."""
    k = (str(device), name)
    t = _ws_tensors.get(k)
    if t is None or t.shape != shape or t.dtype != dtype:
        t = _ws_tensors[k] = torch.empty(shape, dtype=dtype, device=device)
    return t


_pinned_np: dict = {}


def _pinned_host(key: str, count: int, dtype) -> tuple:
    """(numpy view, host address) of a reusable pinned buffer of ``count``
    elements, for :func:`_d2h` (a raw async copy: no tensor views per fit)."""
    ent = _pinned_np.get(key)
    if ent is None or ent[0].size < count or ent[0].dtype != np.dtype(dtype):
        t = torch.empty(max(int(count), 256), dtype=torch.from_numpy(np.zeros(0, dtype)).dtype,
                        pin_memory=True)
        arr = t.numpy()
        ent = _pinned_np[key] = (arr, int(arr.ctypes.data), t)
    return ent[0][:count], ent[1]


def _d2h(host_ptr: int, t: torch.Tensor) -> None:
    """Enqueue the copy of device tensor ``t`` (contiguous) to ``host_ptr``."""
    native.hip().copy_d2h(_stream(), host_ptr, t.data_ptr(), t.numel() * t.element_size())


_DEFERRED: list = []


def defer(fn) -> None:
    """Host work a fit needs done before it returns but not before its first
    level: run by :func:`run_deferred` while the GPU grows the tree (the level
    loop's host waits) instead of on the path to the first kernel."""
    _DEFERRED.append(fn)


def run_deferred() -> None:
    while _DEFERRED:
        _DEFERRED.pop(0)()


_events: dict = {}


def _event(device, key: str) -> torch.cuda.Event:
    """A reusable event per (device, purpose): fits record and wait on it in
    order, and creating one costs host time on the path to the first level."""
    k = (str(device), key)
    ev = _events.get(k)
    if ev is None:
        ev = _events[k] = torch.cuda.Event()
    return ev


def _pinned_copy(t: torch.Tensor, key: str) -> np.ndarray:
    """Start an async D2H copy of ``t`` into a reusable pinned buffer; returns
    the numpy view (valid after the stream is synchronised). Buffers grow
    geometrically and are reused, so steady-state fits allocate nothing."""
    n = t.numel()
    buf = _pinned.get(key)
    if buf is None or buf.numel() < n or buf.dtype != t.dtype:
        cap = max(n, 2 * (buf.numel() if buf is not None and buf.dtype == t.dtype else 0), 1024)
        buf = torch.empty(cap, dtype=t.dtype, pin_memory=True)
        _pinned[key] = buf
    view = buf[:n].view(t.shape)
    view.copy_(t, non_blocking=True)
    return view.numpy()


_ZC_POOL: list = []  # [ndarray, device pointer, host pointer] of mapped host buffers
_ZC_COHERENT = os.environ.get("MPITREE_ZC_COHERENT", "0") == "1"
# single-process assembly: emit straight into host memory (1) or into device memory
# plus one DMA (0); the shared-host assembly of several ranks always stores directly
_ZC_EMIT = os.environ.get("MPITREE_ZC_EMIT", "0") == "1"


def _zc_out(nbytes: int):
    """A pinned, device-mapped host buffer of at least ``nbytes`` for a fit's tree
    columns, as ``(ndarray, device pointer)``: the assembly's emit kernel stores
    into it directly (zero-copy over PCIe: ~55 GB/s on MI355X against ~30-46 GB/s
    for a device write plus a D2H DMA, ``tools/probes/zc_probe.hip``).

    Pinning is the expensive part of a host allocation, so buffers are
    pooled: the returned :class:`TreeArrays` columns are
    numpy views of the pooled ndarray, so a buffer whose ndarray has no
    references besides this pool's is free to reuse."""
    import ctypes

    def free(i) -> bool:  # references: the pool's entry and getrefcount's argument
        return sys.getrefcount(_ZC_POOL[i][0]) <= 2

    best = None
    for i in range(len(_ZC_POOL)):
        if _ZC_POOL[i][0].size >= nbytes and free(i):
            if best is None or _ZC_POOL[i][0].size < _ZC_POOL[best][0].size:
                best = i
    if best is not None:
        return _ZC_POOL[best][0], _ZC_POOL[best][1]
    hip = native.hip()
    if len(_ZC_POOL) >= 8:  # keep a few: drop the oldest free buffer
        drop = [i for i in range(len(_ZC_POOL)) if free(i)]
        if drop:
            hptr = _ZC_POOL.pop(drop[0])[2]
            hip.host_free(hptr)
    size = max(int(nbytes * 1.25), 1 << 16)
    hptr = int(hip.host_alloc(size, coherent=_ZC_COHERENT))
    nd = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(hptr))
    ent = [nd, int(hip.host_device_ptr(hptr)), hptr]
    _ZC_POOL.append(ent)
    return ent[0], ent[1]


def xlog2x_table_f32(device) -> torch.Tensor:
    """fp32 rounding of :func:`xlog2x_table` (the finisher's approximate pass)."""
    key = "f32:" + str(device)
    t = _xtab_cache.get(key)
    if t is None:
        t = xlog2x_table(device)[:XTAB_N].float()
        _xtab_cache[key] = t
    return t


class HipBackend:
    """Device state and kernel launches for one fit on the current GPU."""

    name = "hip"

    def __init__(self, device=None):
        self.hip = native.hip()
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.up = _uploader(self.device)
        self.timing = False

    # ---------------------------------------------------------------- setup
    def setup(self, codes_rm, codes_fm, y, nbins_dev, *, n_bins: int, n_classes: int,
              criterion: Criterion):
        self.codes_rm = codes_rm
        self.codes_fm = codes_fm
        self.n, self.row_elems = codes_rm.shape
        self.F = codes_fm.shape[0]
        self.cb = codes_rm.element_size()
        self.y = y
        self.nbins = nbins_dev
        self.B = int(n_bins)
        self.crit = criterion
        self.reg = criterion == Criterion.SQUARED_ERROR
        self.C = 2 if self.reg else int(n_classes)
        # row permutation; classification packs the label into the top byte
        self.lab_shift = 24 if (not self.reg and self.n < (1 << 24) and self.C <= 256) else 0
        self.row_mask = (1 << self.lab_shift) - 1 if self.lab_shift else 0xFFFFFFFF
        self.idx = torch.empty(self.n, dtype=torch.int32, device=self.device)
        self.hip.init_idx(_stream(), self.idx.data_ptr(),
                          self.y.data_ptr() if not self.reg else 0, self.lab_shift, self.n)
        self.tmp = torch.empty_like(self.idx)
        self.xtab = xlog2x_table(self.device)
        self.xtabf = xlog2x_table_f32(self.device)

    # row permutation, label-packed entries included (level checkpoints)
    def get_rows(self) -> np.ndarray:
        return self.idx.cpu().numpy()

    def set_rows(self, rows) -> None:
        self.idx.copy_(torch.from_numpy(np.ascontiguousarray(rows, dtype=np.int32)))

    def hist_elems(self, F_h: int) -> int:
        return F_h * self.B * (2 if self.reg else self.C)

    def alloc_hist(self, slots: int, F_h: int | None = None):
        F_h = self.F if F_h is None else F_h
        self._F_h = F_h
        dt = torch.int64 if self.reg else torch.int32
        shape = (max(slots, 1), F_h, self.B, 2 if self.reg else self.C)
        if not self.lds_hist(F_h):  # global-atomic histograms add into zeroed slots
            return torch.zeros(shape, dtype=dt, device=self.device)
        return torch.empty(shape, dtype=dt, device=self.device)

    def lds_hist(self, F_h: int | None = None) -> bool:
        """Histograms built in LDS (feature tiles, or class tiles of one feature
        past the budget) rather than by global atomics."""
        F_h = self.F if F_h is None else F_h
        return self.hip.hist_class_tile(F_h, self.B, self.C, self.reg, LDS_BUDGET) > 0

    # ------------------------------------------------------------ histograms
    def build_hist(self, hist, slots, starts, counts, f_lo=0, f_hi=None):
        f_hi = self.F if f_hi is None else f_hi
        F_h = f_hi - f_lo
        if len(slots) == 0:
            return
        slots = np.asarray(slots, dtype=np.int64)
        starts = np.asarray(starts, dtype=np.int64)
        counts = np.asarray(counts, dtype=np.int64)
        total = int(counts.sum())
        lds = self.lds_hist(F_h)
        # ~2 workgroups per CU over the whole level, at most 65535 rows per item
        chunk = int(min(MAX_ITEM_ROWS, max(1024, -(-total // (2 * N_CU)))))
        if not lds:
            chunk = MAX_ITEM_ROWS  # global-atomic fallback: every item adds into hist
        k = np.maximum(1, -(-counts // chunk))
        node_of = np.repeat(np.arange(len(slots)), k)
        first = np.cumsum(k) - k
        i_in = np.arange(node_of.size) - first[node_of]
        c0 = i_in * chunk
        multi = (k > 1) & lds
        slab_base = np.cumsum(np.where(multi, k, 0)) - np.where(multi, k, 0)
        dest = np.where(multi[node_of], slab_base[node_of] + i_in, -1)
        items = np.stack([slots[node_of], starts[node_of] + c0,
                          np.minimum(chunk, counts[node_of] - c0), dest], 1)
        red = np.stack([slots[multi], slab_base[multi], k[multi]], 1)
        nslab = int(k[multi].sum())
        d_items, d_red = self.up(items, red)
        slab = None
        if nslab:
            sw = self.hip.hist_slab_words(F_h, self.B, self.C, self.reg)
            slab = torch.empty((nslab, sw), dtype=hist.dtype, device=self.device)
        self.hip.hist(_stream(), self.codes_rm.data_ptr(), self.cb, self.row_elems * self.cb,
                      self.idx.data_ptr(), self.y.data_ptr(), self.lab_shift, d_items.data_ptr(),
                      items.shape[0], hist.data_ptr(), 0 if slab is None else slab.data_ptr(),
                      F_h, f_lo, self.B, self.C, self.reg, LDS_BUDGET)
        if nslab:
            self.hip.hist_reduce(_stream(), d_red.data_ptr(), red.shape[0], int(k[multi].max()),
                                 slab.data_ptr(), hist.data_ptr(), F_h, self.B, self.C, self.reg)
        self._keep = (slab, d_items, d_red)

    def derive_hist(self, hist, prev_hist, slots, parent_slots, sibling_slots):
        if len(slots) == 0:
            return
        der = np.stack([slots, parent_slots, sibling_slots], 1).astype(np.int64)
        (d_der,) = self.up(der)
        E = hist[0].numel()
        self.hip.hist_derive(_stream(), d_der.data_ptr(), der.shape[0], prev_hist.data_ptr(),
                             hist.data_ptr(), E, self.reg)
        self._keep_d = d_der

    # ------------------------------------------------------------------ scan
    def scan(self, hist, slots, min_samples_leaf=1, f_lo=0, f_hi=None):
        f_hi = self.F if f_hi is None else f_hi
        F_h = f_hi - f_lo
        k = len(slots)
        C = self.C
        R = 7 if self.reg else 5 + 2 * C
        (d_nodes,) = self.up(np.asarray(slots, dtype=np.int64))
        cost = torch.empty((k, F_h), dtype=torch.float64, device=self.device)
        bins = torch.empty((k, F_h), dtype=torch.int32, device=self.device)
        rec = torch.empty((k, R), dtype=torch.int64, device=self.device)
        self.hip.scan(_stream(), hist.data_ptr(), d_nodes.data_ptr(), k, self.nbins.data_ptr(),
                      F_h, f_lo, self.B, C, int(self.crit), int(max(1, min_samples_leaf)),
                      cost.data_ptr(), bins.data_ptr(), rec.data_ptr(), self.xtab.data_ptr(),
                      XTAB_N)
        self.last_rec = rec
        r = rec.cpu().numpy()
        return unpack_records(r, C, self.reg)

    # ------------------------------------------------------------- partition
    def partition(self, starts, counts, features, bins, need_counts=True):
        k = len(starts)
        if k == 0:
            return np.zeros(0, dtype=np.int64)
        starts = np.asarray(starts, dtype=np.int64)
        counts = np.asarray(counts, dtype=np.int64)
        split = np.stack([starts, counts, np.asarray(features, np.int64),
                          np.asarray(bins, np.int64)], 1)
        items = chunk_items(np.arange(k), starts, counts, 1024)
        cursors = np.stack([starts, starts + counts], 1)
        d_split, d_items, d_cur64 = self.up(split, items, cursors)
        cur = d_cur64.view(k, 2).to(torch.int32)
        self.hip.partition(_stream(), self.codes_fm.data_ptr(), self.cb, self.n,
                           self.idx.data_ptr(), self.tmp.data_ptr(), self.row_mask,
                           d_items.data_ptr(), items.shape[0], d_split.data_ptr(), cur.data_ptr())
        if not need_counts:
            self._keep_p = (d_split, d_items, cur)
            return None
        return cur[:, 0].cpu().numpy().astype(np.int64) - starts

    def segment_stats(self, starts, counts):
        k = len(starts)
        items = chunk_items(np.arange(k), np.asarray(starts, np.int64),
                            np.asarray(counts, np.int64), 4096)
        (d_items,) = self.up(items)
        if self.reg:
            out = torch.zeros((k, 4), dtype=torch.int64, device=self.device)
            out[:, 2] = np.iinfo(np.int64).max
            out[:, 3] = np.iinfo(np.int64).min
        else:
            out = torch.zeros((k, self.C), dtype=torch.int32, device=self.device)
        self.hip.seg_stats(_stream(), self.idx.data_ptr(), self.y.data_ptr(), self.lab_shift,
                           self.reg, d_items.data_ptr(), items.shape[0], out.data_ptr(), self.C)
        return out.cpu().numpy().astype(np.int64)

    # -------------------------------------------------------------- finisher
    def finisher_supported(self) -> bool:
        if self.reg:  # (features past 256: more LDS tiles per node, no tiny kernel)
            return self.B <= 256
        # C <= 256, any F, B <= 4096 (16-bit codes past 256 bins: multi-pass
        # scans): the block finisher tiles features (and classes' words) through
        # LDS when one node's histogram does not fit in one pass
        return self.hip.finish_feature_tile(self.F, self.B, self.C) > 0

    @property
    def max_finisher_rows(self) -> int:
        """Finisher jobs index the x*log2(x) table with row counts (keep them
        below it); past 256 classes a job holds at most 255 rows, so a node's
        present classes and counts fit the finisher's 8-bit compacted histograms."""
        return int(min(XTAB_N - 1, self.hip.finish_job_rows_cap(int(self.C))))

    # ------------------------------------------------ pre-order position space
    def begin_positions(self, P: int):
        """Allocate the fit's position space: every node is written at its
        pre-order position with holes (a subtree of r rows owns 2r - 1
        positions); ``assemble_positions`` removes the holes on the device."""
        if P >= 2**31 - 1:
            raise ValueError("position space exceeds 2^31 (more than ~1e9 rows)")
        self.P = P = int(P)
        # reused device scratch: only the records need clearing (n = 0 marks a hole)
        rec = _workspace(self.device, "pos_rec", P * 24)
        self.pos_rec = rec[: P * 24].view(torch.int32).view(P, 6)
        self.pos_rec.zero_()
        dt = torch.int64 if self.reg else torch.int32
        sb = P * self.C * (8 if self.reg else 4)
        self.pos_st = _workspace(self.device, "pos_st", sb)[:sb].view(dt).view(P, self.C)

    def put_positions(self, pos, feature, tbin, lpos, rpos, depth, nsamp, stats):
        """Write host-grown (level-wise) nodes into the position space."""
        if len(pos) == 0:
            return
        rec = np.stack([feature, tbin, lpos, rpos, depth, nsamp], 1)
        d_pos, d_rec, d_st = self.up(np.asarray(pos, np.int64), rec,
                                     np.asarray(stats, np.int64))
        self.pos_rec.index_copy_(0, d_pos, d_rec.reshape(-1, 6).to(torch.int32))
        self.pos_st.index_copy_(0, d_pos, d_st.reshape(-1, self.C).to(self.pos_st.dtype))

    def assemble_positions(self, edges, crit: int, y_exp: int = 0, d_edges=None,
                           thr_pos=None, shared=None) -> TreeArrays:
        """Compact the position space into the finished, pre-ordered
        :class:`TreeArrays` (numpy views of one mapped host buffer; every column
        is computed on the device, nothing is derived on the host afterwards).
        ``d_edges``: the device fp64 threshold table ``[F, W]`` (any row stride);
        otherwise ``edges`` (host ``[F, W]``) is uploaded. Rank -> emit run back
        to back; the emit kernel stores the columns straight into pinned host
        memory (zero-copy over PCIe: no device staging buffer, no separate D2H),
        laid out from the device node count, then the host waits once.
        ``shared``: the node-local shared-host assembly of a subtree-ownership fit
        (``parallel/shared_tree.py``): dict(comm, pool, segs, S)."""
        P, C = self.P, self.C
        hip = self.hip
        s = _stream()
        if d_edges is None and thr_pos is None:
            d_edges = torch.from_numpy(np.ascontiguousarray(edges, np.float64)).to(self.device)
        tiles = hip.asm_tiles(P)
        bpn = int(hip.asm_node_bytes(C, self.reg))
        al = lambda x: (x + 255) // 256 * 256  # noqa: E731
        o_total = al(max(tiles, 1) * 4)
        o_rank = o_total + 256
        ws = _workspace(self.device, "asm", o_rank + al(P * 4))
        base = ws.data_ptr()
        total = ws[o_total : o_total + 16].view(torch.int64)  # {nodes, depth}
        hip.asm_rank(s, self.pos_rec.data_ptr(), P, base, base + o_total, base + o_rank)

        def emit(out_dev: int, cap_nodes: int, **kw):
            hip.asm_emit(s, self.pos_rec.data_ptr(), self.pos_st.data_ptr(), self.reg, P, C,
                         base + o_rank, 0 if d_edges is None else d_edges.data_ptr(),
                         0 if d_edges is None else int(d_edges.stride(0)),
                         base + o_total, out_dev, bool(self.reg), int(crit), int(y_exp),
                         self.xtab.data_ptr(), XTAB_N,
                         thr_pos=0 if thr_pos is None else thr_pos.data_ptr(),
                         cap_nodes=cap_nodes, **kw)

        if shared is not None:
            return self._assemble_shared(shared, emit, total, base + o_rank, bpn)
        # the emit lays the columns out from the device node count, so a buffer
        # sized for the previous fit's count on this position space (a refit of
        # the same data: the same count) is written in the same pass; a larger
        # tree (the kernel writes nothing past the buffer) is emitted again
        key = (str(self.device), P, C, bool(self.reg))
        guess = min(max(_ASM_HINT.get(key, 0), 1), P) * bpn
        nd, dptr = _zc_out(guess)
        if _ZC_EMIT:  # the emit kernel stores into the host buffer (PCIe writes)
            emit(dptr, nd.size // bpn)
        else:  # the emit writes device memory, one DMA copies the guessed bytes
            dbuf = _workspace(self.device, "asm.out", P * bpn)
            emit(dbuf.data_ptr(), 0)
            hip.copy_d2h(s, int(nd.ctypes.data), dbuf.data_ptr(), guess)
        h_total = _pinned_copy(total, "asm.total")
        torch.cuda.current_stream(self.device).synchronize()
        self._check_finisher_watch()
        N, max_depth = int(h_total[0]), int(h_total[1])
        _ASM_HINT[key] = N
        nbytes = N * bpn
        if _ZC_EMIT and nbytes > nd.size:
            nd, dptr = _zc_out(nbytes)
            emit(dptr, nd.size // bpn)
            torch.cuda.current_stream(self.device).synchronize()
        elif not _ZC_EMIT and nbytes > guess:  # (a larger tree than the guess)
            if nbytes > nd.size:
                nd, dptr = _zc_out(nbytes)
                guess = 0
            hip.copy_d2h(s, int(nd.ctypes.data) + guess, dbuf.data_ptr() + guess, nbytes - guess)
            torch.cuda.current_stream(self.device).synchronize()
        self.pos_rec = self.pos_st = None
        return TreeArrays.from_packed(nd[:nbytes], N, C, bool(self.reg), max_depth=max_depth)

    def _assemble_shared(self, sh, emit, total, rank_ptr: int, bpn: int):
        """Each rank of one node writes its own nodes (rank 0 also the replicated
        prefix) into one shared host buffer (``parallel/shared_tree.py``). None
        (on every rank alike) when the node's /dev/shm cannot hold a new buffer
        for the tree: the caller falls back to the node exchange."""
        from ..parallel.shared_tree import GATHER_HDR, HEADER, shm_free_bytes

        comm, pool, segs, S = sh["comm"], sh["pool"], sh["segs"], int(sh["S"])
        hip = self.hip
        s = _stream()
        Pn, me = int(comm.world_size), int(comm.rank)
        W = GATHER_HDR + int(segs.shape[0])
        nw = W * (Pn + 1) + 4 * int(segs.shape[0])
        g = _workspace(self.device, "shm.seg", nw * 8)[: nw * 8].view(torch.int64)
        gvec, gall, tab = g[:W], g[W : W * (Pn + 1)], g[W * (Pn + 1) :]
        hip.shm_seg_count(s, segs.data_ptr(), S, me, rank_ptr, self.P, total.data_ptr(),
                          gvec.data_ptr())
        gvec[1].fill_(pool.free_mask())
        gvec[2].fill_(shm_free_bytes())
        comm.all_gather_seg_counts(gall, gvec, segs, S)
        hip.shm_seg_prefix(s, gall.data_ptr(), Pn, W, segs.data_ptr(), S, me, total.data_ptr(),
                           tab.data_ptr())
        kw = dict(tab=tab.data_ptr(), n_tab=S, me=me, emit_prefix=me == 0)
        slot = pool.take_next()  # (agreed last fit: emit before the host wait)
        if slot is not None:
            emit(slot.dev + HEADER, (slot.nbytes - HEADER) // bpn, **kw)
        gv = gall.view(Pn, W)
        h = _pinned_copy(torch.cat([total, gv[:, 1], gv[:, 2]]), "shm.total")
        torch.cuda.current_stream(self.device).synchronize()
        self._check_finisher_watch()
        N, max_depth = int(h[0]), int(h[1])
        nbytes = N * bpn
        masks = [int(v) for v in h[2 : 2 + Pn]]
        free = [int(v) for v in h[2 + Pn : 2 + 2 * Pn]]
        if slot is None or nbytes > slot.nbytes - HEADER:  # (every rank sees the same N)
            slot = pool.choose(masks, nbytes, shm_free=free)
            if slot is None:
                return None
            emit(slot.dev + HEADER, 0, **kw)
            torch.cuda.current_stream(self.device).synchronize()
        pool.barrier(slot)
        pool.plan_next(masks, slot, nbytes, shm_free=free)
        self.pos_rec = self.pos_st = None
        return TreeArrays.from_packed(slot.nd[HEADER : HEADER + nbytes], N, self.C, bool(self.reg),
                                      max_depth=max_depth)

    def small_fit_supported(self, comm=None) -> bool:
        """One-workgroup whole-tree fit (``small_fit.hip``): classification on
        at most 1024 rows, any number of classes (the reference's published
        n-class sweep), one process."""
        return (not self.reg and self.n <= int(self.hip.small_fit_max_rows())
                and self.C < 65536 and getattr(comm, "world_size", 1) == 1
                and os.environ.get("MPITREE_SMALL_FIT", "1") != "0")

    def fit_small(self, params, edges, d_edges=None) -> TreeArrays:
        """Grow the whole tree in one launch and assemble it (one sync)."""
        n, F, C = self.n, self.F, self.C
        self.begin_positions(max(2 * n - 1, 1))
        ord_buf = _workspace(self.device, "small.ord", 2 * 2 * (F + 1) * max(n, 1))
        md = -1 if params.max_depth is None else int(params.max_depth)
        self.hip.small_fit(_stream(), self.codes_fm.data_ptr(), self.cb,
                           int(self.codes_fm.stride(0)), n, F, self.y.data_ptr(), C,
                           int(self.crit), md,
                           int(params.min_samples_split), int(max(1, params.min_samples_leaf)),
                           self.xtab.data_ptr(), XTAB_N, ord_buf.data_ptr(),
                           self.pos_rec.data_ptr(), self.pos_st.data_ptr(), self.P)
        return self.assemble_positions(edges, int(self.crit), 0, d_edges=d_edges)

    def _check_finisher_watch(self):
        watch = list(_FIN_WATCH)
        _FIN_WATCH.clear()
        for w in watch:
            if int(w[0]) != 0:
                raise RuntimeError(
                    "subtree finisher: a workgroup's wait for handed-off work timed out "
                    "; the tree is incomplete")

    def launch_finisher(self, d_jobs, J: int, job_rows: int, params, rec, cnt, counter=None,
                        grid=None, slot: int = 0, share: int = 1):
        """Launch the block + wave finisher kernels on ``J`` device jobs
        (int64 [J][5 + C] = {start, count, depth, root position, buffer, counts},
        largest first for load balance) writing into position space rec/cnt.
        ``share`` > 1: this launch grows about 1 / share of the tree's subtrees (a
        rank of a multi-GPU fit): the tiny-subtree kernel then runs 8-wave
        workgroups, twice as many as the occupancy-first 16 for 64 features -- its
        few subtrees spread over more CUs (P = 8 ownership rank 2.01-2.36 ->
        1.96-1.97 ms; one GPU keeps 16: 3.41 vs 3.58 ms with 8)."""
        if J <= 0:
            return
        C = self.C
        if counter is None:  # eight int32 work cursors, zero at launch
            counter = torch.zeros(128, dtype=torch.int32, device=self.device)
        if self.reg:
            self._launch_finisher_reg(d_jobs, J, job_rows, params, rec, cnt, counter, grid, slot)
            return
        tiny_rows = int(os.environ.get("MPITREE_TINY_ROWS", 64))
        md = -1 if params.max_depth is None else int(params.max_depth)
        grid = int(os.environ.get("MPITREE_FIN_GRID", 2 * N_CU)) if grid is None else int(grid)
        # every tiny subtree has >= 2 rows and they partition the job rows; each
        # workgroup reserves records kFinTinyBatch at a time
        tiny = _i64_scratch(self.device, "fin.tiny",
                            int(job_rows // 2 + J + 1 + grid * _tiny_batch(self.hip)), 8)
        if C > 2:  # (the hand-off queue is on the two-class kernel only)
            grid = min(grid, J)
        # subtrees handed to idle workgroups (each > 2 tiny_rows rows, disjoint)
        task_cap = int(job_rows // (2 * max(tiny_rows, 1) + 1) + 16)
        steal = os.environ.get("MPITREE_FIN_STEAL", "1" if C <= 2 else "-1")
        if steal == "0":
            task_cap = 0  # no hand-offs: spare workgroups only wait for the end
        elif steal == "-1":
            task_cap = -1  # no queue at all (claims past the jobs exit at once)
        tasks = _i64_scratch(self.device, "fin.tasks", max(task_cap, 1), 5 + C)
        flags, epoch = _task_flags(self.device, max(task_cap, 0) + grid, slot)
        prof = None
        if os.environ.get("MPITREE_FIN_PROF"):
            prof = torch.zeros((grid, 10), dtype=torch.int64, device=self.device)
        self.hip.finish(_stream(), self.codes_rm.data_ptr(), self.row_elems * self.cb // 4,
                        self.codes_fm.data_ptr(), self.cb, self.n, self.idx.data_ptr(),
                        self.tmp.data_ptr(), self.y.data_ptr(), self.lab_shift, d_jobs.data_ptr(),
                        J, counter.data_ptr(), self.nbins.data_ptr(), self.F, self.B, C,
                        int(self.crit), md, int(params.min_samples_split),
                        int(max(1, params.min_samples_leaf)), self.xtab.data_ptr(),
                        self.xtabf.data_ptr(), XTAB_N,
                        rec.data_ptr(), cnt.data_ptr(), tasks.data_ptr(), flags.data_ptr(),
                        epoch, task_cap, grid, tiny_rows, tiny.data_ptr(), 4 * N_CU,
                        0 if prof is None else prof.data_ptr(),
                        tiny_waves=8 if share > 1 else 0,
                        tiny_order=_tiny_order(self.device, tiny.shape[0], C > 2))
        self._fin_keep = (counter, tasks, tiny, d_jobs)
        # the hand-off queue's watchdog word (+ completed tasks), read
        # with the assembly's node-count sync: a finisher that gave up waiting
        # must fail the fit, never leave holes in the tree
        _FIN_WATCH.append(_pinned_copy(counter[100:101], f"fin.watch{len(_FIN_WATCH)}"))
        if prof is not None:
            self.last_finisher_prof = prof.cpu().numpy()

    def _launch_finisher_reg(self, d_jobs, J, job_rows, params, rec, st64, counter, grid_o=None,
                             slot=0):
        tiny_rows = int(os.environ.get("MPITREE_TINY_ROWS", 64))
        md = -1 if params.max_depth is None else int(params.max_depth)
        grid = os.environ.get("MPITREE_FIN_GRID") if grid_o is None else grid_o
        if grid is None:  # as many persistent workgroups as fit a CU (LDS tile, VGPRs)
            key = (self.B, self.cb)
            if key not in _REG_PER_CU:
                _REG_PER_CU[key] = int(self.hip.finish_reg_blocks_per_cu(self.B, self.cb))
            grid = _REG_PER_CU[key] * N_CU
        grid = int(grid)
        task_cap = int(job_rows // (2 * max(tiny_rows, 1) + 1) + 16)
        steal = os.environ.get("MPITREE_FIN_STEAL", "1")
        if steal == "0":
            task_cap = 0
        elif steal == "-1":
            task_cap, grid = -1, min(grid, J)
        cap = int(job_rows // 2 + J + 1 + grid * _tiny_batch(self.hip))
        tiny = _i64_scratch(self.device, "fin.tiny", cap, 8)
        tasks = _i64_scratch(self.device, "fin.tasks", max(task_cap, 1), 7)
        flags, epoch = _task_flags(self.device, max(task_cap, 0) + grid, slot)
        self.hip.finish_reg(_stream(), self.codes_rm.data_ptr(), self.row_elems * self.cb // 4,
                            self.codes_fm.data_ptr(), self.cb, self.n, self.idx.data_ptr(),
                            self.tmp.data_ptr(), self.y.data_ptr(), d_jobs.data_ptr(), J,
                            counter.data_ptr(), self.nbins.data_ptr(), self.F, self.B, md,
                            int(params.min_samples_split), int(max(1, params.min_samples_leaf)),
                            rec.data_ptr(), st64.data_ptr(), grid, tiny_rows, tiny.data_ptr(),
                            4 * N_CU, tasks.data_ptr(), flags.data_ptr(), epoch, task_cap,
                            _tiny_order(self.device, tiny.shape[0], True))
        self._fin_keep = (counter, tasks, tiny, d_jobs)
        _FIN_WATCH.append(_pinned_copy(counter[100:101], f"fin.watch{len(_FIN_WATCH)}"))

    def finish_subtrees(self, starts, counts, depths, params, stats=None, positions=None):
        """See :meth:`_finish_subtrees`."""
        return self._finish_subtrees(starts, counts, depths, params, stats, positions)

    def _finish_subtrees(self, starts, counts, depths, params, stats=None, positions=None):
        """Grow every job's subtree on the device.

        With ``positions`` (the jobs' pre-order positions in the fit's position
        space, see :meth:`begin_positions`) the nodes stay on the device and
        ``None`` is returned. Without, the jobs get a private position space
        and a compact node table comes back (the distributed merge format):
        arrays feature, bin, left, right, depth, nsamp, stats with child links
        indexing the table, and ``roots[j]``: the row of job j's root.
        """
        J = len(starts)
        starts = np.asarray(starts, np.int64)
        counts = np.asarray(counts, np.int64)
        depths = np.asarray(depths, np.int64)
        C = self.C
        table_mode = positions is None
        span = 2 * counts - 1  # a subtree of r rows owns 2r - 1 positions
        if table_mode:
            positions = np.cumsum(span) - span
            rec = torch.zeros((max(int(span.sum()), 1), 6), dtype=torch.int32, device=self.device)
            cnt = torch.empty((rec.shape[0], C), device=self.device,
                              dtype=torch.int64 if self.reg else torch.int32)
        else:
            rec, cnt = self.pos_rec, self.pos_st
        positions = np.asarray(positions, np.int64)
        order = np.argsort(-counts, kind="stable")  # largest first
        st = np.asarray(stats, np.int64).reshape(J, C)
        # {start, count, depth, root position, row buffer, class counts[C]}
        jobs = np.concatenate([np.stack([starts[order], counts[order], depths[order],
                                         positions[order], np.zeros(J, np.int64)], 1),
                               st[order]], 1)
        (d_jobs,) = self.up(jobs)
        self.launch_finisher(d_jobs, J, int(counts.sum()), params, rec, cnt)
        self._after_finisher(rec, starts, counts, positions)
        if not table_mode:
            return None
        # compact the private position space into the merge table
        P = rec.shape[0]
        tiles = self.hip.asm_tiles(P)
        tile = torch.empty(max(tiles, 1), dtype=torch.int32, device=self.device)
        total = torch.zeros(2, dtype=torch.int64, device=self.device)
        rank = torch.empty(P, dtype=torch.int32, device=self.device)
        self.hip.asm_rank(_stream(), rec.data_ptr(), P, tile.data_ptr(), total.data_ptr(),
                          rank.data_ptr())
        live = torch.nonzero(rank >= 0).squeeze(1)  # ascending position = table row
        r = rec[live]
        inner = r[:, 0] >= 0
        lk = torch.where(inner, rank[r[:, 2].long().clamp(min=0)], -1)
        rk = torch.where(inner, rank[r[:, 3].long().clamp(min=0)], -1)
        r = torch.stack([r[:, 0], r[:, 1], lk, rk, r[:, 4], r[:, 5]], 1)
        ni = r.cpu().numpy()
        nc = cnt[live].cpu().numpy().astype(np.int64)
        roots = rank[torch.from_numpy(positions).to(self.device)].cpu().numpy().astype(np.int64)
        return dict(feature=ni[:, 0], bin=ni[:, 1], left=ni[:, 2], right=ni[:, 3],
                    depth=ni[:, 4], nsamp=ni[:, 5], stats=nc, roots=roots, i32=ni, cnt=nc)

    def _after_finisher(self, rec, starts, counts, positions):
        """Hook on the finished position records (the exact engine maps codes back)."""

    def sync(self):
        if self.timing:
            torch.cuda.synchronize(self.device)


def chunk_items(ids, starts, counts, chunk):
    """[n, 3] int64 items {id, start, count} cutting segments into <= chunk rows."""
    ids = np.asarray(ids, dtype=np.int64)
    k = np.maximum(1, -(-counts // chunk))
    node_of = np.repeat(np.arange(len(ids)), k)
    first = np.cumsum(k) - k
    c0 = (np.arange(node_of.size) - first[node_of]) * chunk
    return np.stack([ids[node_of], starts[node_of] + c0,
                     np.maximum(0, np.minimum(chunk, counts[node_of] - c0))], 1)


def unpack_records(r: np.ndarray, C: int, reg: bool) -> dict:
    """Split-record rows (see split_scan.hip select_kernel) -> dict of arrays."""
    out = {
        "gain": r[:, 0].copy().view(np.float64),
        "feature": r[:, 1].astype(np.int32),
        "bin": r[:, 2].astype(np.int32),
        "n_left": r[:, 3].copy(),
        "m": r[:, 4].copy(),
    }
    if reg:
        out["left"] = np.stack([r[:, 3], r[:, 5]], 1)
    else:
        out["left"] = r[:, 5 : 5 + C].copy()
    return out
