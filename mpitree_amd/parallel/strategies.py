"""Distribution strategies: the communication hooks of the level-wise engine.

The reference has exactly one strategy: recursive subtree task parallelism
where every rank redundantly computes the upper levels, the communicator is
split by rank parity at each node, and pickled subtrees are exchanged with
``allgather`` (``mpitree/tree/decision_tree.py:319-338, 446-477``). It never
parallelises the root, holds all rows on every rank, and idles half the
ranks whenever a split is lopsided.

Here the same collective contract holds (every rank calls ``fit`` and every
rank returns the identical full tree), but work is divided MI355X-first with
one fused collective per tree level instead of per node:

``FeatureParallelComm`` ("feature")
    Rows replicated, features split into contiguous blocks. Each rank builds
    and scans histograms of its own features only; one ``all_gather`` of the
    per-node best candidates (a few dozen bytes per node) picks the global
    split (ties to the lowest feature, as in the reference). Every rank holds
    every feature-major column, so the row partition needs no communication.
``DataParallelComm`` ("data")
    Rows sharded; histograms of the level's built nodes are summed with one
    ``all_reduce`` (integer counts: exact and order-independent), after which
    every rank scans identically. Suited to n >> node count (10M x 128).
``SubtreeComm`` ("subtree")
    The reference's strategy made load-balanced: upper levels are computed
    redundantly with no communication until the first level with at least
    ``4 * P`` units (split nodes whose children keep growing + finisher jobs);
    that level assigns the units to ranks by greedy longest-processing-time on
    row counts (not by rank parity), each rank grows only its own units --
    device level loop and finisher -- and one ``all_gather`` of the finished
    position ranges completes the tree on every rank (GPU device loop,
    ``ops/device_grower.py``). Host-driven fits hand out only the finisher's
    subtree jobs that way.
"auto"
    Replicated rows: subtree ownership on the GPU device loop (feature-parallel
    levels with load-balanced subtree finishing on host-driven fits when
    ``F >= world_size``); row-sharded input: data-parallel. Exact thresholds on
    continuous features run the presorted-list engine feature-parallel
    (``ops/exact_grower.py``).

Collectives run on the backend's device (RCCL over xGMI for GPU fits, gloo
for CPU fits), so the same code is exercised by the multi-process CPU tests.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ..core.levelwise import LocalComm
from . import process_group as pgm

__all__ = [
    "DistComm",
    "FeatureParallelComm",
    "DataParallelComm",
    "SubtreeComm",
    "make_comm",
    "lpt_assign",
    "feature_blocks",
]


def feature_blocks(F: int, P: int) -> list:
    """Contiguous, balanced feature ranges; boundaries on multiples of 4 when possible."""
    if F >= 4 * P:
        q = F // 4
        b = [4 * (q * r // P) for r in range(P)] + [F]
    else:
        b = [F * r // P for r in range(P)] + [F]
    return [(b[r], b[r + 1]) for r in range(P)]


def lpt_assign(m: np.ndarray, P: int) -> np.ndarray:
    """Greedy longest-processing-time assignment of jobs (row counts) to ranks."""
    order = np.argsort(-np.asarray(m), kind="stable")
    load = np.zeros(P, dtype=np.int64)
    owner = np.empty(len(m), dtype=np.int64)
    for j in order:
        r = int(np.argmin(load))  # ties -> lowest rank
        owner[j] = r
        load[r] += int(m[j]) + 1
    return owner


_REC_FIXED = 5  # gain bits, feature, bin, n_left, m


def pack_records(res: dict) -> np.ndarray:
    left = np.asarray(res["left"], dtype=np.int64)
    K = left.shape[0]
    out = np.empty((K, _REC_FIXED + left.shape[1]), dtype=np.int64)
    out[:, 0] = np.asarray(res["gain"], dtype=np.float64).view(np.int64)
    out[:, 1] = res["feature"]
    out[:, 2] = res["bin"]
    out[:, 3] = res["n_left"]
    out[:, 4] = res.get("m", np.zeros(K, np.int64))
    out[:, _REC_FIXED:] = left
    return out


def unpack_records(r: np.ndarray) -> dict:
    return {
        "gain": r[:, 0].copy().view(np.float64),
        "feature": r[:, 1].astype(np.int32),
        "bin": r[:, 2].astype(np.int32),
        "n_left": r[:, 3].copy(),
        "m": r[:, 4].copy(),
        "left": r[:, _REC_FIXED:].copy(),
    }


class DistComm(LocalComm):
    """Common plumbing: rank/world, collective device, subtree exchange."""

    kind = "dist"

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.device = pgm.comm_device()
        self.bytes_communicated = 0

    # ------------------------------------------------------------ helpers
    def _t(self, a: np.ndarray) -> torch.Tensor:
        return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def _all_gather(self, a: np.ndarray) -> np.ndarray:
        """all_gather equal-shaped int64 arrays -> [P, *a.shape]."""
        t = self._t(a.astype(np.int64, copy=False)).reshape(1, -1)
        out = torch.empty((self.world_size, t.shape[1]), dtype=t.dtype, device=self.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        self.bytes_communicated += t.numel() * 8 * self.world_size
        return out.cpu().numpy().reshape((self.world_size,) + a.shape)

    def _all_reduce(self, a: np.ndarray, op=dist.ReduceOp.SUM) -> np.ndarray:
        t = self._t(a.astype(np.int64, copy=False))
        dist.all_reduce(t, op=op, group=self.group)
        self.bytes_communicated += t.numel() * 8
        return t.cpu().numpy()

    # ---------------------------------------------------- subtree exchange
    def finish_assignment(self, m: np.ndarray) -> np.ndarray:
        self._owner = lpt_assign(m, self.world_size)
        return self._owner == self.rank

    def merge_subtrees(self, local: dict, owned: np.ndarray, n_jobs: int) -> dict:
        """All ranks receive every job's nodes: one table, roots in job order.

        Three collectives in total: the per-rank node counts, the job roots
        (shifted to each rank's offset) and the padded node tables.
        """
        P = self.world_size
        C = local["stats"].shape[1]
        T = int(len(local["feature"]))
        sizes = self._all_gather(np.array([T], dtype=np.int64)).reshape(P)
        offs = np.concatenate([[0], np.cumsum(sizes)])
        roots_local = np.zeros(n_jobs, dtype=np.int64)
        roots_local[np.nonzero(owned)[0]] = np.asarray(local["roots"], np.int64) + offs[self.rank]
        roots = self._all_reduce(roots_local)
        W = 6 + C
        Tmax = int(sizes.max())
        pack = np.zeros((max(Tmax, 1), W), dtype=np.int64)
        if T:
            pack[:T, 0] = local["feature"]
            pack[:T, 1] = local["bin"]
            pack[:T, 2] = local["left"]
            pack[:T, 3] = local["right"]
            pack[:T, 4] = local["depth"]
            pack[:T, 5] = local["nsamp"]
            pack[:T, 6:] = local["stats"]
        allp = self._all_gather(pack)  # [P, Tmax, W]
        out = np.concatenate([allp[r, : sizes[r]] for r in range(P)], 0)
        for r in range(P):  # child links become global table rows
            blk = out[offs[r] : offs[r + 1]]
            inner = blk[:, 0] >= 0
            blk[inner, 2] += offs[r]
            blk[inner, 3] += offs[r]
        return dict(feature=out[:, 0].astype(np.int32), bin=out[:, 1].astype(np.int32),
                    left=out[:, 2], right=out[:, 3], depth=out[:, 4].astype(np.int32),
                    nsamp=out[:, 5], stats=out[:, 6:], roots=roots)

    def any_failed(self, failed: bool) -> bool:
        """All-reduce of a failure flag: True on every rank if any rank failed."""
        return bool(self._all_reduce(np.array([1 if failed else 0]),
                                     op=dist.ReduceOp.MAX)[0])

    def all_gather_rows(self, t):
        """All-gather a [k, w] int32 device tensor with per-rank k; returns the
        concatenation [sum k, w] on the tensor's device (padded exchange)."""
        import torch

        k = int(t.shape[0])
        sizes = self._all_gather(np.array([k], dtype=np.int64)).reshape(-1)
        kmax = int(max(1, sizes.max()))
        w = int(t.shape[1])
        buf = torch.zeros((kmax, w), dtype=t.dtype, device=self.device)
        if k:
            buf[:k].copy_(t.to(self.device))
        out = torch.empty((self.world_size * kmax, w), dtype=t.dtype, device=self.device)
        dist.all_gather_into_tensor(out, buf, group=self.group)
        self.bytes_communicated += buf.numel() * buf.element_size() * self.world_size
        parts = [out[r * kmax : r * kmax + int(sizes[r])] for r in range(self.world_size)]
        return torch.cat(parts, 0).to(t.device)

    def all_gather_rows_counted(self, buf, k_dev):
        """All-gather the first ``k_dev`` rows of ``buf`` ([cap, w] on the device;
        ``k_dev``: a one-element device int64 count a kernel wrote). The counts
        are exchanged on the device and read with ONE host wait -- the kernel
        that packed the rows and the count exchange finish together -- where
        :meth:`all_gather_rows` needs the local count on the host first. Rows
        past each rank's count are exchanged padded and dropped."""
        import torch

        P = self.world_size
        k_cap = torch.empty(2, dtype=torch.int64, device=k_dev.device)
        k_cap[0:1].copy_(k_dev.reshape(1))
        k_cap[1] = int(buf.shape[0])
        sizes_d = torch.empty(2 * P, dtype=torch.int64, device=k_dev.device)
        self.all_gather_device(sizes_d, k_cap)
        kc = sizes_d.cpu().numpy().reshape(P, 2)  # the one host wait
        sizes = kc[:, 0]
        kmax = int(max(1, sizes.max()))
        k, cap, w = int(sizes[self.rank]), int(buf.shape[0]), int(buf.shape[1])
        over = np.nonzero(kc[:, 0] > kc[:, 1])[0]
        if over.size:  # every rank sees every count and capacity: all raise here
            r = int(over[0])
            raise RuntimeError(f"row exchange: rank {r} packed {int(kc[r, 0])} rows into a "
                               f"buffer of {int(kc[r, 1])}")
        if kmax <= cap:
            src = buf[:kmax].contiguous()
        else:  # a peer has more rows than this buffer holds: pad a copy
            src = torch.empty((kmax, w), dtype=buf.dtype, device=buf.device)
            src[:k].copy_(buf[:k])
        out = torch.empty((P * kmax, w), dtype=buf.dtype, device=buf.device)
        self.all_gather_device(out.view(-1), src.view(-1))
        return torch.cat([out[r * kmax : r * kmax + int(sizes[r])] for r in range(P)], 0)

    # ------------------------------------------- device-resident collectives
    # The device level loop enqueues these between its kernels: with RCCL the
    # collective runs on the process group's stream ordered after the current
    # stream's kernels and the current stream waits for it -- no host sync.
    # A gloo group (CPU rehearsal of GPU ranks) stages through host memory.
    def _staged(self, t: torch.Tensor) -> bool:
        return t.device.type != self.device.type

    def all_gather_device(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """``out[r * inp.numel():...] = inp`` of rank r (flat, same dtype)."""
        if self._staged(inp):
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather_into_tensor(o, inp.cpu(), group=self.group)
            out.copy_(o)
        else:
            dist.all_gather_into_tensor(out, inp, group=self.group)
        self.bytes_communicated += inp.numel() * inp.element_size() * self.world_size

    def all_gather_seg_counts(self, out: torch.Tensor, inp: torch.Tensor, segs, S: int) -> None:
        """The shared-host assembly's per-segment node counts (``segs``/``S``: the
        segment table, used by simulated communicators only)."""
        self.all_gather_device(out, inp)

    def all_reduce_device(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> None:
        if self._staged(t):
            h = t.cpu()
            dist.all_reduce(h, op=op, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op, group=self.group)
        self.bytes_communicated += t.numel() * t.element_size()

    def reduce_device(self, t: torch.Tensor, dst: int, async_op: bool = False):
        """Sum ``t`` over the ranks into rank ``dst``'s ``t`` (other ranks' ``t``
        is left as it was or unspecified). With RCCL and ``async_op`` the reduce
        is enqueued on the process group's stream behind the current stream's
        kernels and the call returns at once -- the caller keeps launching work
        (the next feature block's histogram) and ``wait()`` on the returned work
        orders the current stream after the reduce. Returns None when done."""
        self.bytes_communicated += t.numel() * t.element_size()
        gdst = dst if self.group is None else dist.get_global_rank(self.group, dst)
        if self._staged(t):
            h = t.cpu()
            dist.reduce(h, dst=gdst, op=dist.ReduceOp.SUM, group=self.group)
            if self.rank == dst:
                t.copy_(h)
            return None
        return dist.reduce(t, dst=gdst, op=dist.ReduceOp.SUM, group=self.group,
                           async_op=async_op)

    def reduce_scatter_device(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """``out`` = chunk ``rank`` of the sum over the ranks of ``inp`` (flat, P
        equal contiguous chunks): one collective where P reduces to the chunks'
        owners would each pay RCCL's latency."""
        self.bytes_communicated += inp.numel() * inp.element_size()
        if self._staged(inp):  # (gloo group: a host all-reduce, then this rank's chunk)
            h = inp.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            out.copy_(h.view(self.world_size, -1)[self.rank].view(out.shape))
            return
        dist.reduce_scatter_tensor(out.view(-1), inp, op=dist.ReduceOp.SUM, group=self.group)

    def all_to_all_device(self, out: torch.Tensor, inp: torch.Tensor, out_splits: list,
                          in_splits: list) -> None:
        """Rows (dim 0) of ``inp`` go to ranks by ``in_splits``; ``out`` receives by
        ``out_splits`` (host lists, one entry per rank)."""
        if self._staged(inp):
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)
        row = inp[0].numel() * inp.element_size() if inp.dim() > 1 else inp.element_size()
        self.bytes_communicated += int(sum(in_splits)) * row

    def check_consistent(self, digest: int) -> bool:
        """Cross-rank check that every rank built the same tree."""
        a = self._all_gather(np.array([digest], dtype=np.int64))
        return bool((a == a[0]).all())


class FeatureParallelComm(DistComm):
    kind = "feature"
    rows_replicated = True

    def feature_range(self, F: int):
        if F < self.world_size:
            raise ValueError(f"feature-parallel needs n_features >= world size ({F} < "
                             f"{self.world_size}); use strategy='subtree' or 'data'")
        return feature_blocks(F, self.world_size)[self.rank]

    def combine_scan(self, res: dict) -> dict:
        rec = pack_records(res)
        allr = self._all_gather(rec)  # [P, K, R]
        gains = allr[:, :, 0].copy().view(np.float64)  # [P, K]
        feats = allr[:, :, 1]
        # max gain; ties -> lowest feature (ranks own increasing feature blocks)
        best = np.zeros(rec.shape[0], dtype=np.int64)
        bg = gains[0].copy()
        bf = feats[0].copy()
        for r in range(1, self.world_size):
            better = (gains[r] > bg) | ((gains[r] == bg) & (feats[r] < bf) & (feats[r] >= 0))
            better &= gains[r] > -np.inf
            best = np.where(better, r, best)
            bg = np.where(better, gains[r], bg)
            bf = np.where(better, feats[r], bf)
        chosen = allr[best, np.arange(rec.shape[0])]
        return unpack_records(chosen)


class DataParallelComm(DistComm):
    kind = "data"
    rows_replicated = False

    def __init__(self, group=None, n_total: int | None = None, sharded: bool = False):
        super().__init__(group)
        self.n_total = n_total
        self.sharded = sharded

    def local_rows(self, n: int):
        if self.sharded:
            return 0, n
        P, r = self.world_size, self.rank
        return n * r // P, n * (r + 1) // P

    def reduce_hist(self, hist, n_slots: int):
        if n_slots == 0:
            return
        h = hist[:n_slots]
        if h.device == self.device:
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
        else:  # e.g. GPU histograms over a gloo group (single-card rehearsal)
            t = h.to(self.device)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            h.copy_(t)
        self.bytes_communicated += h.numel() * h.element_size()

    def reduce_stats(self, stats: np.ndarray, reg: bool) -> np.ndarray:
        if not reg:
            return self._all_reduce(stats)
        s = self._all_reduce(stats[:, :2])
        mn = self._all_reduce(stats[:, 2], op=dist.ReduceOp.MIN)
        mx = self._all_reduce(stats[:, 3], op=dist.ReduceOp.MAX)
        return np.concatenate([s, mn[:, None], mx[:, None]], 1)

    def fit_kwargs(self) -> dict:
        # host-driven (CPU) data-parallel fits grow every level with per-level
        # histogram all-reduces: a subtree's rows are spread over the ranks, so
        # the single-process finisher does not apply. GPU fits ignore this: the
        # device loop sends each subtree job's rows to its owner first
        # (DeviceGrower._dp_finish) and uses the single-GPU finisher split point.
        return {"finisher_rows": 0}


class SubtreeComm(DistComm):
    kind = "subtree"
    rows_replicated = True

    def __init__(self, group=None, n_total: int = 0):
        super().__init__(group)
        self.n_total = n_total

    def fit_kwargs(self) -> dict:
        # hand subtrees to ranks early: ~8 jobs per rank below the root
        return {"finisher_rows": max(2, self.n_total // (8 * self.world_size))}


class AutoComm(FeatureParallelComm):
    """``strategy="auto"`` with replicated rows. GPU fits on the device-driven
    loop use subtree ownership (replicated levels until the LPT switch level,
    then each rank grows its own units:
    :class:`~mpitree_amd.ops.device_grower.DeviceGrower`); exact thresholds on
    continuous features run feature-parallel (``ops/exact_grower.py``); the
    host-driven level-wise builder (CPU fits) runs feature-parallel levels with
    load-balanced subtree finishing."""

    kind = "auto"


def make_comm(strategy: str, X, y, *, device="auto", data_sharded=False, regression=False):
    """Build the communication strategy for a collective fit; returns (comm, X, y)."""
    group = pgm.ensure_initialized(device)
    if group is None or dist.get_world_size() == 1:
        return LocalComm(), X, y
    n, F = X.shape
    P = dist.get_world_size()
    strategy = (strategy or "auto").lower()
    if strategy == "auto":
        if data_sharded:
            strategy = "data"
        elif F >= P:
            return AutoComm(), X, y
        else:
            strategy = "subtree"
    if data_sharded and strategy != "data":
        raise ValueError("data_sharded=True requires strategy='data'")
    if strategy == "feature":
        return FeatureParallelComm(), X, y
    if strategy == "data":
        return DataParallelComm(n_total=n, sharded=data_sharded), X, y
    if strategy == "subtree":
        return SubtreeComm(n_total=n), X, y
    raise ValueError(f"unknown strategy {strategy!r}")
