"""Device-driven level-wise growth for single-GPU classification fits.

The host-driven :class:`~mpitree_amd.core.levelwise.LevelwiseBuilder` reads
every level's split records back and rebuilds the next level's work lists in
numpy -- one device round trip and ~100 small host operations per level. Here
the same algorithm runs with the planning on the GPU (``grow.hip``):

per level, all on one stream and with device-side work counts
    histogram items -> slab reduction -> sibling derivation -> scan/select
    -> ``grow_plan_kernel`` (writes decided nodes into the pre-order position
    space, appends finisher jobs, builds the partition list and the next
    level's lists) -> partition + copy-back

so the host only enqueues fixed-shape launches. Grids are host-known upper
bounds (a level has at most ``min(2**L, n // (finisher_rows + 1) + 1)``
frontier nodes, because frontier nodes hold more than ``finisher_rows`` rows);
surplus workgroups exit on the device count. The host learns that the tree is
finished from a lagged read of host-mapped counters the planner stores, then
sorts the device job list (largest first) and launches the subtree finisher;
the position space is compacted by ``assemble.hip``. The resulting tree is
bitwise identical to the host-driven builder's (tests/test_gpu_kernels.py).

Multi-GPU (one process per GPU, RCCL over xGMI; collectives are enqueued on
the stream between the level kernels, never a host round trip):

* feature-parallel (``strategy="feature"`` / ``"auto"``): rows replicated,
  every rank builds and scans histograms of its own contiguous feature block
  only; one ``all_gather_into_tensor`` of the per-node split records per level
  feeds ``fp_combine_kernel`` (max gain, ties to the lowest feature), after
  which the planner and partition run identically on every rank;
* data-parallel (``strategy="data"``): rows sharded (a replicated input is
  binned per rank for its own shard only). Each level's built (smaller-child)
  histograms are built in one pass over the rank's rows, permuted block-major
  and summed with ONE ``reduce_scatter`` (integer counts: exact, order
  independent), so rank r receives the global histograms of its feature block.
  (Unequal blocks: each block is built and summed into its owner with a
  ``reduce`` enqueued right behind its kernels.) Every rank then scans only
  its own block (deriving larger siblings from its block of the parent) and
  the split records take the
  feature-parallel all-gather + ``fp_combine_kernel``. Local row segments are
  fixed up after the partition (``grow_dp_fixup_kernel``); regression purity
  takes one min/max all-reduce per level. (Fewer features than ranks: one
  all-reduce of the whole built histograms instead.)
* subtree jobs (nodes of at most ``finisher_rows`` rows) are split across
  ranks (serpentine over the largest-first job order); data-parallel ranks
  first send each job's rows to its owner (one ``all_to_all``; the owner lays
  them out in both code layouts in one pass, ``dp_route.hip dp_place``); the
  owners write their jobs' nodes into the node-shared host tree (one small
  all-gather of segment counts), or one all-gather of the finished nodes when
  the ranks span hosts.

Every mode produces the single-GPU tree bit for bit (tests/test_gpu_kernels.py,
tests/test_distributed.py).

Reference parity: mpitree/tree/decision_tree.py:93-166 (growth),
:63-91 (split search), :150-164 (recursion / stopping rules), :446-477
(subtree task parallelism, here the job split + node all-gather).
"""

from __future__ import annotations

import os
import time

import numpy as np
import torch

from ..models.tree_arrays import TreeArrays
from ..utils.observability import profiling
from . import hip_backend as hb
from ..parallel.failure import ABORT, check_abort, fault_point
from ..parallel import shared_tree
from ..parallel.strategies import feature_blocks

__all__ = ["DeviceGrower", "device_loop_supported"]

REC_DUMP = None  # list: the single-rank level loop appends each level's split records
# dict (per-rank simulations, bench/sim_dp_ranks.py): the single-rank level loop
# adds "hists" (each level's slot histograms) and "jobs" / "idx" / "tmp" / "row_mask"
# (the sorted finisher jobs and the row buffers they index)
DUMP = None

_WORKSPACES: dict = {}  # (device, n, F, B, C, reg, fr) -> level-loop buffers
_HOST_CTL: dict = {}  # device index -> (device pointer, numpy view [64, 16] int32)
_FIT_SEQ = [0]  # per-process fit counter: tags host slots so stale values never match
OWN_CAP = 2048  # ownership units sorted at the switch level (grow.hip kOwnMax)


def own_min_units(P: int) -> int:
    """Units (split nodes that keep growing + finisher jobs) the switch level
    needs before the ranks take ownership: more units balance the LPT better,
    each replicated level before the switch costs every rank a full level.
    2 per rank from P = 4 on (1M x 64 at P = 8: 2.24 vs 2.32 ms max rank;
    P = 4: equal, ``profiles/r4/sim_own_variants.log``), 4 below."""
    k = int(os.environ.get("MPITREE_OWN_UNITS_PER_RANK", "2" if P >= 4 else "4"))
    return max(2, k * P)
POLL_TIMEOUT_S = float(os.environ.get("MPITREE_POLL_TIMEOUT", "120"))
# histogram work items per CU and level (1 or 2): fewer, larger items write fewer
# LDS slabs for the reduction to read back
def hist_items_per_cu(reg: bool) -> int:
    """Histogram work items per CU and level: 1 -- half the slabs for the
    reduction to read back. Regression since round 5 (int64 {count, sum} slabs:
    1M x 64 9.35 -> 9.07 ms, profiles/r5/ab_hist_items_reg.log), classification
    since round 6 (C = 64 85.3 -> 83.3 ms, 10M x 128 41.86 -> 41.39 ms, 1024 bins
    15.0 -> 14.7 ms, the flagship / 100k / 200k x 512 unchanged;
    profiles/r6/ab_knobs_*.log, ab_hi_*.log); ``MPITREE_HIST_ITEMS`` = 2 restores
    two."""
    env = os.environ.get("MPITREE_HIST_ITEMS")
    return max(1, min(2, int(env))) if env else 1


def fp_prefix_pays(n: int, F: int, P: int, reg: bool) -> bool:
    """Whether the replicated levels before the ownership switch run
    feature-parallel (``MPITREE_OWN_FP_PREFIX`` = 1 / 0 forces it). A rank then
    histograms 1 / P of the features -- saving (1 - 1/P) of a level's per-row x
    feature histogram cost -- but each level adds a record all-gather, a select
    and a combine (~40 us with RCCL latency, an estimate: no multi-GPU box has
    measured it). The per-row x feature costs are measured, not assumed:
    ``bench/calib_hist.py`` fits the level-0 histogram (items + slab reduction)
    as ``a + b rows x features`` over 250k..4M rows x 16..128 features --
    classification b = 0.56 ps (a = 20 us), regression (int64 {count, sum} slabs)
    b = 1.38 ps (a = 74 us), ``profiles/r6/calib_hist.jsonl``. The 1M x 64
    classification tree breaks even at P = 8 and stays replicated; its regression
    tree and 10M-row fits gain."""
    env = os.environ.get("MPITREE_OWN_FP_PREFIX")
    if env is not None:
        return env != "0"
    per = 1.38e-12 if reg else 0.56e-12  # (s per row x feature of one level, measured)
    return (1.0 - 1.0 / max(P, 1)) * n * F * per > 40e-6


def own_jobs_at_switch(be) -> int:
    """``MPITREE_OWN_JOBS=1``: at the ownership switch the owned children that would
    keep growing become finisher jobs (up to the finisher's row limit), so a rank
    runs no level after the switch (0: own levels until the jobs are small)."""
    if os.environ.get("MPITREE_OWN_JOBS", "0") == "0":
        return 0
    return int(be.max_finisher_rows)


def _wait_slot(hctl, slot: int, tag: int):
    """Spin until the planner's store of ``tag`` into host slot ``slot`` lands
    (coherent host memory: no event, no stream sync, no driver call)."""
    row = hctl[slot]
    if row[2] == tag:
        return
    t_end = time.perf_counter() + POLL_TIMEOUT_S
    k = 0
    while row[2] != tag:
        k += 1
        if (k & 0xFFFF) == 0:
            if ABORT.is_set():  # a peer rank failed the collective fit
                check_abort()
            if time.perf_counter() > t_end:
                raise RuntimeError("device level loop: planner result never arrived "
                                   f"(slot {slot}, tag {tag}); the GPU stream is stuck")
            time.sleep(0)


def _host_ctl(hip, dev):
    """Host-mapped coherent slots the planner stores each level's {next frontier
    size, finisher jobs} into (no copy kernel, no pinned D2H per level)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ent = _HOST_CTL.get(key)
    if ent is None:
        import ctypes

        hptr = hip.host_alloc(64 * 16 * 4)
        view = np.ctypeslib.as_array((ctypes.c_int32 * (64 * 16)).from_address(hptr))
        ent = _HOST_CTL[key] = (hip.host_device_ptr(hptr), view.reshape(64, 16))
    return ent


def device_loop_supported(be, params, comm) -> bool:
    if os.environ.get("MPITREE_DEVICE_LOOP", "1") == "0":
        return False
    if getattr(comm, "world_size", 1) != 1:
        if getattr(comm, "kind", "") not in ("auto", "subtree", "feature", "data"):
            return False
    if params.finisher_rows <= 0 or not be.finisher_supported():
        return False
    # the planner drives the LDS histogram path only (feature or class tiles)
    if not be.lds_hist():
        return False
    # the level's [KMAX][F][B][C] histograms (two level parities, or one when
    # derive-free) plus the item slabs must fit (many classes: ~19.7 MB per node
    # at 64 x 256 x 300)
    n, F, B, C, reg = be.n, be.F, be.B, be.C, bool(be.reg)
    fr = int(params.finisher_rows)
    par = 1 if derive_free_levels(n, F, B, C, reg, fr, be.hip, be.device) else 2
    need = level_loop_bytes(n, F, B, C, reg, fr, be.hip, par)
    if need <= total_device_bytes(be.device) // 64:  # (no free-memory query: ~10 us a fit)
        return True
    return need <= agreed_free_bytes(comm, be.device) // 2


def slab_rows(n_loc: int) -> int:
    """Item slabs a level can need: only nodes split over several items use
    them, and such items hold >= 1024 rows each plus one partial item per node
    (plan_hist_items: <= 2 n / 1024)."""
    return 2 * (n_loc // 1024) + 16


def level_loop_bytes(n, F, B, C, reg, fr, hip, parities: int = 2) -> int:
    """Device bytes of the level loop's histogram buffers (``parities`` level
    parities) and item slabs for ``n`` rows with finisher jobs of at most ``fr``
    rows."""
    KMAX = n // (fr + 1) + 2
    IMAX = KMAX + n // 1024 + 2 * hb.N_CU + 16
    esz = 8 if reg else 4
    hist = parities * KMAX * F * B * (2 if reg else C) * esz
    slab = min(IMAX, slab_rows(n)) * int(hip.hist_slab_words(F, B, C, reg)) * esz
    return int(hist + slab)


_TOTAL_BYTES: dict = {}


def total_device_bytes(device) -> int:
    """The device's memory size (cached: a property query per fit costs host time)."""
    key = str(device)
    v = _TOTAL_BYTES.get(key)
    if v is None:
        try:
            v = int(torch.cuda.get_device_properties(device).total_memory)
        except Exception:  # pragma: no cover - (no device: tests on CPU)
            v = 0
        _TOTAL_BYTES[key] = v
    return v


def derive_free_levels(n, F, B, C, reg, fr, hip, device) -> bool:
    """Whether the level loop keeps ONE histogram buffer and builds every child
    from rows (no parent - sibling derivation, which needs the parent level's
    histograms): when two parities would take more than 40 % of the device
    (1M x 64 with 300 classes: 154 GB of histograms for 255-row finisher jobs).
    ``MPITREE_DERIVE_FREE`` = 1 / 0 forces it."""
    env = os.environ.get("MPITREE_DERIVE_FREE")
    if env is not None:
        return env != "0"
    total = total_device_bytes(device)
    if total <= 0:
        return False
    return level_loop_bytes(n, F, B, C, reg, fr, hip, 2) > 0.4 * total


def free_device_bytes(dev) -> int:
    try:
        return int(torch.cuda.mem_get_info(dev)[0])
    except Exception:  # pragma: no cover - (no CUDA context: tests on CPU)
        return 1 << 62


def agreed_free_bytes(comm, dev) -> int:
    """Free device bytes an engine decision may use: this rank's own reading
    on a single-rank fit, the minimum over the ranks otherwise (ranks sharing a
    card, or a fit near a threshold, read different values -- one rank taking
    another engine than its peers would mismatch every collective after it).
    ``MPITREE_FREE_BYTES`` overrides this rank's reading (tests)."""
    env = os.environ.get("MPITREE_FREE_BYTES")
    local = int(env) if env else free_device_bytes(dev)
    if getattr(comm, "world_size", 1) <= 1 or not hasattr(comm, "_all_reduce"):
        return local
    import torch.distributed as tdist

    return int(comm._all_reduce(np.array([local], np.int64), op=tdist.ReduceOp.MIN)[0])


def exchange_ranges(be, comm, ranges: torch.Tensor, bound: int):
    """Every rank wrote the positions inside its own ``ranges`` (int64 [cap, 2]
    {lo, hi}, unused rows {0, 0}) of the position space and nothing else differs
    between ranks: ``own_pack`` (assemble.hip) marks those ranges and packs their
    live positions as {pos, record[6], stats[C]} rows; one all-gather; every
    rank's rows are scattered back, so each position then holds its one writer's
    record everywhere. ``bound``: at most this many rows (a subtree of r rows has
    <= 2r - 1 nodes). One host wait: the packed row counts of every rank, exchanged
    on the device (``all_gather_rows_counted``). Returns the gathered rows (keep
    until the stream has passed the scatter)."""
    hip = be.hip
    s = hb._stream()
    Pp = int(be.pos_rec.shape[0])
    C, reg = be.C, bool(be.reg)
    dt = torch.int64 if reg else torch.int32
    esz = 8 if reg else 4
    tiles = int(hip.asm_tiles(Pp))
    bound = int(min(Pp, bound))
    al = lambda x: (x + 255) // 256 * 256  # noqa: E731
    o_tile, o_total = 0, al(max(tiles, 1) * 4)
    o_rank = o_total + 256
    o_mask = o_rank + al(Pp * 4)
    o_rows = o_mask + al(Pp)
    buf = hb._workspace(be.device, "own_exchange", o_rows + bound * (7 + C) * esz)
    buf[o_mask : o_mask + Pp].zero_()
    base = buf.data_ptr()
    hip.own_pack(s, ranges.data_ptr(), int(ranges.shape[0]), base + o_mask, be.pos_rec.data_ptr(),
                 be.pos_st.data_ptr(), reg, Pp, C, base + o_tile, base + o_total, base + o_rank,
                 base + o_rows, row_cap=bound)
    k_dev = buf[o_total : o_total + 8].view(torch.int64)
    if hasattr(comm, "all_gather_rows_counted"):
        allr = comm.all_gather_rows_counted(
            buf[o_rows : o_rows + bound * (7 + C) * esz].view(dt).view(bound, 7 + C), k_dev)
    else:  # (stand-in communicators: the local count first)
        h_k = hb._pinned_copy(k_dev, "own.k")
        torch.cuda.current_stream(be.device).synchronize()
        k = int(h_k[0])
        if k > bound:
            raise RuntimeError(f"node exchange: {k} nodes exceed the bound {bound}")
        rows = buf[o_rows : o_rows + k * (7 + C) * esz].view(dt).view(k, 7 + C)
        allr = comm.all_gather_rows(rows)
    hip.own_scatter(s, allr.data_ptr(), int(allr.shape[0]), C, be.pos_rec.data_ptr(),
                    be.pos_st.data_ptr(), reg)
    return allr


class DeviceGrower:
    def __init__(self, be, params, comm=None, checkpoint=None):
        self.be = be
        self.p = params
        self.comm = comm
        self.ckpt = checkpoint  # utils/level_checkpoint.LevelCheckpoint (or None)
        self.timings: dict = {}
        self.stats: dict = {}

    # ------------------------------------------------------- checkpoint
    def _ckpt_save(self, lvl, ws, sets, hists, rank, P):
        """After level ``lvl``'s kernels: one sync, then the loop's device state
        (nothing is saved once the next frontier is empty: the fit is about to
        finish)."""
        be = self.be
        torch.cuda.synchronize(be.device)
        nxt = sets[(lvl + 1) % 2]
        if int(nxt["ctl"][0]) == 0:
            return
        kc = int(sets[lvl % 2]["ctl"][0])  # this level's frontier (the next derives from it)
        jc = int(ws["job_count"][0])
        arrs = {"set_" + k: v.cpu().numpy() for k, v in nxt.items()}
        arrs["hist"] = hists[lvl % 2][: max(kc, 1)].cpu().numpy()
        arrs["hist_k"] = np.array([kc], np.int64)
        arrs["pos_rec"] = be.pos_rec.cpu().numpy()
        arrs["pos_st"] = be.pos_st.cpu().numpy()
        arrs["jobs"] = ws["jobs"][: max(jc, 1)].cpu().numpy()
        arrs["job_count"] = np.array([jc], np.int64)
        arrs["idx"] = be.idx.cpu().numpy()
        arrs["tmp"] = be.tmp.cpu().numpy()
        arrs["own_state"] = ws["own_state"].cpu().numpy()  # subtree ownership (per rank)
        arrs["own_ranges"] = ws["own_ranges"].cpu().numpy()
        self.ckpt.save_device(lvl, arrs, rank, P)

    def _ckpt_restore(self, st, ws, sets, hists):
        """Load a saved level's state into the workspace; returns that level."""
        be = self.be
        lvl = int(st["level"][0])
        dev = be.device

        def put(dst, a):
            dst.copy_(torch.from_numpy(np.ascontiguousarray(a)).to(dev))

        for k, v in sets[(lvl + 1) % 2].items():
            put(v, st["set_" + k])
        kc = int(st["hist_k"][0])
        if kc:
            put(hists[lvl % 2][:kc], st["hist"])
        put(be.pos_rec, st["pos_rec"])
        put(be.pos_st, st["pos_st"])
        jc = int(st["job_count"][0])
        if jc:
            put(ws["jobs"][:jc], st["jobs"][:jc])
        ws["job_count"].fill_(jc)
        put(be.idx, st["idx"])
        put(be.tmp, st["tmp"])
        if "own_state" in st:
            put(ws["own_state"], st["own_state"])
            put(ws["own_ranges"], st["own_ranges"])
        return lvl

    # ------------------------------------------------------------ buffers
    def _lists(self, KMAX, IMAX, TMAX, MMAX, C, reg, dev):
        i64 = dict(dtype=torch.int64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        k_reg = KMAX if reg else 1
        return dict(
            pos=torch.empty(KMAX, **i64), start=torch.empty(KMAX, **i64),
            cnt=torch.empty(KMAX, **i32), depth=torch.empty(KMAX, **i32),
            stats=torch.empty((1 if reg else KMAX, C), **i32),
            items=torch.empty((IMAX, 4), **i64),
            red=torch.empty((KMAX, 3), **i64), der=torch.empty((KMAX, 3), **i64),
            tasks=torch.empty((TMAX, 3), **i64), ctl=torch.zeros(16, **i32),
            stats64=torch.empty((k_reg, 2), **i64), minmax=torch.empty((k_reg, 2), **i64),
            mitems=torch.empty((MMAX if reg else 1, 3), **i64),
            gcnt=torch.empty(KMAX, **i32), src=torch.empty(KMAX, **i32),
        )

    @staticmethod
    def _owners(J: int, P: int, device) -> torch.Tensor:
        """Serpentine job owners over the largest-first order (0..P-1, P-1..0, ...):
        near-even row totals, identical on every rank (the order is total)."""
        k = torch.arange(J, device=device)
        lap, off = k // P, k % P
        return torch.where(lap % 2 == 0, off, P - 1 - off)

    def _run_jobs(self, d_jobs, n: int, counter=None, split: bool = True):
        """Finish the (largest-first) job list; with several ranks and ``split``
        each takes its serpentine share (subtree ownership: the list is this
        rank's already)."""
        be, comm = self.be, self.comm
        if comm is not None and comm.world_size > 1 and split:
            owner = self._owners(d_jobs.shape[0], comm.world_size, d_jobs.device)
            d_jobs = d_jobs[owner == comm.rank]
            counter = None
        J = int(d_jobs.shape[0])
        if J:
            be.launch_finisher(d_jobs.contiguous(), J, n, self.p, be.pos_rec, be.pos_st,
                               counter, share=int(getattr(comm, "world_size", 1) or 1))

    def _job_segs(self, d_jobs) -> torch.Tensor:
        """The finisher jobs' position ranges and owners, int64 [J][3] = {lo, hi,
        owner} (a job of r rows owns 2r - 1 positions from its root; owners
        serpentine over the largest-first order, as ``_dp_finish`` sends them)."""
        J = int(d_jobs.shape[0])
        lo = d_jobs[:, 3]
        own = self._owners(J, self.comm.world_size, d_jobs.device).to(torch.int64)
        return torch.stack([lo, lo + 2 * d_jobs[:, 1] - 1, own], 1).contiguous()

    def _dp_finish(self, d_jobs, W: int):
        """Data-parallel subtree finishing: each job's rows are spread over the
        ranks; every rank sends its share of job j to owner(j) (serpentine over
        the largest-first order; one all_to_all of row-major codes + targets),
        the owner lays its jobs' rows out contiguously and runs the finisher on
        them (into the shared position space). The routing -- owners, send
        offsets, per-rank counts, the owned jobs' layout -- runs on the device
        (``dp_route.hip``); the one host wait reads the all_to_all split sizes.
        Jobs: int64 [J][W] = {local start, rows, depth, pos, buffer, stats[C],
        local rows, src}."""
        be, comm, p = self.be, self.comm, self.p
        hip = be.hip
        dev = be.device
        s = hb._stream
        P, r = comm.world_size, comm.rank
        C = be.C
        J = int(d_jobs.shape[0])
        d_jobs = d_jobs.contiguous()
        i64 = dict(dtype=torch.int64, device=dev)
        note = getattr(comm, "note_phase", None)  # (tracing / simulated communicators)
        if note is not None:
            note("dp_finish")
        # every rank's local rows per job: [P, J]
        allc = torch.empty(P * J, **i64)
        comm.all_gather_device(allc, d_jobs[:, 5 + C].contiguous())
        soff = torch.empty(J, **i64)
        hdr = torch.empty(4 + 2 * P, **i64)
        jobs2 = torch.empty((J // P + 2, 5 + C), **i64)  # (owned: ceil(J / P))
        seg = torch.empty((P * (J // P + 2), 3), **i64)
        hip.dp_plan(s(), d_jobs.data_ptr(), J, W, C, allc.data_ptr(), P, r, soff.data_ptr(),
                    hdr.data_ptr(), jobs2.data_ptr(), seg.data_ptr())
        rb = int(be.row_elems * be.cb)
        n_send = int(be.n)  # (every local row belongs to at most one job)
        codes_s = hb._workspace(dev, "dp.send", n_send * rb)
        ysz = be.y.element_size()
        # (slice first: a grown workspace need not be a multiple of the element size)
        y_s = hb._workspace(dev, "dp.send_y", n_send * ysz)[: n_send * ysz].view(be.y.dtype)
        y64 = be.y.dtype == torch.int64
        hip.dp_gather(s(), d_jobs.data_ptr(), J, W, C, be.idx.data_ptr(), be.tmp.data_ptr(),
                      int(be.row_mask), be.codes_rm.data_ptr(), rb, be.y.data_ptr(), y64,
                      soff.data_ptr(), codes_s.data_ptr(), y_s.data_ptr(),
                      int(min(max(p.finisher_rows, 1), be.n)))
        h = hb._pinned_copy(hdr, "dp.hdr")
        torch.cuda.current_stream(dev).synchronize()  # (the split sizes, for the host)
        Jm, R_tot = int(h[0]), int(h[1])
        sc = [int(v) for v in h[4 : 4 + P]]
        rc = [int(v) for v in h[4 + P : 4 + 2 * P]]
        n_out = sum(sc)
        codes_r = torch.empty(max(R_tot, 1) * rb, dtype=torch.uint8, device=dev)
        y_r = torch.empty(max(R_tot, 1), dtype=be.y.dtype, device=dev)
        comm.all_to_all_device(codes_r[: R_tot * rb], codes_s[: n_out * rb],
                               [v * rb for v in rc], [v * rb for v in sc])
        comm.all_to_all_device(y_r[:R_tot], y_s[:n_out], rc, sc)
        self.stats["dp_rows_exchanged"] = n_out
        if Jm == 0:
            return
        codes2 = torch.empty((R_tot, be.row_elems), dtype=be.codes_rm.dtype, device=dev)
        codes_fm = torch.empty((be.F, R_tot), dtype=be.codes_rm.dtype, device=dev)
        y2 = torch.empty(R_tot, dtype=be.y.dtype, device=dev)
        # both code layouts the finisher reads, in one pass over the received rows
        hip.dp_place(s(), seg.data_ptr(), P * Jm, codes_r.data_ptr(), y_r.data_ptr(), y64, rb,
                     R_tot, be.F, int(be.cb), codes2.data_ptr(), codes_fm.data_ptr(),
                     y2.data_ptr())
        be2 = getattr(self, "_dp_be", None)
        if be2 is None or be2.device != dev:
            be2 = self._dp_be = hb.HipBackend(dev)
        be2.setup(codes2, codes_fm, y2, be.nbins, n_bins=be.B, n_classes=C, criterion=be.crit)
        be2.launch_finisher(jobs2[:Jm], Jm, R_tot, p, be.pos_rec, be.pos_st, share=P)
        self._dp_keep = (codes_r, y_r, codes2, y2, codes_fm, jobs2, seg)

    def _exchange_nodes(self):
        """Every rank ends with every finished node: compact the positions this
        rank's finisher wrote ({pos, record[6], counts[C]} rows), all-gather
        them and scatter into the local position space. Level nodes are on
        every rank already and every job has one owner (the job order is a
        total order, see ``job_sort_kernel``), so each position has exactly
        one writer."""
        be, comm = self.be, self.comm
        dt = torch.int64 if be.reg else torch.int32  # regression sums need 64 bits
        grown = be.pos_rec[:, 5] > 0
        pre = getattr(self, "_pre_live", None)
        if pre is not None:
            grown &= ~pre
            self._pre_live = None
        live = torch.nonzero(grown).squeeze(1)
        rows = torch.cat([live.to(dt)[:, None], be.pos_rec[live].to(dt),
                          be.pos_st[live].to(dt)], 1)
        allr = comm.all_gather_rows(rows)
        pos = allr[:, 0].long()
        be.pos_rec.index_copy_(0, pos, allr[:, 1:7].to(torch.int32).contiguous())
        be.pos_st.index_copy_(0, pos, allr[:, 7:].to(be.pos_st.dtype).contiguous())

    def _exchange_owned(self, ws):
        """Subtree ownership: this rank wrote every position inside its owned
        ranges (the switch level's LPT units) and nothing else differs between
        ranks (:func:`exchange_ranges`)."""
        self._keep_x = exchange_ranges(self.be, self.comm, ws["own_ranges"],
                                       2 * int(self.stats.get("own_rows", self.be.P)) + 16)

    def _level_profile(self, marks):
        """Per-level device times (ms) from the HIP events (MPITREE_PROFILE=1)."""
        names = ("hist", "derive", "scan", "plan", "partition")
        marks[-1][-1].synchronize()
        rows = []
        for m in marks:
            d = {k: m[i].elapsed_time(m[i + 1]) for i, k in enumerate(names) if i + 1 < len(m)}
            rows.append(d)
            for k, v in d.items():
                self.timings["device_" + k] = self.timings.get("device_" + k, 0.0) + v / 1e3
        self.stats["level_profile"] = rows

    @staticmethod
    def _ptrs(lists) -> dict:
        return {k: v.data_ptr() for k, v in lists.items()}

    # --------------------------------------------------------------- fit
    def _workspace(self, key, make):
        """Level-loop buffers, reused by consecutive fits of one shape (the
        allocations and pinned buffers cost more host time than a level)."""
        ws = _WORKSPACES.pop(key, None)
        if ws is None:
            ws = make()
        _WORKSPACES[key] = ws  # most recently used last
        while len(_WORKSPACES) > 2:
            _WORKSPACES.pop(next(iter(_WORKSPACES)))
        return ws

    def _mode(self, F: int):
        """(feature-parallel?, data-parallel?, subtree ownership?, f_lo, f_hi) of
        this rank."""
        comm = self.comm
        P = getattr(comm, "world_size", 1)
        kind = getattr(comm, "kind", "local")
        if P <= 1:
            return False, False, False, 0, F
        if kind == "data":
            if F >= P:  # the built histograms are reduced to their feature block's owner
                lo, hi = feature_blocks(F, P)[int(comm.rank)]
                return False, True, False, int(lo), int(hi)
            return False, True, False, 0, F
        if kind == "feature" and F >= P:
            lo, hi = comm.feature_range(F)
            return True, False, False, int(lo), int(hi)
        # "subtree" / "auto": replicated levels, then each rank grows the units
        # the switch level's LPT gives it
        return False, False, True, 0, F

    def fit(self, n: int, n_classes: int, n_features: int, edges, y_exp: int = 0,
            root=None, d_edges=None) -> TreeArrays:
        """Grow the tree. ``n``: this rank's rows (all rows unless data-parallel);
        ``edges``: host edge table ``[F, W]`` or a BinMapper (only materialised
        when ``d_edges``, the device copy, is absent); ``root``: root statistics
        when the caller already has them (gpu_prepare), which saves a device
        round trip."""
        be, p, comm = self.be, self.p, self.comm
        hip = be.hip
        dev = be.device
        reg = bool(be.reg)
        C, F, B = (2 if reg else n_classes), n_features, be.B
        fr = int(p.finisher_rows)
        md = -1 if p.max_depth is None else int(p.max_depth)
        mss, msl = int(p.min_samples_split), int(max(1, p.min_samples_leaf))
        fp, dp, own, f_lo, f_hi = self._mode(F)
        F_h = f_hi - f_lo
        P = getattr(comm, "world_size", 1)
        # subtree ownership: the replicated levels before the switch run
        # feature-parallel -- each rank histograms and scans its feature block
        # only, one all-gather of the split records per level (fp_combine), and
        # the switch level builds every child of the first owned level from rows
        fpx = own and F >= P and self.ckpt is None and fp_prefix_pays(int(n), F, P, reg)
        x_lo, x_hi = feature_blocks(F, P)[int(comm.rank)] if fpx else (0, F)
        # data-parallel with >= P features: built histograms reduced per feature
        # block to the block's owner (reduce-scatter by feature), scans per block
        dprs = dp and F_h < F
        blocks = feature_blocks(F, P) if dprs else None
        # equal blocks: every rank's built histograms laid out block-major in one
        # buffer and summed with ONE reduce-scatter per level (P reduces to the
        # blocks' owners paid P collective latencies)
        rs_one = (dprs and len({hi - lo for lo, hi in blocks}) == 1
                  and hasattr(comm, "reduce_scatter_device")
                  and os.environ.get("MPITREE_DP_REDUCE_SCATTER", "1") != "0")
        # ... built in ONE pass over this rank's rows (all features, node-major) and
        # permuted block-major on the device, instead of P passes of one block each
        one_build = rs_one and os.environ.get("MPITREE_DP_ONE_BUILD", "1") != "0"
        F_slab = F if one_build else F_h  # (item slabs of a full-width build)
        s = hb._stream
        t0 = time.perf_counter()
        n_loc = int(n)
        if root is None:
            root_full = be.segment_stats(np.array([0]), np.array([n_loc]))[0]  # one small sync
        else:
            root_full = np.asarray(root, dtype=np.int64)
        if dp:  # global root statistics and row count (one small host collective)
            root_full = comm.reduce_stats(np.asarray(root_full, np.int64)[None, :], reg)[0]
        n = int(root_full[0]) if reg else int(np.sum(root_full))  # global rows
        be.begin_positions(2 * n - 1)
        if reg:  # {count, sum, min, max}: a root with equal targets is a leaf
            root = root_full[:2]
            pure = root_full[2] == root_full[3]
        else:
            root = root_full
            pure = int((root > 0).sum()) <= 1
        root_term = (md == 0) or n < mss or n < 2 * msl or pure
        W = 5 + C + (2 if dp else 0)  # finisher job row width (dp: + local rows, src)
        jobs_host = None
        if root_term:
            be.put_positions([0], [-1], [-1], [-1], [-1], [0], [n], root[None, :])
        elif n <= fr:  # the whole tree is one finisher job
            row = [0, n, 0, 0, 0] + list(root) + ([n_loc, 0] if dp else [])
            jobs_host = np.asarray(row, np.int64)[None, :]
        self.timings["stats"] = time.perf_counter() - t0
        levels = 0
        J = 0
        t0 = time.perf_counter()
        comm_bytes = []
        shared = None
        if not root_term and jobs_host is None:
            KMAX = n // (fr + 1) + 2
            IMAX = KMAX + n_loc // 1024 + 2 * hb.N_CU + 16
            PMAX = KMAX + n_loc // 1024 + 16
            JMAX = n // 2 + 2
            R = 7 if reg else 5 + 2 * C
            # multi-item nodes hold > max(1024, level rows / 512) rows each
            RMAX = int(min(KMAX, max(2 * hb.N_CU + 1, n_loc // 1024 + 1)))
            TMAX = RMAX + IMAX // 16 + 16
            MMAX = KMAX + n_loc // 4096 + 16
            E = F_h * B * C
            hdt = torch.int64 if reg else torch.int32
            # two classes, <= 256 bins, no collective between scan and plan: the
            # planner builds the split records from the scan's per-feature results
            # (no select launch)
            fsel = (not (reg or dp or fp) and bool(hip.scan_fused_select_ok(B, C, int(be.crit)))
                    and os.environ.get("MPITREE_FUSED_SELECT", "1") != "0")
            dfree = derive_free_levels(n_loc, F_h, B, C, reg, fr, hip, dev)
            if dfree:
                self.stats["derive_free"] = True

            def make():
                i64 = dict(dtype=torch.int64, device=dev)
                return dict(
                    sets=[self._lists(KMAX, IMAX, TMAX, MMAX, C, reg, dev) for _ in range(2)],
                    hists=[torch.empty((KMAX, F_h, B, C), dtype=hdt, device=dev)
                           for _ in range(1 if dfree else 2)] * (2 if dfree else 1),
                    slab=torch.empty((min(IMAX, slab_rows(n_loc)),
                                      hip.hist_slab_words(F_slab, B, C, reg)), dtype=hdt,
                                     device=dev),
                    rec=torch.empty((KMAX, R), **i64),
                    grec=torch.empty((P * KMAX * R) if (fp or dprs or fpx) else 1, **i64),
                    # the other ranks' feature blocks of this rank's built histograms
                    rs=[torch.empty((KMAX, hi - lo, B, C), dtype=hdt, device=dev)
                        if r != int(comm.rank) else None
                        for r, (lo, hi) in enumerate(blocks)] if dprs and not rs_one else None,
                    rsb=torch.empty(P * KMAX * F_h * B * C, dtype=hdt, device=dev)
                    if rs_one else None,
                    hall=torch.empty(KMAX * F * B * C, dtype=hdt, device=dev)
                    if one_build else None,
                    cost=torch.empty((KMAX, F_h), dtype=torch.float64, device=dev),
                    bins=torch.empty((KMAX, F_h), dtype=torch.int32, device=dev),
                    ident=torch.arange(KMAX, **i64),
                    split=torch.empty((KMAX, 4), **i64),
                    pitems=torch.empty((PMAX, 3), **i64),
                    cursors=torch.empty((KMAX, 2), dtype=torch.int32, device=dev),
                    jobs=torch.empty((JMAX, W), **i64),
                    jobs_sorted=torch.empty((min(JMAX, hip.job_sort_max()), W), **i64),
                    job_count=torch.zeros(1, dtype=torch.int32, device=dev),
                    fin_counter=torch.zeros(128, dtype=torch.int32, device=dev),
                    root=torch.empty(4 if reg else C, **i64),
                    root_host=torch.empty(4 if reg else C, dtype=torch.int64, pin_memory=True),
                    own_state=torch.zeros(4, dtype=torch.int32, device=dev),
                    own_ranges=torch.zeros((OWN_CAP if own else 1, 2), **i64),
                    own_node=torch.empty(KMAX if own else 1, dtype=torch.int32, device=dev),
                    own_job=torch.empty(JMAX if own else 1, dtype=torch.int32, device=dev),
                    # every unit's child segments {lo, hi, owner} (shared-host assembly)
                    own_segs=torch.zeros((2 * OWN_CAP if own else 1, 3), **i64),
                    # fused selection: per-feature left counts and node totals (scan)
                    sel_left=torch.empty((KMAX, F_h, 2) if fsel else 1, dtype=torch.int32,
                                         device=dev),
                    sel_tot=torch.empty((KMAX, 4) if fsel else 1, dtype=torch.int32,
                                        device=dev),
                )

            ws = self._workspace((str(dev), n, n_loc, F, f_lo, F_h, B, C, reg, fr, dp, own, fsel,
                                  fpx, dfree, rs_one, one_build), make)
            sets, hists, slab, rec = ws["sets"], ws["hists"], ws["slab"], ws["rec"]
            cost, bins, ident, split = ws["cost"], ws["bins"], ws["ident"], ws["split"]
            pitems, cursors, jobs, job_count = (ws["pitems"], ws["cursors"], ws["jobs"],
                                                ws["job_count"])
            hctl_dev, hctl = _host_ctl(hip, dev)
            _FIT_SEQ[0] = (_FIT_SEQ[0] + 1) % (1 << 18)
            tag0 = _FIT_SEQ[0] << 12
            ptrs = [self._ptrs(x) for x in sets]
            ck, rank = self.ckpt, int(getattr(comm, "rank", 0))
            state = None
            if ck is not None:
                ck.layout = (f"device fr={fr} K={KMAX} I={IMAX} J={JMAX} T={TMAX} M={MMAX} "
                             f"F={F_h}@{f_lo} W={W} dfree={int(dfree)}")
                state = ck.load_device(rank, P, (lambda a: comm._all_gather(a)) if P > 1
                                       else None)
            first_lvl = 0  # levels before it ran in an earlier process (resume)
            if own:  # (subtree ownership: not switched yet)
                ws["own_state"].zero_()
            if state is not None:
                first_lvl = self._ckpt_restore(state, ws, sets, hists) + 1
                self.stats["resumed_from_level"] = first_lvl - 1
                del state
            else:
                # level 0: the root, built from rows (one init launch; root stats H2D)
                chunk = int(min(hb.MAX_ITEM_ROWS,
                                max(1024, -(-n_loc // (hist_items_per_cu(reg) * hb.N_CU)))))
                ws["root_host"].numpy()[: root_full.size] = root_full
                ws["root"].copy_(ws["root_host"], non_blocking=True)
                hip.grow_init(s(), ptrs[0], n_loc, n, chunk, C, int(reg), ws["root"].data_ptr(),
                              job_count.data_ptr())
            ck_every = max(1, int(os.environ.get("MPITREE_CKPT_EVERY", "1")))
            cb, rs = be.cb, be.row_elems * be.cb
            bufs = (be.idx.data_ptr(), be.tmp.data_ptr())
            lvl = first_lvl
            done_at = None
            prof = profiling()
            marks = []  # per level: events at start and after hist, derive, scan, plan, partition

            def mark():
                if prof:
                    e = torch.cuda.Event(enable_timing=True)
                    e.record()
                    marks[-1].append(e)

            own_args = {}
            if own:
                own_args = dict(P=P, rank=rank, min_units=own_min_units(P), cap=OWN_CAP,
                                state=ws["own_state"].data_ptr(),
                                ranges=ws["own_ranges"].data_ptr(),
                                node_owner=ws["own_node"].data_ptr(),
                                job_owner=ws["own_job"].data_ptr(),
                                jobs_at_switch=own_jobs_at_switch(be),
                                segs=ws["own_segs"].data_ptr(), build_all=int(fpx))

            # (the planner makes 2 items per "CU")
            plan_cu = hb.N_CU * hist_items_per_cu(reg) // 2
            # single-rank and subtree-ownership levels (no collective between the
            # kernels, no per-phase profile events): one C++ call enqueues a level
            ctx = None
            if not (dp or fp or prof) and os.environ.get("MPITREE_LEVEL_CTX", "1") != "0":
                # the workspace's context is reused when nothing but the host slot
                # tag differs from the last fit (building its ~60 fields costs ~30 us
                # of host time while the GPU waits for the first level)
                ctx_key = (bufs, be.codes_rm.data_ptr(), be.codes_fm.data_ptr(),
                           be.y.data_ptr(), be.pos_rec.data_ptr(), be.pos_st.data_ptr(),
                           be.nbins.data_ptr(), be.xtab.data_ptr(), hctl_dev, cb, rs,
                           be.lab_shift, be.row_mask, be.n, int(be.crit), md, mss, msl,
                           plan_cu, hb.LDS_BUDGET, tuple(sorted(own_args.items())))
                cached = ws.get("ctx")
                if cached is not None and cached[0] == ctx_key:
                    ctx = cached[1]
                    ctx.set_tag0(tag0)
            if ctx is None and not (dp or fp or prof) and os.environ.get(
                    "MPITREE_LEVEL_CTX", "1") != "0":
                ctx = hip.GrowCtx(dict(
                    hist0=hists[0].data_ptr(), hist1=hists[1].data_ptr(), idx=bufs[0],
                    tmp=bufs[1], codes_rm=be.codes_rm.data_ptr(),
                    codes_fm=be.codes_fm.data_ptr(), y=be.y.data_ptr(), slab=slab.data_ptr(),
                    rec=rec.data_ptr(), cost=cost.data_ptr(), bins=bins.data_ptr(),
                    ident=ident.data_ptr(), split=split.data_ptr(), pitems=pitems.data_ptr(),
                    cursors=cursors.data_ptr(), jobs=jobs.data_ptr(),
                    job_count=job_count.data_ptr(), pos_rec=be.pos_rec.data_ptr(),
                    pos_st=be.pos_st.data_ptr(), nbins=be.nbins.data_ptr(),
                    xtab=be.xtab.data_ptr(), xtab_n=hb.XTAB_N, host_ctl=hctl_dev, cb=cb,
                    row_bytes=rs, lab_shift=be.lab_shift, row_mask=be.row_mask, n_codes=be.n,
                    n_loc=n_loc, F_h=F_h, f_lo=f_lo, B=B, C=C, reg=int(reg), crit=int(be.crit),
                    E=E, max_depth=md, mss=mss, msl=msl, fr=fr, n_cu=plan_cu,
                    lds_budget=hb.LDS_BUDGET, KMAX=KMAX, IMAX=IMAX, TMAX=TMAX, RMAX=RMAX,
                    PMAX=PMAX, MMAX=MMAX, tag0=tag0, derive_free=int(dfree),
                    **(dict(sel_left=ws["sel_left"].data_ptr(), sel_tot=ws["sel_tot"].data_ptr())
                       if fsel else {})), ptrs[0], ptrs[1], own_args)
                ws["ctx"] = (ctx_key, ctx)

            def plan(cur, nxt, lvl, fixup=False):
                hip.grow_plan(s(), cur, nxt, rec.data_ptr(), split.data_ptr(), pitems.data_ptr(),
                              cursors.data_ptr(), cur["ctl"] + 4 * 5, be.pos_rec.data_ptr(),
                              0 if reg else be.pos_st.data_ptr(),
                              be.pos_st.data_ptr() if reg else 0, int(reg), (lvl + 1) % 2,
                              jobs.data_ptr(), job_count.data_ptr(), C, md, plan_cu, mss, msl,
                              fr, 0 if fixup else hctl_dev + (lvl % 64) * 64,
                              tag0 + (lvl % 4096) + 1, dp=int(dp), fixup=fixup, own=own_args,
                              derive_free=int(dfree))

            fpx_on = fpx  # (until the switch: feature-parallel levels)
            # a level can switch only once it has min_units units (<= 2^level)
            x_first = max(0, int(np.ceil(np.log2(max(1, own_min_units(P)))))) if fpx else 0
            while True:
                if P > 1:  # failure containment: a failed peer / injected fault
                    check_abort()
                    fault_point(comm, f"level:{lvl}")
                b0 = getattr(comm, "bytes_communicated", 0)
                if ctx is not None and not fpx_on:
                    ctx.level(s(), lvl)
                    if hb._DEFERRED:  # (host work of the setup, now that the GPU is busy)
                        hb.run_deferred()
                    if REC_DUMP is not None:  # (tools: per-level split records)
                        REC_DUMP.append(rec[: int(min(2 ** min(lvl, 40), KMAX))].clone())
                    if DUMP is not None:
                        kbd = int(min(2 ** min(lvl, 40), KMAX))
                        DUMP.setdefault("hists", []).append(hists[lvl % 2][:kbd].clone())
                    if ck is not None and (lvl - first_lvl + 1) % ck_every == 0:
                        self._ckpt_save(lvl, ws, sets, hists, rank, P)
                    lvl += 1
                    if lvl - 2 >= first_lvl:
                        _wait_slot(hctl, (lvl - 2) % 64, tag0 + ((lvl - 2) % 4096) + 1)
                        if int(hctl[(lvl - 2) % 64, 0]) == 0:
                            done_at = lvl - 2
                            break
                    if lvl > 4096:
                        raise RuntimeError("device level loop did not terminate")
                    continue
                if prof:
                    marks.append([])
                    mark()
                cur, nxt = ptrs[lvl % 2], ptrs[(lvl + 1) % 2]
                nxt_t = sets[(lvl + 1) % 2]
                H, Hp = hists[lvl % 2], hists[(lvl + 1) % 2]
                l_lo, l_F = (x_lo, x_hi - x_lo) if fpx_on else (f_lo, F_h)
                if fpx_on:  # this rank's feature block, node-major
                    H = H.view(-1)[: KMAX * l_F * B * C].view(KMAX, l_F, B, C)
                    Hp = Hp.view(-1)[: KMAX * l_F * B * C].view(KMAX, l_F, B, C)
                kb = int(min(2 ** min(lvl, 40), KMAX))
                ib = int(min(IMAX, kb + n_loc // 1024 + 2 * hb.N_CU + 1))
                ctl = cur["ctl"]
                # rows alternate between the two permutation buffers level by level
                src, dst = bufs[lvl % 2], bufs[(lvl + 1) % 2]
                rb = int(min(kb, RMAX))
                if dp:  # built slots <= splits of the previous level (lagged read)
                    if lvl - 2 >= first_lvl:
                        nbb = int(hctl[(lvl - 2) % 64, 0])
                    else:
                        nbb = 1 if lvl < 2 else KMAX  # (resumed: no lagged value yet)
                    nbb = max(1, min(nbb, KMAX))

                def build(Ht, lo, nf):
                    # classification: the hist launch also zeroes the slots the slab
                    # reduction adds into (one launch less per level)
                    hip.hist(s(), be.codes_rm.data_ptr(), cb, rs, src, be.y.data_ptr(),
                             be.lab_shift, cur["items"], ib, Ht.data_ptr(), slab.data_ptr(), nf,
                             lo, B, C, reg, hb.LDS_BUDGET, dcount=ctl + 4 * 2,
                             zred=0 if reg else cur["red"], zred_bound=0 if reg else rb,
                             zcount=0 if reg else ctl + 4 * 3)
                    if reg:  # slabs summed straight into the slot
                        hip.hist_reduce(s(), cur["red"], rb, 1, slab.data_ptr(), Ht.data_ptr(),
                                        nf, B, C, True, dcount=ctl + 4 * 3)
                    else:
                        hip.hist_reduce_tasks(s(), cur["red"], rb, cur["tasks"],
                                              int(min(TMAX, rb + ib // 16 + 1)), slab.data_ptr(),
                                              Ht.data_ptr(), nf, B, C, ctl + 4 * 3, ctl + 4 * 7,
                                              zero=False)

                if rs_one:
                    # every block's built slots, block-major, then one reduce-scatter:
                    # this rank's block of the global histograms lands in H
                    chunk = nbb * F_h * B * C
                    flat = ws["rsb"]
                    if one_build:
                        Hall = ws["hall"][: nbb * F * B * C].view(nbb, F, B, C)
                        build(Hall, 0, F)
                        flat[: P * chunk].view(P, nbb, F_h * B * C).copy_(
                            Hall.view(nbb, P, F_h * B * C).transpose(0, 1))
                    else:
                        for r, (lo, hi) in enumerate(blocks):
                            build(flat[r * chunk : (r + 1) * chunk].view(nbb, F_h, B, C), lo,
                                  hi - lo)
                    comm.reduce_scatter_device(H.view(-1)[:chunk], flat[: P * chunk])
                elif dprs:
                    # block r of the built slots -> rank r, enqueued behind block r's
                    # kernels: the reduce of block r overlaps the build of block r + 1
                    works = []
                    for r, (lo, hi) in enumerate(blocks):
                        Hr = H if r == rank else ws["rs"][r]
                        build(Hr, lo, hi - lo)
                        works.append(comm.reduce_device(Hr[:nbb], r, async_op=True))
                    for w in works:
                        if w is not None:
                            w.wait()
                else:
                    build(H, l_lo, l_F)
                    if dp:  # sum the built slots' histograms over the row shards
                        comm.all_reduce_device(H[:nbb])
                mark()
                # classification: the scan derives the larger siblings itself
                # (parent - built sibling, written back for select / next level)
                fuse = lvl > 0 and not reg
                if lvl > 0 and reg:
                    hip.hist_derive(s(), cur["der"], kb, Hp.data_ptr(), H.data_ptr(),
                                    l_F * B * C, reg, dcount=ctl + 4 * 4)
                hip.scan(s(), H.data_ptr(), ident.data_ptr(), kb, be.nbins.data_ptr(), l_F, l_lo,
                         B, C, int(be.crit), msl, cost.data_ptr(), bins.data_ptr(),
                         rec.data_ptr(), be.xtab.data_ptr(), hb.XTAB_N, dcount=ctl,
                         der=cur["der"] if fuse else 0, prev=Hp.data_ptr() if fuse else 0,
                         nbuilt=ctl + 4 * 1 if fuse else 0,
                         node_tot=0 if reg else cur["stats"])
                if fp or dprs or fpx_on:  # every rank's best split of each node -> the global best
                    g = ws["grec"][: P * kb * R]
                    comm.all_gather_device(g, rec[:kb].reshape(-1))
                    hip.fp_combine(s(), g.data_ptr(), P, kb, R, ctl, rec.data_ptr())
                mark()
                plan(cur, nxt, lvl)
                if hb._DEFERRED:
                    hb.run_deferred()
                mark()
                pb = int(min(PMAX, n_loc // 1024 + kb + 1))
                hip.partition(s(), be.codes_fm.data_ptr(), cb, be.n, src, dst, be.row_mask,
                              pitems.data_ptr(), pb, split.data_ptr(), cursors.data_ptr(),
                              dcount=ctl + 4 * 6, copy_back=False)
                if dp:  # local segments of the next frontier / new jobs, then its work items
                    plan(cur, nxt, lvl, fixup=True)
                if reg:  # purity of the next frontier, read by the next planner
                    kbn = int(min(2 * kb, KMAX))
                    hip.seg_minmax(s(), dst, be.y.data_ptr(), nxt["mitems"],
                                   int(min(MMAX, 2 * kb + n_loc // 4096 + 1)), nxt["minmax"],
                                   nxt["ctl"] + 4 * 8)
                    if dp:  # global min / max: one MAX all-reduce of (-min, max)
                        mm = nxt_t["minmax"][:kbn]
                        mm[:, 0].neg_()
                        comm.all_reduce_device(mm, op=torch.distributed.ReduceOp.MAX)
                        mm[:, 0].neg_()
                mark()
                if comm is not None and P > 1:
                    comm_bytes.append(int(getattr(comm, "bytes_communicated", 0) - b0))
                if ck is not None and (lvl - first_lvl + 1) % ck_every == 0:
                    self._ckpt_save(lvl, ws, sets, hists, rank, P)
                # lagged completion check: the planner stored the next level's
                # frontier size + job count into host slot lvl % 64
                lvl += 1
                if fpx_on and lvl - 1 >= x_first:
                    # the next level's kernels depend on whether this one switched:
                    # wait for its planner (levels that cannot switch keep the lag)
                    L = lvl - 1
                    _wait_slot(hctl, L % 64, tag0 + (L % 4096) + 1)
                    self.stats["fp_prefix_levels"] = L + 1
                    if int(hctl[L % 64, 0]) == 0:
                        done_at = L
                        break
                    if int(hctl[L % 64, 3]):  # switched: own levels (all features) follow
                        fpx_on = False
                    continue
                if lvl - 2 >= first_lvl:
                    _wait_slot(hctl, (lvl - 2) % 64, tag0 + ((lvl - 2) % 4096) + 1)
                    if int(hctl[(lvl - 2) % 64, 0]) == 0:
                        done_at = lvl - 2
                        break
                if lvl > 4096:
                    raise RuntimeError("device level loop did not terminate")
            levels = done_at + 1
            J = int(hctl[done_at % 64, 1])  # finisher jobs appended (own: this rank's)
            switched = bool(own and hctl[done_at % 64, 3])
            if prof:
                self._level_profile(marks[:levels])
            if switched:  # this rank's units: every job is its own, ranges to exchange
                self._owned = ws
                self.stats["own_units"] = int(hctl[done_at % 64, 4])
                self.stats["own_rows"] = int(hctl[done_at % 64, 5])
            elif P > 1:  # positions the (replicated) level loop decided: on every rank already
                self._pre_live = be.pos_rec[:, 5] > 0
            if J:
                counter = None
                if J <= hip.job_sort_max():  # one-workgroup sort, zeroes the counters too
                    d_jobs = ws["jobs_sorted"][:J]
                    counter = ws["fin_counter"]
                    hip.job_sort(s(), jobs.data_ptr(), J, W, d_jobs.data_ptr(),
                                 counter.data_ptr())
                else:
                    # largest first, ties by root position (the kernel's total order)
                    order = torch.argsort(jobs[:J, 1] * (1 << 32) - jobs[:J, 3],
                                          descending=True)
                    d_jobs = jobs[:J].index_select(0, order)
                if DUMP is not None:
                    DUMP.update(jobs=d_jobs.clone(), idx=be.idx.clone(), tmp=be.tmp.clone(),
                                row_mask=int(be.row_mask))
                if dp:
                    self._dp_finish(d_jobs, W)
                    self._dp_segs = self._job_segs(d_jobs)
                else:
                    self._run_jobs(d_jobs, n, counter, split=not switched)
        elif jobs_host is not None:
            J = 1
            (d_jobs,) = be.up(jobs_host)
            if P > 1 and not own:
                self._pre_live = be.pos_rec[:, 5] > 0
            if dp:
                self._dp_finish(d_jobs.view(1, -1), W)
                self._dp_segs = self._job_segs(d_jobs.view(1, -1))
            else:  # (ownership: one job -- every rank grows it, nothing to exchange)
                self._run_jobs(d_jobs.view(1, -1), n, split=not own)
        if comm is not None and P > 1:
            check_abort()
            fault_point(comm, "exchange")  # (after the switch: peers wait in the exchange)
            t1 = time.perf_counter()
            b0 = comm.bytes_communicated
            owned = getattr(self, "_owned", None)
            dp_segs, self._dp_segs = getattr(self, "_dp_segs", None), None
            pool = None
            if owned is not None or (dp_segs is not None and
                                     dp_segs.shape[0] <= int(hip.shm_max_segs())):
                pool = shared_tree.pool_for(comm, hip)
            if dp_segs is not None and pool is not None:
                # data-parallel: every finisher job has one owner, whose finisher
                # wrote its positions; the owners write their jobs' nodes (rank 0
                # also the level nodes, on every rank alike) into the node-shared
                # host tree, as subtree ownership does (no node all-gather)
                shared = dict(comm=comm, pool=pool, segs=dp_segs, S=int(dp_segs.shape[0]))
                self.stats["assembly"] = "shared-host"
            elif owned is not None:
                # ranks of one node: each writes its own nodes into a shared host
                # buffer (no node exchange); otherwise one all-gather of the nodes
                if pool is not None:
                    shared = dict(comm=comm, pool=pool, segs=self._owned["own_segs"],
                                  S=2 * int(self.stats["own_units"]))
                    self.stats["assembly"] = "shared-host"
                else:
                    self._exchange_owned(self._owned)
            elif not (own and getattr(self, "_pre_live", None) is None):
                self._exchange_nodes()
            self._owned = None
            self.timings["exchange"] = time.perf_counter() - t1
            self.stats["comm_bytes_per_level"] = comm_bytes
            self.stats["comm_bytes_exchange"] = int(comm.bytes_communicated - b0)
            self.stats["mode"] = ("data" if dp else "feature" if fp
                                  else "subtree-owned" if own else "replicated")
            self.stats["feature_block"] = [f_lo, f_hi]
            if dp:
                self.stats["dp_reduce"] = ("reduce-scatter" if rs_one else
                                           "reduce-to-owner" if dprs else "all-reduce")
        self.timings["levels"] = time.perf_counter() - t0
        self.stats["levels"] = levels
        self.stats["finisher_subtrees"] = J
        t0 = time.perf_counter()
        # thresholds come from the device edge table (uploaded when absent)
        table = None
        if d_edges is None:
            table = edges if isinstance(edges, np.ndarray) else edges.padded_edges()
        b_asm = getattr(comm, "bytes_communicated", 0)
        ta = be.assemble_positions(table, int(p.criterion), y_exp, d_edges=d_edges,
                                   shared=shared)
        if ta is None:  # (/dev/shm too small for the tree, on every rank alike)
            self.stats["assembly"] = "exchange (/dev/shm short)"
            if owned is not None:
                self._exchange_owned(owned)
            else:
                self._exchange_nodes()
            ta = be.assemble_positions(table, int(p.criterion), y_exp, d_edges=d_edges)
        if shared is not None:  # (the shared assembly's segment-count all-gather)
            self.stats["comm_bytes_exchange"] = int(self.stats.get("comm_bytes_exchange", 0)
                                                    + comm.bytes_communicated - b_asm)
        self.timings["assemble"] = time.perf_counter() - t0
        if self.ckpt is not None:
            self.stats["checkpoint_levels_saved"] = self.ckpt.saved_levels
            self.ckpt.clear()
        self._dp_keep = None
        return ta
