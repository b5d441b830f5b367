"""Exact thresholds on continuous features: the device-driven presorted-list engine.

The reference scores every unique value of a feature as a threshold
(``mpitree/tree/decision_tree.py:73-90``) and splits its work by handing
subtrees to MPI sub-communicators (``:446-477``). The histogram engines are
exact only while a feature has at most 256 values; beyond that a GPU fit runs
this engine (``ops/csrc/exact2.hip``, classification and regression):

* setup: every feature column of this rank's block sorted once (a batched
  one-sweep radix sort of 32-bit value keys, ``exact_setup.hip``) into 4-byte list
  entries {row, duplicate flag, label} (+ the fixed-point targets for
  regression) and a per-row value-rank table;
* a fixed chain of launches per level (chunk totals, carries, scan, select,
  planner, flags, stable partition) whose work counts live in device memory:
  the host enqueues levels back to back and reads one lagged host-mapped slot
  per level to learn that the frontier is empty -- no per-level ``.cpu()``;
* segments of at most 256 rows leave as finisher jobs: subtree-local 8-bit
  codes (the offset of each value's first entry in the segment) feed the same
  histogram finishers as the binned engines.

Multi-GPU (one process per GPU, RCCL over xGMI; every rank holds all rows, the
reference's contract): **feature-parallel**. Rank r sorts, scans and partitions
only its contiguous feature block -- setup, scans and partitions all shrink
with 1/P -- and per level one ``all_gather`` of the per-node split records
(``fp_combine_kernel``: max gain, ties to the lowest feature) plus one
``all_reduce`` of the n-bit row-direction flags (the split feature's owner
sets them) keep the ranks in lock step. The jobs are split across ranks
(serpentine over the largest-first order), one ``all_to_all`` brings every rank
all features' finisher codes at its own jobs' positions, and one exchange of the
finished position ranges plus one of the thresholds each rank resolved leave
every rank with the same tree, equal to the single-GPU tree bit for bit.
Partition per level: count, per-segment prefix, grid-stride scatter (no
look-back chain; ``xe_part_count_kernel`` / ``xe_part_prefix_kernel``).
``fit(checkpoint=...)``: level resume (both list buffers, frontier, position
space, finisher jobs).
"""

from __future__ import annotations

import os
import time

import numpy as np
import torch

from . import hip_backend as hb
from .device_grower import _host_ctl, _wait_slot, _FIT_SEQ, exchange_ranges
from ..core.criterion import Criterion
from ..parallel.failure import check_abort, fault_point

__all__ = ["ExactGrower", "exact_supported", "needs_exact"]

MAX_ROWS = 1 << 24
_WS: dict = {}
_DEBUG_SYNC = os.environ.get("MPITREE_EXACT_SYNC", "0") != "0"
_DEBUG_STEP = os.environ.get("MPITREE_EXACT_SYNC") == "2"  # (+ a sync after every launch)


def _step(dev, what):
    if _DEBUG_STEP:
        torch.cuda.synchronize(dev)
        print(f"  exact: {what} done", flush=True)


def exact_supported(n: int, C: int, regression: bool) -> bool:
    """Rows index 24 bits of a list entry. Labels of up to 128 classes ride in
    the entries; more classes are gathered from a row-indexed label array."""
    from . import native

    if n >= MAX_ROWS:
        return False
    return regression or 1 <= C <= int(native.hip().xe_max_classes())


def exact_finisher_rows(F: int, C: int, regression: bool) -> int:
    """Rows of the largest segment the engine hands to a finisher job (0: its
    levels grow to the leaves -- the local-code finishers take <= 256 classes and
    the regression finisher <= 256 features)."""
    from . import native

    hip = native.hip()
    fr = int(hip.xe_local_max())
    if regression and F > 256:
        fr = 0
    if not regression and (C > 256 or int(hip.finish_feature_tile(F, 256, C)) <= 0):
        fr = 0
    return fr


def exact_workspace_bytes(n: int, F_loc: int, C: int, regression: bool, fr: int,
                          chunk: int, rec_width: int) -> int:
    """Device bytes of one fit's list engine on a rank holding ``F_loc`` features:
    the sorted lists (+ fixed-point targets), the setup sort's temporaries, the
    per-item / per-node level buffers (sized by ``KMAX = n / (fr + 1)``: with no
    finisher every level can hold ~n / 2 nodes, and the (items x features x
    classes) chunk totals and carries grow as n F C) and the position space."""
    KMAX = n // (fr + 1) + 2
    IMAX = KMAX + n // max(chunk, 1) + 2
    Cc = 1 if regression else max(int(C), 1)
    Cs = 2 if regression else max(int(C), 1)
    b = 0
    b += 2 * F_loc * n * 4 + F_loc * n * 4             # E[2], rank_at
    b += 4 * F_loc * n * 4                              # setup keys[2], rows[2]
    if regression:
        b += 2 * F_loc * n * 8                          # Y[2]
    b += 2 * IMAX * F_loc * Cc * 8                      # tot, carry
    b += IMAX * F_loc * (16 + 4) + 4 * IMAX * F_loc * 8  # cbest, cmin, pstat
    b += KMAX * (F_loc * 4 + rec_width * 8 + 64 + 2 * Cs * 8)  # nmin, rec, lists
    b += (2 * n) * (6 * 4 + Cs * 8 + 8)                 # position space + thresholds
    return int(b)


def exact_fits_memory(n: int, F: int, C: int, regression: bool, P: int = 1,
                      free_bytes: int | None = None, comm=None) -> bool:
    """Whether the list engine's workspace fits in half of the free device memory
    (else the fit takes 256 quantile bins: ADVICE r4 -- at 1M x 64 with 300
    classes the no-finisher chunk totals alone would need ~150 GB each). A
    workspace within 1/64 of the device needs no free-memory query; otherwise a
    multi-rank fit (``comm``) decides from the minimum over the ranks, so every
    rank takes the same engine."""
    from . import native
    from .device_grower import agreed_free_bytes, total_device_bytes

    hip = native.hip()
    F_loc = -(-F // max(P, 1))
    fr = exact_finisher_rows(F, C, regression)
    need = exact_workspace_bytes(n, F_loc, C, regression, fr, int(hip.xe_chunk()),
                                 int(hip.xe_rec_width(0 if regression else int(C))))
    if free_bytes is None:
        if need <= total_device_bytes(torch.device("cuda", torch.cuda.current_device())) // 64:
            return True
        free_bytes = agreed_free_bytes(comm, None)
    return need <= free_bytes // 2


def needs_exact(mapper) -> bool:
    """A binned fit cannot be exact: some feature kept quantile edges."""
    ex = np.asarray(getattr(mapper, "exact", []), dtype=bool)
    return bool(ex.size) and not bool(ex.all())


def _packed_labels(C: int) -> bool:
    from . import native

    return C <= int(native.hip().xe_packed_classes())


def own_sizes(fj: torch.Tensor, own: torch.Tensor, P: int) -> torch.Tensor:
    """Rows of each rank's jobs (device [P])."""
    return torch.zeros(P, dtype=torch.int64, device=fj.device).index_add_(0, own, fj[:, 1])


def own_positions(fj: torch.Tensor, own: torch.Tensor, P: int, sizes=None):
    """Job segment positions grouped by owner rank (ascending rank, jobs in
    finisher order within a rank) and each rank's row total (host list: a host
    wait unless ``sizes`` already holds them)."""
    dev = fj.device
    if sizes is None:
        sizes = own_sizes(fj, own, P).cpu()
    sizes = [int(v) for v in sizes.tolist()]
    order = torch.argsort(own, stable=True)
    js = fj.index_select(0, order)
    cnt = js[:, 1]
    excl = torch.cumsum(cnt, 0) - cnt
    total = int(sum(sizes))
    rep_start = torch.repeat_interleave(js[:, 0] - excl, cnt, output_size=total)
    pos = rep_start + torch.arange(total, device=dev)
    return pos, sizes


def _owners(J: int, P: int, device) -> torch.Tensor:
    k = torch.arange(J, device=device)
    lap, off = k // P, k % P
    return torch.where(lap % 2 == 0, off, P - 1 - off)


class ExactGrower:
    """One exact-threshold fit on the current GPU (optionally feature-parallel)."""

    def __init__(self, params, comm=None, checkpoint=None):
        self.p = params
        self.comm = comm
        self.ckpt = checkpoint  # utils/level_checkpoint.LevelCheckpoint (or None)
        self.timings: dict = {}
        self.stats: dict = {}

    # -------------------------------------------------------- checkpoint
    def _ckpt_save(self, lvl, ws, E, Y, be, pos_thr, rank, P):
        """After level ``lvl``'s partition: one sync, then the loop's device
        state -- both list buffers (this rank's features), the next frontier,
        the position space and the finisher jobs (nothing once the next
        frontier is empty: the loop is about to end)."""
        torch.cuda.synchronize(be.device)
        nxt = ws["L"][(lvl + 1) % 2]
        if int(nxt["ctl"][0]) == 0:
            return
        jc = int(ws["job_count"][0])
        arrs = {"set_" + k: v.cpu().numpy() for k, v in nxt.items()}
        for i in range(2):
            arrs[f"E{i}"] = E[i].cpu().numpy()
            if Y[i] is not None:
                arrs[f"Y{i}"] = Y[i].cpu().numpy()
        arrs["pos_rec"] = be.pos_rec.cpu().numpy()
        arrs["pos_st"] = be.pos_st.cpu().numpy()
        arrs["pos_thr"] = pos_thr.cpu().numpy()
        arrs["jobs"] = ws["jobs"][: max(jc, 1)].cpu().numpy()
        arrs["job_count"] = np.array([jc], np.int64)
        self.ckpt.save_device(lvl, arrs, rank, P)

    def _ckpt_restore(self, st, ws, E, Y, be, pos_thr) -> int:
        """Load a saved level's state; returns that level."""
        lvl = int(st["level"][0])
        dev = be.device

        def put(dst, a):
            dst.copy_(torch.from_numpy(np.ascontiguousarray(a)).to(dev))

        for k, v in ws["L"][(lvl + 1) % 2].items():
            put(v, st["set_" + k])
        for i in range(2):
            put(E[i], st[f"E{i}"])
            if Y[i] is not None:
                put(Y[i], st[f"Y{i}"])
        put(be.pos_rec, st["pos_rec"])
        put(be.pos_st, st["pos_st"])
        put(pos_thr, st["pos_thr"])
        jc = int(st["job_count"][0])
        if jc:
            put(ws["jobs"][:jc], st["jobs"][:jc])
        ws["job_count"].fill_(jc)
        return lvl

    # ------------------------------------------------------------- setup
    def _setup(self, Xd, F, f_lo, F_loc, y32, yfix, reg):
        """Sorted lists of this rank's features: E0 (+ Y0); the setup's sorted
        rows and value ranks by sorted position (threshold bins, resolved once
        after growth)."""
        dev = Xd.device
        n = Xd.shape[0]
        hip = self.hip
        s = hb._stream()
        E = [torch.empty((F_loc, n), dtype=torch.int32, device=dev) for _ in range(2)]
        Y = [torch.empty((F_loc, n), dtype=torch.int64, device=dev) for _ in range(2)] if reg \
            else [None, None]
        rank_at = torch.empty((F_loc, n), dtype=torch.int32, device=dev)
        # labels packed in the entries (<= 128 classes) or gathered by row (more)
        packed = not reg and _packed_labels(int(self.C))
        ylab = y32.data_ptr() if packed else 0
        yf = yfix.data_ptr() if reg else 0
        if Xd.dtype == torch.float32:
            keys = [torch.empty((F_loc, n), dtype=torch.int32, device=dev) for _ in range(2)]
            rows = [torch.empty((F_loc, n), dtype=torch.int32, device=dev) for _ in range(2)]
            tb = int(hip.exact_setup_temp_bytes(n, F_loc))
            temp = torch.empty(max(tb, 1), dtype=torch.uint8, device=dev)
            chunk = int(hip.exact_setup_chunk())
            nc = -(-n // chunk)
            cnt = torch.empty((F_loc, nc), dtype=torch.int32, device=dev)
            nuniq = torch.empty(F_loc, dtype=torch.int32, device=dev)
            hip.exact_setup_sort(s, Xd.data_ptr(), n, F_loc, keys[0].data_ptr(),
                                 keys[1].data_ptr(), rows[0].data_ptr(), rows[1].data_ptr(),
                                 temp.data_ptr(), tb, cnt.data_ptr(), nuniq.data_ptr(),
                                 xs=F, f_lo=f_lo, ylab=ylab)
            # (the sort carried the packed labels: the emit gathers none)
            hip.xe_emit(s, keys[1].data_ptr(), rows[1].data_ptr(), n, F_loc, nc, chunk,
                        cnt.data_ptr(), 0, yf, E[0].data_ptr(),
                        Y[0].data_ptr() if reg else 0, rank_at.data_ptr())
            root_rows = rows[1]
            sorted_keys = keys[1]  # (kept for the threshold-rank searches after growth)
            del keys, rows, temp, cnt, nuniq  # (stream-ordered frees)
        else:  # fp64: per-feature stable sorts (ties by row id, -0.0 == 0.0)
            xt = Xd[:, f_lo:f_lo + F_loc].t().contiguous()
            vals, order = torch.sort(xt, dim=1, stable=True)
            del xt
            new = torch.ones_like(vals, dtype=torch.bool)
            new[:, 1:] = vals[:, 1:] != vals[:, :-1]
            nxt_same = torch.zeros_like(new)
            nxt_same[:, :-1] = ~new[:, 1:]
            dup = (~new) | nxt_same
            rank = torch.cumsum(new, 1, dtype=torch.int32) - 1
            o32 = order.to(torch.int32)
            ent = o32 | (dup.to(torch.int32) << 24)
            if packed:
                ent = ent | (y32[order].to(torch.int32) << 25)
            E[0].copy_(ent)
            rank_at.copy_(rank)
            root_rows = o32
            sorted_keys = None
            if reg:
                Y[0].copy_(yfix[order])
            del vals, order, new, nxt_same, dup, rank, ent
        return E, Y, (root_rows, rank_at, sorted_keys)

    # --------------------------------------------------------------- fit
    def fit(self, Xd: torch.Tensor, y_codes: torch.Tensor, root, C: int, crit: Criterion,
            y_exp: int = 0, timings=None):
        """Grow the tree of ``Xd`` (device [n, F] fp32/fp64, every rank the same
        rows) with int32 labels ``y_codes`` (``C`` classes) or int64 fixed-point
        targets (regression, ``C = 0``); ``root``: the root statistics (class
        counts, or {count, sum, min, max})."""
        from . import native

        t0 = time.perf_counter()
        hip = self.hip = native.hip()
        p, comm = self.p, self.comm
        reg = crit == Criterion.SQUARED_ERROR
        Cs = 2 if reg else int(C)
        Cc = 1 if reg else int(C)
        Cx = 0 if reg else int(C)
        n, F = Xd.shape
        dev = Xd.device
        self.C = Cx
        P = int(getattr(comm, "world_size", 1) or 1)
        rank = int(getattr(comm, "rank", 0) or 0)
        if P > 1:
            if F < P:
                raise ValueError(f"exact feature-parallel fit needs n_features >= world size "
                                 f"({F} < {P})")
            from ..parallel.strategies import feature_blocks

            blocks = feature_blocks(F, P)
            f_lo, f_hi = blocks[rank]
        else:
            blocks = [(0, F)]
            f_lo, f_hi = 0, F
        F_loc = f_hi - f_lo
        s = hb._stream
        y32 = None if reg else y_codes.to(torch.int32).contiguous()
        yfix = y_codes.to(torch.int64).contiguous() if reg else None
        self._y32 = y32
        E, Y, ranks = self._setup(Xd, F, f_lo, F_loc, y32, yfix, reg)
        if timings is not None:
            timings["exact_setup"] = time.perf_counter() - t0

        # ---- position space and finisher backend (local codes)
        be = hb.HipBackend(dev)
        be.n, be.F, be.C = n, F, (2 if reg else int(C))
        be.reg = reg
        be.crit = crit
        be.xtab = hb.xlog2x_table(dev, n + 2)  # every count of a node is a table read
        be.xtabf = hb.xlog2x_table_f32(dev)
        be.begin_positions(2 * n - 1)
        pos_thr = hb._workspace(dev, "xe.thr", (2 * n - 1) * 8)[: (2 * n - 1) * 8].view(
            torch.float64)
        md = -1 if p.max_depth is None else int(p.max_depth)
        mss, msl = int(p.min_samples_split), int(max(1, p.min_samples_leaf))
        root = np.asarray(root, dtype=np.int64)
        if reg:
            root_stats = root[:2]
            pure = n == 0 or root[2] == root[3]
        else:
            root_stats = root
            pure = int((root > 0).sum()) <= 1
        if md == 0 or n < mss or n < 2 * msl or pure:
            be.put_positions([0], [-1], [-1], [-1], [-1], [0], [n], root_stats[None, :])
            self.stats.update(levels=0, finisher_subtrees=0)
            return be.assemble_positions(None, int(crit), y_exp, thr_pos=pos_thr)

        fr = exact_finisher_rows(F, Cx, reg)  # (0: levels to the leaves)
        env = os.environ.get("MPITREE_EXACT_FINISHER_ROWS")  # (tests: 0 = no finisher)
        if env is not None:
            fr = max(0, min(fr, int(env)))
        chunk = int(hip.xe_chunk())
        KMAX = n // (fr + 1) + 2
        IMAX = KMAX + n // chunk + 2
        JMAX = n // 2 + 2
        R = int(hip.xe_rec_width(Cx))
        JW = 5 + Cs
        i64 = dict(dtype=torch.int64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        key = (str(dev), n, F_loc, Cx, P, KMAX, IMAX)
        ws = _WS.get(key)
        if ws is None:
            _WS.clear()

            def lists():
                return dict(pos=torch.empty(KMAX, **i64), start=torch.empty(KMAX, **i64),
                            cnt=torch.empty(KMAX, **i32), depth=torch.empty(KMAX, **i32),
                            stats=torch.empty((KMAX, Cs), **i64),
                            minmax=torch.empty((KMAX, 2), **i64),
                            items=torch.empty((IMAX, 4), **i64),
                            ifirst=torch.empty(KMAX + 1, **i32), ctl=torch.zeros(16, **i32))

            ws = _WS[key] = dict(
                L=[lists(), lists()],
                tot=torch.empty((IMAX, F_loc, Cc), **i64),
                carry=torch.empty((IMAX, F_loc, Cc), **i64),
                cmm=torch.empty((IMAX, 2), **i64),
                cbest=torch.empty((IMAX, F_loc, 2), **i64),
                cmin=torch.empty((IMAX, F_loc), **i32),  # two-pass scan references
                nmin=torch.empty((KMAX, F_loc), **i32),
                gthr=torch.empty(KMAX, dtype=torch.float32, device=dev),
                rec=torch.empty((KMAX, R), **i64),
                grec=torch.empty((P * KMAX * R) if P > 1 else 1, **i64),
                split=torch.empty((KMAX, 4), **i64),
                pitems=torch.empty((IMAX, 4), **i64),
                pfirst=torch.empty(KMAX + 1, **i32),
                flag=torch.empty((n + 31) // 32, dtype=torch.int32, device=dev),
                flagb=torch.zeros((n + 31) // 32 * 32, dtype=torch.uint8, device=dev),
                # look-back status words (tagged per fit and level: zeroed once)
                # (one status word per partition wave unit: xe_part_units per item)
                pstat=torch.zeros((int(hip.xe_part_units()) * IMAX, F_loc), **i64),
                sitem=torch.empty((KMAX, 2), **i32),  # (partition-counted chunk totals)
                tick=torch.zeros(4, **i32),
                jobs=torch.empty((JMAX, JW), **i64),
                job_count=torch.zeros(1, **i32),
                root=torch.empty(Cs, **i64),
            )
        L = ws["L"]
        ptr = {k: (v.data_ptr() if isinstance(v, torch.Tensor) else 0) for k, v in ws.items()}
        flag_bytes = os.environ.get("MPITREE_EXACT_FLAG_BYTES", "1") != "0"
        lp = [{k: v.data_ptr() for k, v in x.items()} for x in L]
        ctx = hip.XeCtx(dict(
            E0=E[0].data_ptr(), E1=E[1].data_ptr(),
            Y0=Y[0].data_ptr() if reg else 0, Y1=Y[1].data_ptr() if reg else 0,
            rank_of=0, X=Xd.data_ptr(), x64=int(Xd.dtype == torch.float64),
            n=n, F=F, f_lo=f_lo, F_loc=F_loc, C=Cx, crit=int(crit), msl=msl,
            **({} if reg or _packed_labels(Cx) else {"ylab": y32.data_ptr()}),
            xtab=be.xtab.data_ptr(), xtab_n=int(be.xtab.numel()), tot=ptr["tot"],
            carry=ptr["carry"],
            cmm=ptr["cmm"], cbest=ptr["cbest"], cmin=ptr["cmin"], nmin=ptr["nmin"],
            gthr=ptr["gthr"],
            rec=ptr["rec"], split=ptr["split"],
            pitems=ptr["pitems"], pfirst=ptr["pfirst"], flag=ptr["flag"],
            **({"flagb": ptr["flagb"]} if flag_bytes else {}),
            pstat=ptr["pstat"], tick=ptr["tick"], pos_rec=be.pos_rec.data_ptr(),
            **({"sitem": ptr["sitem"]} if os.environ.get("MPITREE_EXACT_PART_TOT", "1") != "0"
               else {}),
            pos_st=be.pos_st.data_ptr(), pos_thr=pos_thr.data_ptr(), jobs=ptr["jobs"],
            job_count=ptr["job_count"], max_depth=md, mss=mss, fr=fr), lp[0], lp[1])
        ws["root"].copy_(torch.from_numpy(np.ascontiguousarray(root_stats, np.int64)))
        ws["tick"].zero_()  # work tickets + the look-back watchdog
        ck = self.ckpt
        state = None
        if ck is not None:
            # (a state saved with other finisher rows / chunk / buffer sizes is ignored)
            ck.layout = f"exact fr={fr} chunk={chunk} K={KMAX} I={IMAX} J={JMAX} R={R} F={F_loc}"
            state = ck.load_device(rank, P, (lambda a: comm._all_gather(a)) if P > 1 else None)
        first_lvl = 0  # levels before it ran in an earlier process (resume)
        if state is not None:
            first_lvl = self._ckpt_restore(state, ws, E, Y, be, pos_thr) + 1
            ctx.resume_at(first_lvl)
            self.stats["resumed_from_level"] = first_lvl - 1
            del state
        else:
            ctx.init(s(), ws["root"].data_ptr())
        ck_every = max(1, int(os.environ.get("MPITREE_CKPT_EVERY", "1")))
        self._keep = (ctx, E, Y, ranks)

        # ---- level loop: enqueue only; a lagged host-mapped slot tells the end
        hctl_dev, hctl = _host_ctl(hip, dev)
        _FIT_SEQ[0] = (_FIT_SEQ[0] + 1) % (1 << 18)
        ctx.begin(_FIT_SEQ[0] + 1)
        tag0 = _FIT_SEQ[0] << 12
        t1 = time.perf_counter()
        lvl, done_at = first_lvl, None
        comm_bytes = []
        while True:
            if P > 1:  # failure containment: a failed peer / injected fault
                check_abort()
                fault_point(comm, f"level:{lvl}")
            b0 = getattr(comm, "bytes_communicated", 0)
            kb = int(min(2 ** min(lvl, 40), KMAX))
            ib = int(min(IMAX, kb + n // chunk + 1))
            _step(dev, f"level {lvl} start")
            ctx.level_scan(s(), lvl, ib, kb)
            _step(dev, "scan + select")
            if P > 1:  # every rank's best split per node -> the global best
                g = ws["grec"][: P * kb * R]
                comm.all_gather_device(g, ws["rec"][:kb].reshape(-1))
                hip.fp_combine(s(), g.data_ptr(), P, kb, R, lp[lvl % 2]["ctl"],
                               ws["rec"].data_ptr())
            ctx.plan(s(), lvl, hctl_dev + (lvl % 64) * 64, tag0 + (lvl % 4096) + 1)
            _step(dev, "plan")
            if P > 1:  # the split feature's owner sets the left rows; summed over ranks
                if flag_bytes:  # (the byte pack then writes every flag word)
                    ws["flagb"].zero_()
                else:
                    ws["flag"].zero_()
                ctx.flag(s(), lvl, ib, 0)
                comm.all_reduce_device(ws["flag"])
                comm_bytes.append(int(getattr(comm, "bytes_communicated", 0) - b0))
            else:
                ctx.flag(s(), lvl, ib, 1)
            _step(dev, "flag")
            ctx.partition(s(), lvl, ib, kb)
            _step(dev, "partition")
            if ck is not None and (lvl - first_lvl + 1) % ck_every == 0:
                self._ckpt_save(lvl, ws, E, Y, be, pos_thr, rank, P)
            if _DEBUG_SYNC:  # (MPITREE_EXACT_SYNC=1: sync + report every level)
                torch.cuda.synchronize(dev)
                ni = int(L[lvl % 2]["ctl"][1])
                st = ws["pstat"][: min(ni, 4)].cpu().numpy().astype(np.uint64)
                print(f"exact level {lvl}: next frontier {int(L[(lvl + 1) % 2]['ctl'][0])}, "
                      f"jobs {int(ws['job_count'][0])}, tickets {ws['tick'].tolist()}, "
                      f"items {ni}, partition status tags {(st >> np.uint64(34)).tolist()} "
                      f"states {((st >> np.uint64(32)) & np.uint64(3)).tolist()}", flush=True)
            lvl += 1
            if lvl - 2 >= first_lvl:
                _wait_slot(hctl, (lvl - 2) % 64, tag0 + ((lvl - 2) % 4096) + 1)
                if int(hctl[(lvl - 2) % 64, 0]) == 0:
                    done_at = lvl - 2
                    break
            if lvl > 4096:
                raise RuntimeError("exact level loop did not terminate")
        J = int(hctl[done_at % 64, 1])
        self.stats["levels"] = done_at + 1
        self.stats["finisher_subtrees"] = J
        if timings is not None:
            timings["levels"] = time.perf_counter() - t1
        t2 = time.perf_counter()
        if J:
            self._finish(ws, be, E, Y, Xd, J, JW, F, f_lo, F_loc, blocks, n, reg, pos_thr, P,
                         rank)
        self._resolve_bins(be, ranks, Xd, F, f_lo, F_loc, n, pos_thr, P)
        if P > 1:
            self.stats["comm_bytes_per_level"] = comm_bytes
            self.stats["mode"] = "feature"
            self.stats["feature_block"] = [f_lo, f_hi]
        if timings is not None:
            timings["finisher"] = time.perf_counter() - t2
        t3 = time.perf_counter()
        if P > 1:  # a rank whose look-back timed out shared corrupt records / flags:
            # every rank must raise, not only that one (MAX of the watchdog words)
            comm.all_reduce_device(ws["tick"][2:3], op=torch.distributed.ReduceOp.MAX)
        watch = hb._pinned_copy(ws["tick"][2:3], "exact.watch")
        ta = be.assemble_positions(None, int(crit), y_exp, thr_pos=pos_thr)  # (synchronises)
        if int(watch[0]) != 0:
            raise RuntimeError("exact engine: a look-back wait timed out; the tree is invalid")
        if timings is not None:
            timings["assemble"] = time.perf_counter() - t3
        self._keep = None
        if ck is not None:
            self.stats["checkpoint_levels_saved"] = ck.saved_levels
            ck.clear()
        return ta

    # --------------------------------------------------------- finisher
    def _resolve_bins(self, be, ranks, Xd, F, f_lo, F_loc, n, pos_thr, P):
        """Threshold bins (value ranks) of every split node: each rank resolves
        the nodes split on its own features (binary search in the setup's
        sorted order); feature-parallel ranks then exchange {position, bin,
        threshold} of what they resolved."""
        hip, comm = self.hip, self.comm
        s = hb._stream
        dev = Xd.device
        Pp = int(be.pos_rec.shape[0])
        root_rows, rank_at, sorted_keys = ranks
        x64 = int(Xd.dtype == torch.float64)
        resolved = torch.zeros(Pp, dtype=torch.uint8, device=dev) if P > 1 else None
        hip.xe_rank(s(), be.pos_rec.data_ptr(), pos_thr.data_ptr(), Pp, root_rows.data_ptr(),
                    rank_at.data_ptr(), Xd.data_ptr(), x64, F, n, f_lo, F_loc,
                    0 if resolved is None else resolved.data_ptr(),
                    keys=0 if sorted_keys is None else sorted_keys.data_ptr())
        if P == 1:
            return
        tiles = int(hip.asm_tiles(Pp))
        tile = torch.empty(max(tiles, 1), dtype=torch.int32, device=dev)
        total = torch.zeros(2, dtype=torch.int64, device=dev)
        rk = torch.empty(Pp, dtype=torch.int32, device=dev)
        hip.asm_rank(s(), be.pos_rec.data_ptr(), Pp, tile.data_ptr(), total.data_ptr(),
                     rk.data_ptr(), mask=resolved.data_ptr())
        if hasattr(comm, "all_gather_rows_counted"):
            # pack into a position-space-sized buffer: the counts travel on the
            # device and the exchange makes one host wait
            rows = hb._workspace(dev, "xe.resolved", Pp * 3 * 8)[: Pp * 3 * 8]
            rows = rows.view(torch.int64).view(Pp, 3)
            hip.xe_resolved_pack(s(), be.pos_rec.data_ptr(), pos_thr.data_ptr(), Pp,
                                 rk.data_ptr(), rows.data_ptr())
            allr = comm.all_gather_rows_counted(rows, total[0:1])
        else:
            k = int(total[0].item())
            rows = torch.empty((max(k, 1), 3), dtype=torch.int64, device=dev)
            hip.xe_resolved_pack(s(), be.pos_rec.data_ptr(), pos_thr.data_ptr(), Pp,
                                 rk.data_ptr(), rows.data_ptr())
            allr = comm.all_gather_rows(rows[:k])
        hip.xe_resolved_scatter(s(), allr.data_ptr(), int(allr.shape[0]),
                                be.pos_rec.data_ptr(), pos_thr.data_ptr())
        self._keep_r = (allr, rows, resolved, tile, total, rk)

    def _exchange_codes(self, loc, fj, own, blocks, rank, P, F, h_sizes=None):
        """Feature-parallel finisher codes: rank r holds its feature block's codes
        (``loc["blk"]``) at every job position; after one all_to_all every rank
        holds all features' codes (``loc["fm"]``) at its own jobs' positions.
        ``fj``: the jobs in finisher order, ``own``: their owners. Blocks travel
        feature-major ([features, positions]: the gathers read runs of positions,
        the jobs' segments)."""
        comm = self.comm
        dev = fj.device
        pos, sizes = own_positions(fj, own, P, h_sizes)
        lo_me, hi_me = blocks[rank]
        Fb_me = hi_me - lo_me
        src = loc["blk"][:Fb_me]
        in_splits = [int(k) * Fb_me for k in sizes]
        send = torch.empty(max(1, sum(in_splits)), dtype=torch.uint8, device=dev)
        o, p0 = 0, 0
        for k in sizes:
            if k:
                torch.index_select(src, 1, pos[p0 : p0 + k],
                                   out=send[o : o + k * Fb_me].view(Fb_me, k))
            o += k * Fb_me
            p0 += k
        mine = pos[int(sum(sizes[:rank])) : int(sum(sizes[: rank + 1]))]
        n_me = int(sizes[rank])
        out_splits = [n_me * (hi - lo) for lo, hi in blocks]
        recv = torch.empty(max(1, sum(out_splits)), dtype=torch.uint8, device=dev)
        comm.all_to_all_device(recv[: sum(out_splits)], send[: sum(in_splits)], out_splits,
                               in_splits)
        off = 0
        for (lo, hi), k in zip(blocks, out_splits):
            if k:
                loc["fm"][lo:hi].index_copy_(1, mine, recv[off : off + k].view(hi - lo, n_me))
            off += k
        self._keep_c = (send, recv)

    def _finish(self, ws, be, E, Y, Xd, J, JW, F, f_lo, F_loc, blocks, n, reg, pos_thr, P,
                rank):
        """Grow the <= 256-row job segments on subtree-local codes; turn the
        finisher's codes back into value ranks and thresholds."""
        hip, comm = self.hip, self.comm
        s = hb._stream
        dev = Xd.device
        jobs = ws["jobs"][:J]
        rb = (F + 15) // 16 * 16
        key = (str(dev), n, F, P)
        cache = _WS.setdefault("loc", {})
        loc = cache.get(key)
        if loc is None:
            cache.clear()
            Fb = max(hi - lo for lo, hi in blocks)
            loc = cache[key] = dict(
                rm=torch.empty((n, rb), dtype=torch.uint8, device=dev),
                fm=torch.empty((F, n), dtype=torch.uint8, device=dev),
                blk=torch.empty((Fb, n), dtype=torch.uint8, device=dev) if P > 1 else None,
                ent=torch.empty(n, dtype=torch.int32, device=dev),
                tmp=torch.empty(n, dtype=torch.int32, device=dev),
                yv=torch.empty(n, dtype=torch.int64, device=dev) if reg else None,
                nbins=torch.full((F,), 256, dtype=torch.int32, device=dev),
            )
        fm_out = loc["blk"] if P > 1 else loc["fm"]
        x64 = int(Xd.dtype == torch.float64)
        fj = jobs.clone()
        fj[:, 4] = 0  # rows live in the virtual row buffer (idx)
        order = torch.argsort(fj[:, 1] * (1 << 32) - fj[:, 3], descending=True)
        fj = fj.index_select(0, order)
        h_sizes = own = None
        if P > 1:  # (the owners' row totals travel to the host while the codes build)
            own = _owners(J, P, dev)
            h_sizes = hb._pinned_copy(own_sizes(fj, own, P), "exact.own_sizes")
            ev = torch.cuda.Event()
            ev.record()
        hip.xe_local_codes(s(), E[0].data_ptr(), E[1].data_ptr(),
                           Y[0].data_ptr() if reg else 0, Y[1].data_ptr() if reg else 0,
                           Xd.data_ptr(), x64, F, f_lo, n, F_loc, 0, jobs.data_ptr(), J, JW,
                           fm_out.data_ptr(), loc["ent"].data_ptr(),
                           loc["yv"].data_ptr() if reg else 0,
                           0 if reg or _packed_labels(self.C) else self._y32.data_ptr(),
                           codes_rm=0 if P > 1 else loc["rm"].data_ptr(), row_bytes=rb)
        if P > 1:
            # every rank grows its own jobs and needs every feature's codes at their
            # positions only: one all_to_all of the feature blocks' codes at the
            # destination's job positions (1 / P of an all-gather of all codes)
            ev.synchronize()
            self._exchange_codes(loc, fj, own, blocks, rank, P, F, h_sizes)
            fj = fj[own == rank].contiguous()
            if fj.shape[0]:
                hip.xe_codes_rm(s(), loc["fm"].data_ptr(), n, F, rb, fj.data_ptr(),
                                int(fj.shape[0]), JW, loc["rm"].data_ptr())
        # the finisher reads the binned engine's fields: point them at the local codes
        be.codes_rm, be.codes_fm = loc["rm"], loc["fm"]
        be.row_elems, be.cb, be.B, be.nbins = rb, 1, 256, loc["nbins"]
        be.idx, be.tmp = loc["ent"], loc["tmp"]
        if reg:
            be.lab_shift, be.row_mask, be.y = 0, 0xFFFFFFFF, loc["yv"]
        else:
            be.lab_shift, be.row_mask, be.y = 24, (1 << 24) - 1, loc["ent"]
        Jm = int(fj.shape[0])
        if Jm:
            be.launch_finisher(fj, Jm, n, self.p, be.pos_rec, be.pos_st, share=P)
        if P > 1:  # finished job ranges -> every rank
            check_abort()
            fault_point(comm, "exchange")
            rg = torch.stack([fj[:, 3], fj[:, 3] + 2 * fj[:, 1] - 1], 1).contiguous()
            if rg.shape[0] == 0:
                rg = torch.zeros((1, 2), dtype=torch.int64, device=dev)
            self._keep_x = exchange_ranges(be, comm, rg, int(2 * fj[:, 1].sum().item()) + 16)
        # finisher split codes -> threshold values (this rank's features; the bins
        # follow in _resolve_bins)
        hip.xe_fix(s(), E[0].data_ptr(), E[1].data_ptr(), Xd.data_ptr(), x64, F, n, f_lo, F_loc,
                   jobs.data_ptr(), J, JW, be.pos_rec.data_ptr(), pos_thr.data_ptr())
        self._keep_f = (loc, fj)
