"""Per-rank critical path of a P-GPU subtree-ownership fit, measured on ONE GPU.

The multi-GPU ``auto`` / ``subtree`` fit (rows replicated on every rank, the
reference's ParallelDecisionTreeClassifier contract) runs the device level loop
replicated until the first level with at least ``k * P`` units (split nodes
whose children keep growing + finisher jobs so far); that level's planner
assigns the units to ranks by greedy LPT on row counts and from then on a rank
grows only its own units -- level loop and finisher -- with no collective until
one all-gather of the finished nodes (``ops/device_grower.py``,
``grow.hip own_switch``). Rank r's kernel sequence therefore does not depend on
the other ranks at all, so it can be run alone: this script fits with a
stand-in communicator (``world_size = P``, ``rank = r``) whose node all-gather
returns the other ranks' nodes from a single-GPU reference fit (the trees are
bit-identical, so the result is the complete tree, and the script checks it
against the reference). Per P it reports, over ranks, the median fit time of
each rank's exact sequence (binning, replicated levels, own levels, own
finisher share, exchange stand-in, assembly + the full tree's D2H):

* ``max_rank_ms`` -- the critical path (what a P-GPU fit waits for, plus the
  real all-gather's latency: ``exchange_mb`` over xGMI);
* ``rows_owned`` / ``units`` -- the LPT's per-rank rows and the unit count.

    python bench/sim_own_ranks.py [--n 1000000] [--features 64] [--ranks 1,2,4,8]
                                  [--regression] [--continuous]

``--regression``: the 1M x 64 MSE regression tree (BASELINE config 5), whose
exchange rows carry int64 {count, sum} statistics.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mpitree_amd.core.levelwise import LocalComm  # noqa: E402
from mpitree_amd.parallel.shared_tree import GATHER_HDR  # noqa: E402


class SimSlot:
    """The shared tree buffer stand-in: mapped pinned host memory holding the
    reference tree's packed columns (the other ranks' nodes) before each fit."""

    def __init__(self, ref_bytes: np.ndarray):
        import ctypes

        from mpitree_amd.ops import native
        from mpitree_amd.parallel.shared_tree import HEADER

        hip = native.hip()
        size = HEADER + ref_bytes.size
        self.host = int(hip.host_alloc(size, coherent=False))
        self.nd = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(self.host))
        self.dev = int(hip.host_device_ptr(self.host))
        self.nbytes = size
        self.ref = ref_bytes
        self.header = HEADER

    def prefill(self):
        self.nd[self.header :] = self.ref


class SimPool:
    """Shared-host assembly stand-in: one slot, no peers to wait for."""

    def __init__(self, slot: SimSlot):
        self.slot = slot

    def free_mask(self) -> int:
        return 1

    def choose(self, masks, need: int, shm_free=None):
        assert need <= self.slot.ref.size, "tree larger than the reference"
        return self.slot

    def take_next(self):
        return self.slot

    def plan_next(self, masks, current, need: int, shm_free=None) -> None:
        return None

    def barrier(self, slot) -> None:
        return None


class SimOwnComm(LocalComm):
    """Rank ``rank`` of a P-rank subtree-ownership group, without other ranks.
    Shared-host assembly (the default on one node): the segment-count all-gather
    returns every segment's node count from the reference fit's position space
    and the shared buffer already holds the reference tree, so the rank writes
    only its own nodes. ``--no-shared`` (``MPITREE_SHM_TREE=0``): the node
    exchange returns this rank's rows plus every node of the reference fit."""

    kind = "subtree"
    simulated = True

    def __init__(self, P: int, rank: int, device, ref_rows: torch.Tensor, ref_pos=None,
                 ref_depth=0, pool=None, ref_recs=None):
        self.world_size = P
        self.rank = rank
        self.device = device
        self.bytes_communicated = 0
        self.ref_rows = ref_rows
        self.ref_pos, self.ref_depth = ref_pos, int(ref_depth)
        self._shm_pool = pool if pool is not None else False
        self._head = torch.tensor([int(ref_depth), 1, 1 << 62], dtype=torch.int64,
                                  device=device)
        self.ref_recs, self._lvl = ref_recs, 0

    def all_gather_device(self, out, inp):
        # feature-parallel prefix levels: every other rank's best split of each
        # node stands in as the reference fit's (global best) record, which the
        # combine picks over this rank's block-best (ties: the lower feature)
        P = self.world_size
        ref = self.ref_recs[self._lvl].reshape(-1)
        self._lvl += 1
        o = out.view(P, -1)
        o.copy_(ref[None, :].expand(P, -1))
        o[self.rank].copy_(inp.view(-1))
        self.bytes_communicated += inp.numel() * inp.element_size() * P

    def all_gather_rows(self, t):
        # bytes of a real exchange: every rank's rows, padded to the largest share
        self.bytes_communicated += self.ref_rows.numel() * self.ref_rows.element_size()
        return torch.cat([t, self.ref_rows.to(t.dtype)], 0)

    def all_gather_seg_counts(self, out, inp, segs, S):
        # every rank's row: its segments' node counts (from the reference positions)
        # (a few small kernels: what the real all-gather costs is estimated apart)
        P, W = self.world_size, inp.numel()
        g = out.view(P, W)
        cnt = torch.searchsorted(self.ref_pos, segs[:S, :2].contiguous()).diff(dim=1)[:, 0]
        mine = segs[:S, 2][None, :] == torch.arange(P, device=segs.device)[:, None]
        H = GATHER_HDR
        g[:, H : H + S] = mine * cnt[None, :]
        g[:, :H] = self._head
        self.bytes_communicated += P * W * 8


def packed_bytes(ta) -> np.ndarray:
    """A finished tree's columns in the device assembly's packed layout
    (``TreeArrays.from_packed``)."""
    cols = [ta.n_samples.astype(np.int64), ta.threshold.astype(np.float64)]
    if ta.value is not None:
        cols += [ta.value.astype(np.float64)]
    else:
        cols += [ta.impurity.astype(np.float64), ta.count.astype(np.int32)]
    cols += [c.astype(np.int32) for c in (ta.feature, ta.threshold_bin, ta.left, ta.right,
                                          ta.depth)]
    return np.concatenate([np.ascontiguousarray(c).view(np.uint8).reshape(-1) for c in cols])


def reference_rows(fit, dev, regression=False):
    """The position-space rows {pos, record[6], stats} of a finished 1-GPU fit:
    int32 class counts, or (regression) int64 {count, fixed-point sum}."""
    from mpitree_amd.ops import hip_backend as hb

    r = fit()
    n_pos = 2 * r.arrays.n_samples[0] - 1
    rec = hb._workspace(dev, "pos_rec", 0)[: n_pos * 24].view(torch.int32).view(-1, 6)
    live = torch.nonzero(rec[:, 5] > 0).squeeze(1)
    if regression:
        st = hb._workspace(dev, "pos_st", 0)[: n_pos * 16].view(torch.int64).view(-1, 2)
        rows = torch.cat([live[:, None], rec[live].long(), st[live]], 1).clone()
    else:
        C = r.arrays.count.shape[1]
        st = hb._workspace(dev, "pos_st", 0)[: n_pos * C * 4].view(torch.int32).view(-1, C)
        rows = torch.cat([live.to(torch.int32)[:, None], rec[live], st[live]], 1).clone()
    return r, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--units-per-rank", type=int, default=None)
    ap.add_argument("--only-rank", type=int, default=None,
                    help="simulate this rank only (profiling one rank's kernel sequence)")
    ap.add_argument("--regression", action="store_true")
    ap.add_argument("--fp-prefix", default=None, choices=["0", "1"],
                    help="force the feature-parallel prefix levels off / on")
    ap.add_argument("--no-shared", action="store_true",
                    help="node exchange + full-tree copy instead of the shared-host assembly")
    ap.add_argument("--cprofile", default=None,
                    help="write a cProfile of the timed fits' host code to this file")
    a = ap.parse_args()
    prof = None
    if a.cprofile:
        import cProfile

        prof = cProfile.Profile()
    if a.fp_prefix is not None:
        os.environ["MPITREE_OWN_FP_PREFIX"] = a.fp_prefix
    if a.units_per_rank is not None:
        os.environ["MPITREE_OWN_UNITS_PER_RANK"] = str(a.units_per_rank)
    from mpitree_amd.core.fit import fit_tree
    from mpitree_amd.utils.datasets import make_classification, make_regression

    dev = torch.device("cuda", 0)
    if a.regression:  # (bench.py --regression: the same generator and seed)
        X, y = make_regression(a.n, a.features, levels=256, seed=0, device=dev)
    else:
        X, y = make_classification(a.n, a.features, n_classes=2, seed=0, device=dev)

    def fit(comm=None):
        return fit_tree(X, y, regression=a.regression, criterion=2 if a.regression else 0,
                        max_depth=None, min_samples_split=2, device="cuda", comm=comm)

    for _ in range(2):
        fit()
    from mpitree_amd.ops import device_grower as dg

    dg.REC_DUMP = []  # the reference fit's per-level split records (prefix stand-in)
    ref, ref_rows = reference_rows(fit, dev, a.regression)
    ref_recs, dg.REC_DUMP = dg.REC_DUMP, None
    ref_pos = ref_rows[:, 0].long().contiguous()  # live positions, ascending
    pool = None
    if not a.no_shared:
        pool = SimPool(SimSlot(packed_bytes(ref.arrays)))
    for P in [int(v) for v in a.ranks.replace("+", ",").split(",")]:
        per_rank = []
        for r in range(P) if a.only_rank is None else [a.only_rank]:
            times, st, ph = [], {}, []
            for i in range(a.reps + 2):
                comm = (SimOwnComm(P, r, dev, ref_rows, ref_pos, ref.arrays.max_depth, pool,
                                   ref_recs) if P > 1 else None)
                if pool is not None:
                    pool.slot.prefill()
                torch.cuda.synchronize()
                if prof is not None and i >= 2:
                    prof.enable()
                t0 = time.perf_counter()
                res = fit(comm)
                torch.cuda.synchronize()
                if prof is not None:
                    prof.disable()
                if i >= 2:
                    times.append((time.perf_counter() - t0) * 1e3)
                st = res.stats
                if i >= 2:
                    ph.append({k: v * 1e3 for k, v in res.timings.items()
                               if isinstance(v, float)})
                assert res.arrays.equal(ref.arrays), f"P={P} rank {r}: tree differs"
            per_rank.append(dict(ms=float(np.median(times)), rows=st.get("own_rows", a.n),
                                 fp_levels=st.get("fp_prefix_levels", 0),
                                 units=st.get("own_units", 0), levels=st.get("levels"),
                                 mode=st.get("mode", "single-gpu"),
                                 exchange_mb=st.get("comm_bytes_exchange", 0) / 1e6,
                                 phases={k: round(float(np.median([d.get(k, 0.0) for d in ph])), 3)
                                         for k in ph[0]}))
        ms = [p["ms"] for p in per_rank]
        out = dict(P=P, max_rank_ms=round(max(ms), 3), mean_rank_ms=round(float(np.mean(ms)), 3),
                   rank_ms=[round(v, 3) for v in ms], rows_owned=[p["rows"] for p in per_rank],
                   units=per_rank[0]["units"], levels=[p["levels"] for p in per_rank],
                   mode=per_rank[0]["mode"], exchange_mb=round(per_rank[0]["exchange_mb"], 2),
                   fp_prefix_levels=[p["fp_levels"] for p in per_rank],
                   nodes=ref.arrays.node_count, tree_equal=True,
                   phases_max_rank=per_rank[int(np.argmax(ms))]["phases"])
        print(json.dumps(out), flush=True)
    if prof is not None:
        import io
        import pstats

        with open(a.cprofile, "w") as f:
            for key in ("tottime", "cumulative"):
                sio = io.StringIO()
                pstats.Stats(prof, stream=sio).sort_stats(key).print_stats(45)
                f.write(f"==== by {key}\n{sio.getvalue()}\n")


if __name__ == "__main__":
    main()
