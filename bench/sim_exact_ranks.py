"""Per-rank critical path of a P-GPU feature-parallel EXACT fit, measured on ONE GPU.

The exact engine (``ops/exact_grower.py``, reference semantics: every unique
value a candidate, ``/root/reference/mpitree/tree/decision_tree.py:73-90``) is
feature-parallel over P ranks: rank r sorts, scans and partitions only its F/P
presorted lists; per level it all-gathers the per-node best records
(``fp_combine``) and all-reduces the n-bit row-direction flags; the finisher jobs
are dealt serpentine, one all_to_all brings every rank all features' local codes
at its own jobs' positions, and the finished position ranges plus the resolved
thresholds are exchanged at the end.

Rank r's kernels depend on the other ranks only through those collectives, so
rank r can run alone against a stand-in communicator that returns what the
other ranks would have contributed -- recorded from a single-GPU reference fit
of the same data (the P-rank tree is bit-identical to the 1-GPU tree, which
the gloo GPU tests pin): the level's global best records, the level's direction
flags, the other feature blocks' finisher codes at the rank's job positions (the
all_to_all), the finished
records of the other ranks' job ranges (as they stand before the threshold
fix), and every resolved threshold. The script checks every simulated rank's
tree against the reference. Reported per P (median over reps):

* ``max_rank_ms`` -- the critical path of a P-GPU fit minus real collective
  latency (``comm_mb`` per rank says what would cross xGMI);
* ``rank_ms`` / ``F_loc`` -- per rank, with its feature-block width.

The stand-in's own copies (a few MB per level) are inside the timing, so the
numbers are an upper bound on the kernels' share.

    python bench/sim_exact_ranks.py [--n 1000000] [--features 64] [--ranks 1,2,4,8]
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


class Recorder:
    """Wraps the extension's exact-engine entry points during the 1-GPU
    reference fit and snapshots what the other ranks would contribute."""

    def __init__(self, hip, eg):
        self.hip, self.eg = hip, eg
        self.rec, self.flag = [], []
        self.prefix = None
        self.fm = None
        self.jobs = None
        self._orig = {k: getattr(hip, k) for k in ("XeCtx", "xe_fix", "xe_codes_rm")}

    def _ws(self):
        return next(v for k, v in self.eg._WS.items() if k != "loc")

    def install(self):
        rec = self
        orig_ctx = self._orig["XeCtx"]

        class Ctx:
            def __init__(self, *a):
                self._c = orig_ctx(*a)

            def __getattr__(self, k):
                return getattr(self._c, k)

            def level_scan(self, s, lvl, ib, kb):
                self._c.level_scan(s, lvl, ib, kb)
                rec.rec.append(rec._ws()["rec"][:kb].clone())

            def flag(self, s, lvl, ib, w):
                self._c.flag(s, lvl, ib, w)
                rec.flag.append(rec._ws()["flag"].clone())

        def codes_rm(s, fm, n, F, rb, jobs, J, JW, rm):
            rec._orig["xe_codes_rm"](s, fm, n, F, rb, jobs, J, JW, rm)
            loc = next(iter(rec.eg._WS["loc"].values()))
            rec.fm = loc["fm"].clone()
            rec.jobs = rec._ws()["jobs"][:J].clone()

        def fix(s, *a):
            from mpitree_amd.ops import hip_backend as hb

            if rec.fm is None:  # (one GPU: the local-codes kernel wrote codes_rm itself)
                loc = next(iter(rec.eg._WS["loc"].values()))
                rec.fm = loc["fm"].clone()
                J = int(a[9])  # xe_fix(s, E0, E1, X, x64, F, n, f_lo, F_loc, jobs, J, JW, ...)
                rec.jobs = rec._ws()["jobs"][:J].clone()
            dev = rec.fm.device
            rows = hb._workspace(dev, "pos_rec", 0)
            rec.prefix = rows.clone()  # position records before the threshold fix
            st = hb._workspace(dev, "pos_st", 0)
            rec.prefix_st = st.clone()
            rec._orig["xe_fix"](s, *a)

        self.hip.XeCtx = Ctx
        self.hip.xe_codes_rm = codes_rm
        self.hip.xe_fix = fix

    def uninstall(self):
        for k, v in self._orig.items():
            setattr(self.hip, k, v)


class SimFeatureComm(LocalComm):
    """Rank ``rank`` of a P-rank feature-parallel exact fit, without other ranks."""

    kind = "feature"
    simulated = True

    def __init__(self, P, rank, ref, n, F, C):
        self.world_size, self.rank = P, rank
        self.ref, self.n, self.F, self.C = ref, n, F, C
        self.bytes_communicated = 0
        self.lvl = 0
        self.flag_lvl = 0
        self.exchanges = 0

    def all_gather_device(self, out, inp):  # the level's best records
        P, r = self.world_size, self.rank
        self.bytes_communicated += inp.numel() * inp.element_size() * P
        o = out.view(P, -1)
        o.copy_(self.ref["rec"][self.lvl].reshape(1, -1).expand(P, -1))
        self.lvl += 1
        o[r].copy_(inp.reshape(-1))

    def all_to_all_device(self, out, inp, out_splits, in_splits):
        """The finisher codes: every other feature block's codes at this rank's
        job positions (the reference fit's codes), this rank's own chunk as sent."""
        from mpitree_amd.ops.exact_grower import _owners, own_positions
        from mpitree_amd.parallel.strategies import feature_blocks

        P, r = self.world_size, self.rank
        self.bytes_communicated += int(sum(in_splits))
        cache = self.ref.setdefault("mine", {})
        if (P, r) not in cache:  # (the stand-in's own bookkeeping: once per rank)
            fj = self.ref["fj"]
            pos, sizes = own_positions(fj, _owners(int(fj.shape[0]), P, fj.device), P)
            cache[(P, r)] = pos[int(sum(sizes[:r])) : int(sum(sizes[: r + 1]))].clone()
        mine = cache[(P, r)]
        off = 0
        for q, (lo, hi) in enumerate(feature_blocks(self.F, P)):
            k = int(out_splits[q])
            if q == r:
                s0 = int(sum(in_splits[:r]))
                out[off : off + k].copy_(inp[s0 : s0 + k])
            elif k:
                torch.index_select(self.ref["fm"][lo:hi], 1, mine,
                                   out=out[off : off + k].view(hi - lo, -1))
            off += k

    def all_reduce_device(self, t, op=None):
        self.bytes_communicated += t.numel() * t.element_size()
        if t.numel() == 1:  # the watchdog word (MAX over ranks): this rank's stands
            return
        t.copy_(self.ref["flag"][self.flag_lvl])
        self.flag_lvl += 1

    def all_gather_rows(self, t):
        self.bytes_communicated += t.numel() * t.element_size() * self.world_size
        self.exchanges += 1
        if t.shape[1] == 3:  # resolved {position, bin, threshold}: every split
            return torch.cat([t, self.ref["resolved"]], 0)
        return torch.cat([t, self.ref["others"][self.rank].to(t.dtype)], 0)


def build_reference(fit, dev, P_list, C):
    from mpitree_amd.ops import exact_grower as eg
    from mpitree_amd.ops import hip_backend as hb
    from mpitree_amd.ops import native

    hip = native.hip()
    R = Recorder(hip, eg)
    R.install()
    try:
        res = fit()
        torch.cuda.synchronize()
    finally:
        R.uninstall()
    pos_rec = hb._workspace(dev, "pos_rec", 0)
    Pp = 2 * int(res.arrays.n_samples[0]) - 1
    fin = pos_rec[: Pp * 24].view(torch.int32).view(Pp, 6)
    thr = hb._workspace(dev, "xe.thr", 0)[: Pp * 8].view(torch.float64)
    split = torch.nonzero(fin[:, 0] >= 0).squeeze(1)
    split = split[fin[split, 5] > 0]
    resolved = torch.stack([split, fin[split, 1].long(), thr[split].view(torch.int64)], 1)
    # records of each rank's finisher job ranges as they stood before the fix
    pre = R.prefix[: Pp * 24].view(torch.int32).view(Pp, 6)
    pst = R.prefix_st[: Pp * C * 4].view(torch.int32).view(Pp, C)
    jobs = R.jobs
    fj = jobs.clone()
    order = torch.argsort(fj[:, 1] * (1 << 32) - fj[:, 3], descending=True)
    fj = fj.index_select(0, order)
    others = {}
    for P in P_list:
        if P == 1:
            continue
        own = eg._owners(int(fj.shape[0]), P, dev)
        for r in range(P):
            mark = torch.zeros(Pp + 1, dtype=torch.int32, device=dev)
            sel = fj[own != r]
            lo, hi = sel[:, 3], sel[:, 3] + 2 * sel[:, 1] - 1
            mark.index_add_(0, lo, torch.ones_like(lo, dtype=torch.int32))
            mark.index_add_(0, hi, -torch.ones_like(hi, dtype=torch.int32))
            inside = torch.cumsum(mark, 0)[:Pp] > 0
            live = torch.nonzero(inside & (pre[:, 5] > 0)).squeeze(1)
            others[(P, r)] = torch.cat([live.to(torch.int32)[:, None], pre[live], pst[live]], 1)
    return res, dict(rec=R.rec, flag=R.flag, fm=R.fm, resolved=resolved, others=others, fj=fj)


def _diff(a, b) -> dict:
    """Which columns of two trees differ, and where first (diagnostics)."""
    out = {"nodes": [int(a.node_count), int(b.node_count)]}
    for k in ("feature", "threshold_bin", "left", "right", "depth", "n_samples", "threshold",
              "count", "value", "impurity"):
        x, y = getattr(a, k), getattr(b, k)
        if x is None or y is None:
            continue
        if x.shape != y.shape:
            out[k] = f"shape {x.shape} vs {y.shape}"
            continue
        ne = ~((x == y) | (np.isnan(x) & np.isnan(y)) if x.dtype.kind == "f" else (x == y))
        if ne.ndim > 1:
            ne = ne.any(axis=tuple(range(1, ne.ndim)))
        if ne.any():
            i = int(np.argmax(ne))
            out[k] = dict(n=int(ne.sum()), first=i, got=str(x[i]), want=str(y[i]),
                          depth=int(b.depth[i]), n_samples=int(b.n_samples[i]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only-rank", type=int, default=None)
    a = ap.parse_args()
    from mpitree_amd.core.fit import fit_tree

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(a.n, a.features, device=dev, generator=g)
    w = torch.randn(a.features, device=dev, generator=g)
    y = ((X @ w + 0.5 * torch.randn(a.n, device=dev, generator=g)) > 0).to(torch.int64)

    def fit(comm=None):
        return fit_tree(X, y, regression=False, criterion=0, max_depth=None,
                        min_samples_split=2, max_bins=None, device="cuda", comm=comm)

    fit()
    P_list = [int(v) for v in a.ranks.replace("+", ",").split(",")]
    ref, data = build_reference(fit, dev, P_list, 2)
    assert ref.engine == "hip-exact", ref.engine
    for P in P_list:
        per_rank = []
        for r in range(P) if a.only_rank is None or P == 1 else [a.only_rank]:
            if P > 1:
                data_r = dict(data, others=data["others"])
                data_r["others"] = {r: data["others"][(P, r)]}
            times, st, ph = [], {}, []
            for i in range(a.reps + 1):
                comm = SimFeatureComm(P, r, data_r, a.n, a.features, 2) if P > 1 else None
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = fit(comm)
                torch.cuda.synchronize()
                if i >= 1:
                    times.append((time.perf_counter() - t0) * 1e3)
                    ph.append({k: v * 1e3 for k, v in res.timings.items()
                               if k in ("exact_setup", "levels", "finisher", "assemble")})
                st = res.stats
                if not res.arrays.equal(ref.arrays):
                    print(json.dumps(dict(P=P, rank=r, diff=_diff(res.arrays, ref.arrays))),
                          flush=True)
                    raise AssertionError(f"P={P} rank {r}: tree differs")
            per_rank.append(dict(ms=float(np.median(times)),
                                 phases={k: round(float(np.median([q[k] for q in ph])), 2)
                                         for k in ph[0]},
                                 F_loc=(st.get("feature_block", [0, a.features])[1]
                                        - st.get("feature_block", [0, a.features])[0]),
                                 comm_mb=(comm.bytes_communicated / 1e6 if comm else 0.0)))
        ms = [p["ms"] for p in per_rank]
        print(json.dumps(dict(P=P, max_rank_ms=round(max(ms), 3),
                              rank_ms=[round(v, 3) for v in ms],
                              F_loc=[p["F_loc"] for p in per_rank],
                              phases_rank0=per_rank[0]["phases"],
                              comm_mb=round(max(p["comm_mb"] for p in per_rank), 2),
                              levels=ref.stats.get("levels"), nodes=ref.arrays.node_count,
                              tree_equal=True)), flush=True)


if __name__ == "__main__":
    main()
