"""Per-rank critical path of a P-GPU data-parallel fit, measured on ONE GPU.

``strategy="data"`` (BASELINE config 4's named strategy) shards the rows: rank r
holds rows [n r / P, n (r + 1) / P). Per level it builds the built slots'
histograms of its own rows, one feature block at a time, and each block is
reduced to its owner rank (a reduce-scatter by feature); every rank scans its
block, the split records are all-gathered and combined, and every rank
partitions its own rows. The finisher jobs' rows then travel to their owners
(one all_to_all) and each rank finishes its own jobs (``ops/device_grower.py``,
``dp_route.hip``).

Rank r's kernel sequence depends on the other ranks only through those
collectives, so it runs alone here with a stand-in communicator that answers
them from a single-GPU reference fit of the same data:

* the level's reduce-scatter (or, for unequal feature blocks, the block reduce)
  returns the reference's (global) built histograms of the rank's feature block
  for that level;
* the record all-gather returns the reference's per-node best records (the
  combine picks the global best, ties to the lower feature, as with real peers);
* the job-row count all-gather returns every rank's rows of each job (from the
  reference's job segments), the all_to_all the other ranks' rows of the rank's
  jobs (ascending row order within a source, as each peer's stable partitions
  keep them);
* the finished nodes: with the node-shared host tree (the default on one node)
  the segment-count all-gather returns every job's node count from the
  reference positions and the shared buffer already holds the reference tree,
  so the rank writes only its own jobs' nodes (``sim_own_ranks.SimPool``);
  ``--no-shared`` keeps the node all-gather, answered with the reference's nodes.

The simulated rank must rebuild the reference tree bit for bit (checked). Per P
it reports the max / mean over ranks of the median fit time and the bytes the
real collectives would move (reduce, record all-gathers, row all_to_all, node
exchange), from which scaling_projection.md adds the xGMI time.

    python bench/sim_dp_ranks.py [--n 10000000] [--features 128] [--ranks 2+4+8]
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


class SimDPComm(LocalComm):
    kind = "data"
    simulated = True
    rows_replicated = False
    sharded = False

    def __init__(self, P, rank, device, ref):
        self.world_size, self.rank, self.device = P, rank, device
        self.ref = ref
        self.bytes_communicated = 0
        self.bytes = dict(reduce=0, records=0, counts=0, rows=0, nodes=0)
        self.calls = 0  # collectives a real group would issue (latency term of the estimate)
        self._red = 0  # block reduces so far (P per level)
        self._rs = 0  # reduce-scatters so far (one per level)
        self._gat = 0  # record all-gathers so far (one per level)
        self._shm_pool = False  # (main sets the shared-tree stand-in)
        self._finishing = False  # set once the level loop is over (job row counts)

    def note_phase(self, name):
        self._finishing = name == "dp_finish"

    def _all_reduce(self, a, op=None):  # (the bin flags: every shard agrees here)
        return a

    def local_rows(self, n):
        P, r = self.world_size, self.rank
        return n * r // P, n * (r + 1) // P

    def reduce_stats(self, stats, reg):
        return self.ref["root"][None, :].copy()

    def reduce_device(self, t, dst, async_op=False):
        lvl, blk = divmod(self._red, self.world_size)
        self._red += 1
        nb = t.shape[0]
        self.bytes["reduce"] += t.numel() * t.element_size()
        self.calls += 1
        if dst == self.rank and lvl < len(self.ref["hists"]):  # (else: a lagged empty level)
            lo, hi = self.ref["blocks"][dst]
            H = self.ref["hists"][lvl]
            k = min(nb, H.shape[0])
            t[:k].copy_(H[:k, lo:hi])
        return None

    def reduce_scatter_device(self, out, inp):
        # one per level: this rank's block of the reference's global built histograms
        lvl = self._rs
        self._rs += 1
        self.bytes["reduce"] += inp.numel() * inp.element_size()
        self.calls += 1
        if lvl < len(self.ref["hists"]):  # (else: a lagged empty level)
            lo, hi = self.ref["blocks"][self.rank]
            H = self.ref["hists"][lvl]
            o = out.view(-1, hi - lo, H.shape[2], H.shape[3])
            k = min(o.shape[0], H.shape[0])
            o[:k].copy_(H[:k, lo:hi])

    def all_gather_device(self, out, inp):
        P = self.world_size
        if not self._finishing:  # a level's split records
            o = out.view(P, -1)
            if self._gat < len(self.ref["recs"]):
                ref = self.ref["recs"][self._gat].reshape(-1)
                o.copy_(ref[None, :].expand(P, -1))
            else:  # (a lagged empty level: nothing reads its records)
                o.copy_(inp.view(1, -1).expand(P, -1))
            self._gat += 1
            o[self.rank].copy_(inp.view(-1))
            self.bytes["records"] += inp.numel() * inp.element_size() * P
            self.calls += 1
            return
        # the finisher jobs' per-rank row counts [P, J]
        out.view(P, -1).copy_(self.ref["allc"])
        self.bytes["counts"] += inp.numel() * inp.element_size() * P
        self.calls += 1

    def all_to_all_device(self, out, inp, out_splits, in_splits):
        r = self.rank
        src = self.ref["recv_codes"][r] if out.dtype == torch.uint8 else self.ref["recv_y"][r]
        out.copy_(src.view(-1)[: out.numel()].view(out.dtype) if out.dtype == torch.uint8
                  else src[: out.numel()])
        if out.dtype == torch.uint8:
            self.bytes["rows"] += int(sum(in_splits))
        self.calls += 1

    def all_reduce_device(self, t, op=None):  # (regression only: not simulated)
        raise NotImplementedError("sim_dp_ranks simulates classification fits")

    def all_gather_rows(self, t):
        self.bytes["nodes"] += self.ref["rows"].numel() * self.ref["rows"].element_size()
        return torch.cat([t, self.ref["rows"].to(t.dtype)], 0)

    def all_gather_seg_counts(self, out, inp, segs, S):
        # every rank's row: its jobs' node counts (from the reference positions)
        P, W = self.world_size, inp.numel()
        g = out.view(P, W)
        cnt = torch.searchsorted(self.ref["pos"], segs[:S, :2].contiguous()).diff(dim=1)[:, 0]
        mine = segs[:S, 2][None, :] == torch.arange(P, device=segs.device)[:, None]
        g[:, GATHER_HDR : GATHER_HDR + S] = mine * cnt[None, :]
        g[:, :GATHER_HDR] = self.ref["head"]
        self.bytes["nodes"] += P * W * 8
        self.calls += 1


def reference(fit, dev, X, y, P, F):
    """The single-GPU fit plus everything the stand-ins answer with."""
    from mpitree_amd.ops import device_grower as dg
    from mpitree_amd.ops import hip_backend as hb
    from mpitree_amd.parallel.strategies import feature_blocks

    dg.REC_DUMP, dg.DUMP = [], {}
    r = fit(None)
    torch.cuda.synchronize()
    recs, dump = dg.REC_DUMP, dg.DUMP
    dg.REC_DUMP = dg.DUMP = None
    n = X.shape[0]
    n_pos = 2 * n - 1
    rec = hb._workspace(dev, "pos_rec", 0)[: n_pos * 24].view(torch.int32).view(-1, 6)
    live = torch.nonzero(rec[:, 5] > 0).squeeze(1)
    C = r.arrays.count.shape[1]
    st = hb._workspace(dev, "pos_st", 0)[: n_pos * C * 4].view(torch.int32).view(-1, C)
    rows = torch.cat([live.to(torch.int32)[:, None], rec[live], st[live]], 1).clone()
    # the finisher jobs' global rows (ascending within a job: stable partitions)
    jobs = dump["jobs"]
    J = jobs.shape[0]
    bufs = (dump["idx"], dump["tmp"])
    mask = dump["row_mask"]
    job_rows = []
    for j in range(J):
        s0, cnt, b = int(jobs[j, 0]), int(jobs[j, 1]), int(jobs[j, 4])
        job_rows.append(torch.sort((bufs[b][s0:s0 + cnt].long() & mask))[0])
    shard = [(n * s // P, n * (s + 1) // P) for s in range(P)]
    allc = torch.zeros((P, J), dtype=torch.int64, device=dev)
    for j, g in enumerate(job_rows):
        for s, (lo, hi) in enumerate(shard):
            allc[s, j] = int(((g >= lo) & (g < hi)).sum())
    return dict(fit=r, recs=recs, hists=dump["hists"], job_rows=job_rows, allc=allc,
                shard=shard, rows=rows, blocks=feature_blocks(F, P), J=J)


def received(ref, codes_rm, yenc, P, r):
    """Rank r's all_to_all input: for each source s, the rows of r's jobs (job
    order) that s holds, ascending -- as row-major codes and targets."""
    J = ref["J"]
    k = torch.arange(J)
    lap, off = k // P, k % P
    owner = torch.where(lap % 2 == 0, off, P - 1 - off)
    mine = torch.nonzero(owner == r).squeeze(1).tolist()
    parts = []
    for s, (lo, hi) in enumerate(ref["shard"]):
        for j in mine:
            g = ref["job_rows"][j]
            parts.append(g[(g >= lo) & (g < hi)])
    idx = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64, device=codes_rm.device)
    return codes_rm.index_select(0, idx).contiguous().view(torch.uint8).view(-1), \
        yenc.index_select(0, idx).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--features", type=int, default=128)
    ap.add_argument("--ranks", default="2+4+8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only-rank", type=int, default=None)
    ap.add_argument("--no-shared", action="store_true",
                    help="node all-gather instead of the node-shared host tree")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from sim_own_ranks import SimPool, SimSlot, packed_bytes
    from mpitree_amd.core.fit import fit_tree
    from mpitree_amd.ops import gpu_prepare
    from mpitree_amd.utils.datasets import make_classification

    dev = torch.device("cuda", 0)
    X, y = make_classification(a.n, a.features, n_classes=2, seed=0, device=dev)

    def fit(comm):
        return fit_tree(X, y, regression=False, criterion=0, max_depth=None,
                        min_samples_split=2, device="cuda", comm=comm)

    for _ in range(2):
        fit(None)
    t_single = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fit(None)
        torch.cuda.synchronize()
        t_single.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps(dict(P=1, max_rank_ms=round(float(np.median(t_single)), 3),
                          mode="single-gpu", n=a.n, features=a.features)), flush=True)
    # the encoded rows every rank's codes come from (the same binning as a fit)
    from mpitree_amd.core.fit import _encode_labels, _encode_targets, fixed_point_exponent

    prep = gpu_prepare.prepare(X, y, regression=False, max_bins=256,
                               encode_labels=_encode_labels, encode_targets=_encode_targets,
                               exponent=fixed_point_exponent, sync=True)
    codes_rm, yenc = prep.codes_rm, prep.y
    for P in [int(v) for v in a.ranks.replace("+", ",").split(",")]:
        ref = reference(fit, dev, X, y, P, a.features)
        ref["root"] = np.bincount(y.cpu().numpy(), minlength=2).astype(np.int64)
        ref["pos"] = ref["rows"][:, 0].long().contiguous()  # live positions, ascending
        ref["head"] = torch.tensor([int(ref["fit"].arrays.max_depth), 1, 1 << 62],
                                   dtype=torch.int64, device=dev)
        pool = None if a.no_shared else SimPool(SimSlot(packed_bytes(ref["fit"].arrays)))
        per_rank = []
        for r in range(P) if a.only_rank is None else [a.only_rank]:
            ref["recv_codes"] = {r: None}
            ref["recv_y"] = {r: None}
            ref["recv_codes"][r], ref["recv_y"][r] = received(ref, codes_rm, yenc, P, r)
            times, comm = [], None
            for i in range(a.reps + 1):
                comm = SimDPComm(P, r, dev, ref)
                if pool is not None:
                    comm._shm_pool = pool
                    pool.slot.prefill()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = fit(comm)
                torch.cuda.synchronize()
                if i >= 1:
                    times.append((time.perf_counter() - t0) * 1e3)
                assert res.arrays.equal(ref["fit"].arrays), f"P={P} rank {r}: tree differs"
            per_rank.append(dict(ms=float(np.median(times)), bytes=dict(comm.bytes),
                                 calls=comm.calls,
                                 levels=res.stats.get("levels"),
                                 rows_exchanged=res.stats.get("dp_rows_exchanged", 0)))
            ref["recv_codes"] = ref["recv_y"] = None
        ms = [p["ms"] for p in per_rank]
        out = dict(P=P, max_rank_ms=round(max(ms), 3), mean_rank_ms=round(float(np.mean(ms)), 3),
                   rank_ms=[round(v, 3) for v in ms], mode="data", tree_equal=True,
                   levels=per_rank[0]["levels"],
                   bytes_per_rank_mb={k: round(max(p["bytes"][k] for p in per_rank) / 1e6, 2)
                                      for k in per_rank[0]["bytes"]},
                   rows_exchanged=[p["rows_exchanged"] for p in per_rank],
                   # scaling_projection.md's xGMI estimate: S (P - 1) / P / 250 GB/s
                   # + 20 us per collective
                   est_collective_ms=round(max(
                       sum(p["bytes"].values()) * (P - 1) / P / 250e9 * 1e3
                       + 0.020 * p["calls"] for p in per_rank), 3),
                   nodes=ref["fit"].arrays.node_count)
        print(json.dumps(out), flush=True)
        del ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
