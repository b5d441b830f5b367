"""Per-rank critical path of a P-GPU feature-parallel fit, measured on ONE GPU.

The multi-GPU ``auto`` fit runs the feature-parallel device level loop (each
rank builds and scans histograms of its F/P feature block; one RCCL all-gather
of split records per level, ``fp_combine_kernel``; the planner and partition
are replicated), then its serpentine share of the subtree finisher jobs, then
one all-gather of the finished nodes. This script runs that exact kernel
sequence for rank 0 in one process: a stand-in communicator reports
``world_size = P`` / ``rank = 0`` and replaces each collective by a local copy
(rank 0's records in every slot), and ``MPITREE_SIM_RANKS = P`` times rank 0's
finisher share alone before finishing the other shares (the tree stays
complete, but it splits only on block-0 features, so its node counts differ a
little from the 1-GPU tree). Reported per P (median of ``--reps`` fits):

* ``fit_ms``: the whole stand-in fit (binning, levels, all finisher shares, assembly);
* ``levels_ms``: the level loop's device time (``MPITREE_PROFILE`` events:
  histogram, derive, scan + combine, plan, partition per level);
* ``rank0_fin_ms`` / ``rest_fin_ms``: rank 0's finisher share / the others';
* ``est_rank_ms = fit_ms - rest_fin_ms``: one rank's fit without the collective
  latencies -- ``collectives`` counts them (one per level + the node exchange,
  each a few to a few tens of us on xGMI).

    python bench/sim_fp_ranks.py [--n 1000000] [--features 64] [--ranks 1,2,4,8]
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
from mpitree_amd.parallel.strategies import feature_blocks  # noqa: E402


class SimFeatureComm(LocalComm):
    """Rank 0 of a P-rank feature-parallel group, without other ranks."""

    kind = "feature"
    simulated = True

    def __init__(self, P: int, device):
        self.world_size = P
        self.rank = 0
        self.device = device
        self.bytes_communicated = 0
        self.collectives = 0

    def feature_range(self, F: int):
        return feature_blocks(F, self.world_size)[0]

    def all_gather_device(self, out, inp):
        out.view(self.world_size, -1).copy_(inp.reshape(1, -1).expand(self.world_size, -1))
        self.bytes_communicated += inp.numel() * inp.element_size() * self.world_size
        self.collectives += 1

    def all_gather_rows(self, t):
        self.bytes_communicated += t.numel() * t.element_size() * self.world_size
        self.collectives += 1
        return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from mpitree_amd.core.fit import fit_tree
    from mpitree_amd.utils.datasets import make_classification

    dev = torch.device("cuda", 0)
    X, y = make_classification(a.n, a.features, n_classes=2, seed=0, device=dev)
    for P in [int(v) for v in a.ranks.split(",")]:
        rows = []
        for i in range(a.reps + 2):
            comm = SimFeatureComm(P, dev) if P > 1 else None
            os.environ["MPITREE_SIM_RANKS"] = str(P) if P > 1 else "0"
            os.environ["MPITREE_PROFILE"] = "0"
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fit_tree(X, y, regression=False, criterion=0, max_depth=None,
                         min_samples_split=2, device="cuda", comm=comm)
            torch.cuda.synchronize()
            fit_ms = (time.perf_counter() - t0) * 1e3
            # the level loop's device time, from a profiled fit (events per kernel group)
            os.environ["MPITREE_PROFILE"] = "1"
            rp = fit_tree(X, y, regression=False, criterion=0, max_depth=None,
                          min_samples_split=2, device="cuda",
                          comm=SimFeatureComm(P, dev) if P > 1 else None)
            lv = rp.stats.get("level_profile") or []
            levels_ms = float(sum(sum(d.values()) for d in lv))
            st = r.stats
            if i >= 2:
                rows.append(dict(fit_ms=fit_ms, levels_ms=levels_ms,
                                 rank0_fin_ms=st.get("sim_rank0_finisher_ms", float("nan")),
                                 rest_fin_ms=st.get("sim_rest_finisher_ms", 0.0),
                                 levels=st.get("levels"), nodes=r.arrays.node_count,
                                 collectives=getattr(comm, "collectives", 0),
                                 comm_bytes=getattr(comm, "bytes_communicated", 0)))
        os.environ["MPITREE_PROFILE"] = "0"
        med = {k: float(np.median([row[k] for row in rows])) for k in rows[0]}
        med["est_rank_ms"] = med["fit_ms"] - (med["rest_fin_ms"] if P > 1 else 0.0)
        med["P"] = P
        med["feature_block"] = list(feature_blocks(a.features, P)[0])
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in med.items()}),
              flush=True)


if __name__ == "__main__":
    main()
