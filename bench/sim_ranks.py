"""Per-rank critical path of a P-GPU ``auto`` fit, measured on ONE GPU.

In the multi-GPU device path every rank runs the (replicated) level loop and a
serpentine share of the finisher jobs, then all-gathers the finished nodes.
``MPITREE_SIM_RANKS=P`` makes a single-process fit time rank 0's share alone on
the GPU (then finish the other shares so the tree is complete); the estimated
per-rank fit time is ``T - rest`` (the all-gather is not included). Sweeping
``MPITREE_FINISHER_ROWS`` shows where the split point between replicated levels
and divided finisher work should sit for each P.

    python bench/sim_ranks.py [--n 1000000] [--features 64] [--fr 512,1024,2048]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--fr", default="256,512,1024,2048,4096")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--regression", action="store_true")
    a = ap.parse_args()
    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    dev = torch.device("cuda", 0)
    if a.regression:
        X, y = make_regression(a.n, a.features, seed=0, device=dev)
        est = DecisionTreeRegressor(device="cuda")
    else:
        X, y = make_classification(a.n, a.features, n_classes=2, seed=0, device=dev)
        est = DecisionTreeClassifier(device="cuda")
    for fr in [int(v) for v in a.fr.split(",")]:
        os.environ["MPITREE_FINISHER_ROWS"] = str(fr)
        for P in [int(v) for v in a.ranks.split(",")]:
            os.environ["MPITREE_SIM_RANKS"] = str(P)
            ts, r0, rest = [], [], []
            for i in range(a.reps + 2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                est.fit(X, y)
                torch.cuda.synchronize()
                if i >= 2:
                    ts.append((time.perf_counter() - t0) * 1e3)
                    st = est.fit_stats_
                    r0.append(st.get("sim_rank0_finisher_ms", float("nan")))
                    rest.append(st.get("sim_rest_finisher_ms", 0.0))
            st = est.fit_stats_
            T = float(np.median(ts))
            out = dict(fr=fr, P=P, fit_ms=round(T, 3),
                       rank0_fin_ms=round(float(np.median(r0)), 3),
                       rest_fin_ms=round(float(np.median(rest)), 3),
                       est_rank_ms=round(T - float(np.median(rest)), 3),
                       levels=st.get("levels"), jobs=st.get("finisher_subtrees"),
                       rank0_jobs=st.get("sim_rank0_jobs"), nodes=st.get("node_count"))
            print(json.dumps(out), flush=True)
    os.environ.pop("MPITREE_SIM_RANKS", None)


if __name__ == "__main__":
    main()
