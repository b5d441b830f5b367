"""Calibration table for the multi-rank level heuristics (``fp_prefix_pays``).

``ops/device_grower.fp_prefix_pays`` weighs what a feature-parallel prefix level
saves -- (1 - 1/P) of the level's histogram build, a cost per row x feature --
against what it adds (a record all-gather, a select and a combine). This script
measures the first term on the GPU instead of assuming it: the level-0
histogram (``hist`` + slab reduction, device events of ``MPITREE_PROFILE=1``)
of single-level fits over a grid of (rows, features), classification and
regression, and fits ``t = a + b * rows * features`` per task by least squares.

    python bench/calib_hist.py [--reps 5]      -> one JSON line per point + a fit line

The level-0 histogram is every row of every feature -- the same work per row x
feature as the top levels' built children, which the prefix divides by P.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rows", default="250000,500000,1000000,2000000,4000000")
    ap.add_argument("--features", default="16,32,64,128")
    a = ap.parse_args()
    os.environ["MPITREE_PROFILE"] = "1"  # per-phase device events (host-driven level path)
    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    dev = torch.device("cuda", 0)
    out = {}
    for reg in (False, True):
        pts = []
        for F in [int(v) for v in a.features.split(",")]:
            for n in [int(v) for v in a.rows.split(",")]:
                if reg:
                    X, y = make_regression(n, F, seed=1, device=dev)
                    est = DecisionTreeRegressor(max_depth=2, device="cuda")
                else:
                    X, y = make_classification(n, F, seed=1, device=dev)
                    est = DecisionTreeClassifier(max_depth=2, device="cuda")
                est.fit(X, y)  # warmup (workspaces, tables)
                ts = []
                for _ in range(a.reps):
                    est.fit(X, y)
                    lp = est.fit_stats_.get("level_profile") or []
                    if lp:
                        ts.append(lp[0].get("hist", 0.0))  # (histogram items + slab reduction)
                t = float(np.median(ts)) if ts else float("nan")
                pts.append((n * F, t))
                print(json.dumps({"task": "regression" if reg else "classification", "rows": n,
                                  "features": F, "level0_hist_ms": round(t, 4),
                                  "ps_per_row_feature": round(t * 1e9 / (n * F), 3)}), flush=True)
                del X, y, est
                torch.cuda.empty_cache()
        A = np.array([[1.0, x] for x, _ in pts])
        b = np.array([t for _, t in pts])
        ok = np.isfinite(b)
        coef, *_ = np.linalg.lstsq(A[ok], b[ok], rcond=None)
        out["regression" if reg else "classification"] = coef
        print(json.dumps({"task": "regression" if reg else "classification",
                          "fit": "t_ms = a + b * rows * features",
                          "a_us": round(coef[0] * 1e3, 2),
                          "b_ps_per_row_feature": round(coef[1] * 1e9, 4)}), flush=True)


if __name__ == "__main__":
    main()
