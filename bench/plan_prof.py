"""Per-phase time of the level planner (grow_plan_kernel) on the flagship fit.

Needs the planner built with -DMT_PLAN_PROF (tools/build_variant.sh planprof
grow.hip -DMT_PLAN_PROF swapped in for the extension): every launch adds each
phase's wall-clock ticks (100 MHz) to a device array, read back here.

    python bench/plan_prof.py [--n 1000000] [--features 64] [--fits 10] [--regression]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["select", "own-switch", "totals", "decide+write", "hist items", "part items",
          "minmax+ctl"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--fits", type=int, default=10)
    ap.add_argument("--regression", action="store_true")
    a = ap.parse_args()
    import mpitree_amd._hip as hipmod
    from mpitree_amd.core.fit import fit_tree
    from mpitree_amd.utils.datasets import make_classification, make_regression

    lib = ctypes.CDLL(hipmod.__file__)
    read = lib.mt_plan_prof_read
    buf = (ctypes.c_ulonglong * 32)()
    dev = torch.device("cuda", 0)
    if a.regression:
        X, y = make_regression(a.n, a.features, levels=256, seed=0, device=dev)
    else:
        X, y = make_classification(a.n, a.features, n_classes=2, seed=0, device=dev)

    def fit():
        return fit_tree(X, y, regression=a.regression, criterion=2 if a.regression else 0,
                        max_depth=None, min_samples_split=2, device="cuda")

    for _ in range(2):
        fit()
    read(buf)  # (reset)
    for _ in range(a.fits):
        r = fit()
    torch.cuda.synchronize()
    read(buf)
    v = np.array(buf[:], dtype=np.float64)
    calls = v[31]
    print(f"plan launches: {int(calls)} ({calls / a.fits:.1f} per fit, "
          f"{r.stats.get('levels')} levels)")
    tot = 0.0
    for k, name in enumerate(PHASES):
        us = v[k] / calls * 0.01  # 100 MHz ticks -> us
        tot += us
        print(f"  {name:14s} {us:7.2f} us/launch")
    print(f"  {'total':14s} {tot:7.2f} us/launch, {tot * calls / a.fits:8.1f} us/fit")


if __name__ == "__main__":
    main()
