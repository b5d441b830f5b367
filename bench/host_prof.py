"""Host-side (Python) cost of one flagship fit, by function (cProfile).

The GPU idles whenever the host is still preparing the next launch; this lists
where the host time of ``fit_tree`` goes (cumulative and own time per call),
excluding nothing -- waits for the device show up under synchronize.

    python bench/host_prof.py [--n 1000000] [--features 64] [--fits 20] [--regression]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--fits", type=int, default=20)
    ap.add_argument("--regression", action="store_true")
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    from mpitree_amd.core.fit import fit_tree
    from mpitree_amd.utils.datasets import make_classification, make_regression

    dev = torch.device("cuda", 0)
    if a.regression:
        X, y = make_regression(a.n, a.features, levels=256, seed=0, device=dev)
    else:
        X, y = make_classification(a.n, a.features, n_classes=2, seed=0, device=dev)

    def fit():
        return fit_tree(X, y, regression=a.regression, criterion=2 if a.regression else 0,
                        max_depth=None, min_samples_split=2, device="cuda")

    for _ in range(3):
        fit()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.fits):
        fit()
    torch.cuda.synchronize()
    pr.disable()
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(f"==== by {key} ({a.fits} fits)")
        print(s.getvalue())


if __name__ == "__main__":
    main()
