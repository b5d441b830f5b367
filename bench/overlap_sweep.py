"""Finisher overlap / grid sweep on the flagship fit (diagnostics)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mpitree_amd.utils.datasets import make_classification
from mpitree_amd.core import fit as fitmod

X, y = make_classification(1_000_000, 64, seed=0)
main = torch.cuda.Stream()
for ov, grid in (("0", "512"), ("1", "512"), ("1", "256"), ("1", "128")):
    os.environ["MPITREE_FIN_OVERLAP"] = ov
    os.environ["MPITREE_FIN_GRID"] = grid
    fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None, min_samples_split=2, device="cuda")
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        with torch.cuda.stream(main):
            r = fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None, min_samples_split=2, device="cuda")
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    tm = {k: round(v * 1e3, 2) for k, v in r.timings.items()}
    print(f"overlap={ov} grid={grid} best={min(ts)*1e3:.2f}ms med={sorted(ts)[2]*1e3:.2f} {tm}", flush=True)
