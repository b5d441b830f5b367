"""Sweep the finisher threshold on the flagship data (diagnostics)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpitree_amd.core import fit as fitmod
from mpitree_amd.utils.datasets import make_classification

X, y = make_classification(1_000_000, 64, seed=0)
frs = [int(v) for v in os.environ.get("SWEEP_FR", "512,1024,2048,4096").split(",")]
for md in (None,):
    for fr in frs:
        os.environ["MPITREE_FINISHER_ROWS"] = str(fr)
        for _ in range(2):
            fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=md,
                            min_samples_split=2, device="cuda")
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            r = fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=md,
                                min_samples_split=2, device="cuda")
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        tm = {k: round(v * 1e3, 2) for k, v in r.timings.items()}
        print(f"md={md} fr={fr} best={min(ts)*1e3:.2f}ms nodes={r.arrays.node_count} "
              f"levels={r.stats.get('levels')} jobs={r.stats.get('finisher_subtrees')} {tm}",
              flush=True)
