"""Sweep finisher thresholds on the flagship data (diagnostics)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mpitree_amd.utils.datasets import make_classification
from mpitree_amd.core import fit as fitmod

X, y = make_classification(1_000_000, 64, seed=0)
for md in (None, 12):
    for fr in [int(v) for v in os.environ.get('SWEEP_FR', '1024,2048,4096,8192').split(',')]:
        for tiny in [int(v) for v in os.environ.get('SWEEP_TINY', '64').split(',')]:
            os.environ["MPITREE_FINISHER_ROWS"] = str(fr)
            os.environ["MPITREE_TINY_ROWS"] = str(tiny)
            fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=md, min_samples_split=2, device="cuda")
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                t = time.perf_counter()
                r = fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=md, min_samples_split=2, device="cuda")
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            tm = {k: round(v * 1e3, 2) for k, v in r.timings.items()}
            print(f"md={md} fr={fr} tiny={tiny} best={min(ts)*1e3:.2f}ms nodes={r.arrays.node_count} "
                  f"levels={r.stats.get('levels')} jobs={r.stats.get('finisher_subtrees')} {tm}", flush=True)
