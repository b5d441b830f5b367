import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
from mpitree_amd.utils.datasets import make_classification
from mpitree_amd.core import fit as fitmod
X, y = make_classification(10_000_000, 128, seed=0)
for fr in (2048, 4096, 8192, 19531):
    os.environ["MPITREE_FINISHER_ROWS"] = str(fr)
    fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None, min_samples_split=2, device="cuda")
    torch.cuda.synchronize()
    ts=[]
    for _ in range(2):
        t=time.perf_counter()
        r = fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None, min_samples_split=2, device="cuda")
        torch.cuda.synchronize(); ts.append(time.perf_counter()-t)
    print(fr, round(min(ts)*1e3,2), {k: round(v*1e3,2) for k,v in r.timings.items()}, r.stats.get("levels"), r.stats.get("finisher_subtrees"), flush=True)
