"""Per-stage wall times of one fit with device syncs (diagnostics)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from mpitree_amd.utils.datasets import make_classification
from mpitree_amd.core import fit as fitmod
from mpitree_amd.ops.hip_backend import HipBackend, gpu_bin_features

def T(label, fn, reps=5):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps): out = fn()
    torch.cuda.synchronize()
    print(f"{label:40s} {(time.perf_counter()-t)/reps*1e3:8.3f} ms", flush=True)
    return out

X, y = make_classification(1_000_000, 64, seed=0)
T("isfinite(X).all()", lambda: bool(torch.isfinite(X).all()))
T("validate_X", lambda: fitmod._validate_X(X))
T("encode_labels (torch.unique)", lambda: fitmod._encode_labels(y, len(y)))
T("gpu_bin_features", lambda: gpu_bin_features(X, 256))
T("small H2D pinned non_blocking", lambda: torch.ones(16, dtype=torch.int64).pin_memory().to('cuda', non_blocking=True))
up_src = torch.empty(256, dtype=torch.int64).pin_memory()
T("H2D from reused pinned", lambda: up_src.to('cuda', non_blocking=True))
T("D2H small", lambda: torch.zeros(16, device='cuda').cpu())
for md in (12, None):
    res = T(f"fit_tree max_depth={md}", lambda: fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=md, min_samples_split=2, device='cuda'))
    print({k: round(v*1e3, 3) for k, v in res.timings.items()})
