"""Host-side probe: time native tree assembly on a real flagship node table."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from mpitree_amd.utils.datasets import make_classification
from mpitree_amd.core import fit as fitmod
from mpitree_amd.core import levelwise as lw
from mpitree_amd.ops import native

cap = {}
orig = lw.LevelwiseBuilder._to_arrays


def spy(self, tab):
    cap["tab"] = tab
    cap["edges"] = self._edges
    return orig(self, tab)


lw.LevelwiseBuilder._to_arrays = spy
X, y = make_classification(1_000_000, 64, seed=0)
for _ in range(3):
    r = fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None,
                        min_samples_split=2, device="cuda")
torch.cuda.synchronize()
tab = cap["tab"]
n = tab.n
cpu = native.cpu()
args = (tab.feature[:n], tab.tbin[:n], tab.left[:n], tab.right[:n], tab.nsamp[:n], tab.stats[:n], 0)
for label, kw in (("plain", ()), ("thr+term", (cap["edges"], 0))):
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        cpu.assemble(*args, *kw)
        ts.append(time.perf_counter() - t)
    print(f"assemble[{label}] n={n}: " + " ".join(f"{v*1e3:.2f}" for v in ts), flush=True)
ts = []
for _ in range(5):
    t = time.perf_counter()
    a = np.empty((n, 8), np.int64); a.fill(0)
    ts.append(time.perf_counter() - t)
print("first-touch 8 cols:", " ".join(f"{v*1e3:.2f}" for v in ts))
print({k: round(v * 1e3, 3) for k, v in r.timings.items()})
