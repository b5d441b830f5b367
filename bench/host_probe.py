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
    cap["fin"] = self._fin
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
fin, cnt, did, roots = cap["fin"]
fin = np.array(fin); cnt = np.array(cnt)
print("affinity cpus:", len(os.sched_getaffinity(0)), "host_threads:", native.host_threads())
for nt in (1, 4, 8, 16):
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        a = cpu.assemble_tree(tab.feature[:n], tab.tbin[:n], tab.left[:n], tab.right[:n],
                              tab.nsamp[:n], tab.stats[:n], fin, cnt, did, roots, cap["edges"], 0, nt)
        ts.append(time.perf_counter() - t)
    print(f"assemble_tree threads={nt} n1={n} T={len(fin)}: total " + " ".join(f"{v*1e3:.2f}" for v in ts)
          + f" | order {a['ms_order']:.2f} scatter {a['ms_scatter']:.2f}", flush=True)
print({k: round(v * 1e3, 3) for k, v in r.timings.items()})
