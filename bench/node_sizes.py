"""Internal-node counts of the flagship tree by node size (which engine grows them)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from mpitree_amd import DecisionTreeClassifier  # noqa: E402
from mpitree_amd.utils.datasets import make_classification  # noqa: E402

X, y = make_classification(1_000_000, 64, seed=0, levels=256, device="cuda")
est = DecisionTreeClassifier(device="cuda").fit(X, y)
ta = est.tree_arrays_
m = ta.n_samples[ta.feature >= 0]
edges = [2, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 7812, 1 << 30]
h, _ = np.histogram(m, bins=edges)
print("internal nodes", len(m), "leaves", int((ta.feature < 0).sum()))
for lo, hi, c in zip(edges[:-1], edges[1:], h):
    rows = int(m[(m >= lo) & (m < hi)].sum())
    print(f"  rows [{lo:>6}, {hi:>10}): {c:>7} internal nodes, rows summed {rows:>9}")
