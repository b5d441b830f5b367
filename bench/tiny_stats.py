"""Shape statistics of the tiny (<= 64-row) subtrees of the flagship tree (diagnostics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpitree_amd import DecisionTreeClassifier  # noqa: E402
from mpitree_amd.utils.datasets import make_classification  # noqa: E402

X, y = make_classification(1_000_000, 64, seed=0, device=torch.device("cuda", 0))
ta = DecisionTreeClassifier(device="cuda").fit(X, y).tree_arrays_
n, left, right = ta.n_samples, ta.left, ta.right
N = len(n)
parent = np.full(N, -1)
inner = left >= 0
parent[left[inner]] = np.nonzero(inner)[0]
parent[right[inner]] = np.nonzero(inner)[0]
roots = np.nonzero((n <= 64) & (parent >= 0) & (n[np.maximum(parent, 0)] > 64))[0]
# internal nodes per tiny subtree: walk pre-order ranges (a subtree is contiguous)
size = np.zeros(N, np.int64)
for i in range(N - 1, -1, -1):
    size[i] = 1 + (size[left[i]] + size[right[i]] if left[i] >= 0 else 0)
internal = np.array([int((left[r:r + size[r]] >= 0).sum()) for r in roots])
rows = n[roots]
print(f"nodes={N} tiny subtrees={len(roots)} rows: mean={rows.mean():.1f} "
      f"hist={np.histogram(rows, bins=[1, 2, 3, 5, 9, 17, 33, 65])[0].tolist()}")
print(f"internal per subtree: mean={internal.mean():.2f} total={internal.sum()} "
      f"zero={int((internal == 0).sum())} hist={np.histogram(internal, bins=[0, 1, 2, 4, 8, 16, 32, 64])[0].tolist()}")
print(f"block-finisher internal nodes (n > 64): {int(((n > 64) & inner).sum())}")
