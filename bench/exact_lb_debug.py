"""Debug probe: one small exact fit with per-level sync and look-back status."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MPITREE_EXACT_SYNC", "2")
from mpitree_amd import DecisionTreeClassifier  # noqa: E402

n, F, C = 3000, 3, 2
rng = np.random.default_rng(n + F)
X = np.round(rng.normal(size=(n, F)), 4).astype(np.float32)
X[:, 0] = np.round(X[:, 0], 1)
s = X[:, 0] + 0.7 * X[:, 1] + rng.normal(scale=0.8, size=n)
y = np.digitize(s, np.quantile(s, np.linspace(0, 1, C + 1)[1:-1]))
try:
    g = DecisionTreeClassifier(device="cuda").fit(X, y)
    h = DecisionTreeClassifier(device="cpu").fit(X, y)
    print("equal:", g.tree_arrays_.equal(h.tree_arrays_), g.tree_arrays_.node_count,
          h.tree_arrays_.node_count, flush=True)
except Exception as e:  # noqa: BLE001
    print("error:", e, flush=True)
