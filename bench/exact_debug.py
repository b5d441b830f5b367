"""Debug probe: the exact engine on the finisher-handoff test's data."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpitree_amd import DecisionTreeClassifier  # noqa: E402

rng = np.random.default_rng(11)
X = rng.normal(size=(30000, 12)).astype(np.float32)
X[:, 3] = np.round(X[:, 3], 2)
y = ((X[:, 0] + X[:, 1] * X[:, 2] + rng.normal(scale=0.5, size=30000)) > 0).astype(np.int64)
a = DecisionTreeClassifier(device="cuda").fit(X, y)
print("default:", a.fit_stats_.get("levels"), a.fit_stats_.get("finisher_subtrees"), flush=True)
os.environ["MPITREE_EXACT_FINISHER_ROWS"] = "0"
b = DecisionTreeClassifier(device="cuda").fit(X, y)
print("fr=0:", b.fit_stats_.get("levels"), b.tree_arrays_.equal(a.tree_arrays_), flush=True)
