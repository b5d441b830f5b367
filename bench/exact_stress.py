"""Repeated exact-engine fits on small random problems vs the CPU builder
(stress check of the ticketed look-back partition): prints one line per fit."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpitree_amd import DecisionTreeClassifier  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
bad = 0
for i in range(reps):
    rng = np.random.default_rng(i)
    n, F, C = int(rng.integers(2000, 60000)), int(rng.integers(2, 20)), int(rng.integers(2, 4))
    X = np.round(rng.normal(size=(n, F)), 3).astype(np.float32)
    s = X[:, 0] + 0.5 * X[:, 1 % F] + rng.normal(scale=0.7, size=n)
    y = np.digitize(s, np.quantile(s, np.linspace(0, 1, C + 1)[1:-1]))
    g = DecisionTreeClassifier(device="cuda").fit(X, y)
    h = DecisionTreeClassifier(device="cpu").fit(X, y)
    ok = g.tree_arrays_.equal(h.tree_arrays_)
    bad += not ok
    print(f"fit {i}: n={n} F={F} C={C} engine={g.fit_stats_['engine']} equal={ok}", flush=True)
print("bad", bad, flush=True)
sys.exit(1 if bad else 0)
