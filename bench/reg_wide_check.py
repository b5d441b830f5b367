"""Wide regression (F past the 4-wave tiny kernel's LDS) on the GPU against the
host builder: the narrow-workgroup regression tiny kernel must give the same tree."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mpitree_amd import DecisionTreeRegressor  # noqa: E402

for n, F in ((20000, 520), (6000, 1000)):
    rng = np.random.default_rng(F)
    X = rng.integers(0, 200, size=(n, F)).astype(np.float32)
    y = (X[:, 0] * 0.5 + X[:, 1] - X[:, 7] + rng.normal(0, 5, n)).astype(np.float64)
    Xd, yd = torch.from_numpy(X).cuda(), torch.from_numpy(y).cuda()
    g = DecisionTreeRegressor(device="cuda").fit(Xd, yd)
    h = DecisionTreeRegressor(device="cpu").fit(X, y)
    ok = g.tree_arrays_.equal(h.tree_arrays_, check_impurity=False)
    print(n, F, g.fit_stats_.get("engine"), g.tree_arrays_.node_count, ok, flush=True)
    assert ok
