"""One flagship (PMC_REG=1: regression) fit after a warmup -- a small trace for PMC counter runs.

rocprofv3 --pmc SQ_INSTS_VALU ... --kernel-trace --output-format csv -- python3 bench/pmc_fit.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor  # noqa: E402
from mpitree_amd.utils.datasets import make_classification, make_regression  # noqa: E402

n = int(os.environ.get("PMC_N", 1_000_000))
F = int(os.environ.get("PMC_F", 64))
if os.environ.get("PMC_REG"):  # the regression config (MSE criterion)
    X, y = make_regression(n, F, seed=0, device=torch.device("cuda", 0))
    est = DecisionTreeRegressor(device="cuda")
else:  # PMC_EXACT=1: continuous features (the exact-threshold engine)
    lv = None if os.environ.get("PMC_EXACT") else 256
    X, y = make_classification(n, F, seed=0, device=torch.device("cuda", 0), levels=lv)
    est = DecisionTreeClassifier(device="cuda")
est.fit(X, y)
torch.cuda.synchronize()
est.fit(X, y)
torch.cuda.synchronize()
print(est.fit_stats_.get("node_count"))
