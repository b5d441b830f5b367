"""Diagnostics for the finisher's hand-off queue (one small fit, counters printed)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpitree_amd.ops import hip_backend as hb  # noqa: E402
from mpitree_amd import DecisionTreeClassifier  # noqa: E402
from mpitree_amd.utils.datasets import make_classification  # noqa: E402

orig = hb.HipBackend.launch_finisher


def spy(self, d_jobs, J, *a, **k):
    out = orig(self, d_jobs, J, *a, **k)
    torch.cuda.synchronize()
    c = self._fin_keep[0].cpu().numpy() if torch.is_tensor(self._fin_keep[0]) else None
    print("J", J, "counters", c.tolist(), flush=True)
    return out


hb.HipBackend.launch_finisher = spy
cases = [(50_000, 16, 2), (50_000, 16, 3), (1_000_000, 64, 2)]
if len(sys.argv) > 1:  # "n,F,C[,ENV=V]" ...: each case with its own env settings
    cases = []
    for a in sys.argv[1:]:
        parts = a.split(",")
        cases.append(tuple(int(v) for v in parts[:3]) + (parts[3:],))
for case in cases:
    n, F, C = case[:3]
    for kv in (case[3] if len(case) > 3 else []):
        k, v = kv.split("=")
        os.environ[k] = v
    print("case", case, flush=True)
    X, y = make_classification(n, F, n_classes=C, seed=1, device="cuda")
    clf = DecisionTreeClassifier(device="cuda").fit(X, y)
    same = None
    if n < 100_000:
        h = DecisionTreeClassifier(device="cpu").fit(X.cpu().numpy(), y.cpu().numpy())
        same = clf.tree_arrays_.equal(h.tree_arrays_)
    print(n, F, C, clf.tree_arrays_.node_count, same, flush=True)
