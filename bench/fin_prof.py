"""Per-workgroup phase profile of the block subtree finisher (diagnostics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MPITREE_FIN_PROF"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpitree_amd.core import fit as fitmod  # noqa: E402
from mpitree_amd.ops import hip_backend as hb  # noqa: E402
from mpitree_amd.utils.datasets import make_classification  # noqa: E402

keep = {}
orig = hb.HipBackend.launch_finisher


def spy(self, d_jobs, J, *a, **k):
    out = orig(self, d_jobs, J, *a, **k)
    keep["prof"] = self.last_finisher_prof
    keep["counts"] = d_jobs[:, 1].cpu().numpy()
    return out


hb.HipBackend.launch_finisher = spy
C_ARG = int(os.environ.get("FIN_PROF_CLASSES", "2"))
X, y = make_classification(1_000_000, 64, n_classes=C_ARG, seed=0)
for _ in range(3):
    r = fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None, min_samples_split=2,
                        device="cuda")
torch.cuda.synchronize()
P = keep["prof"]
wall = (P[:, 1] - P[:, 0]) / 100.0  # 100 MHz wall clock -> us
start = (P[:, 0] - P[:, 0].min()) / 100.0
print(f"blocks={len(P)} jobs={len(keep['counts'])} job rows: max={keep['counts'].max()} "
      f"mean={keep['counts'].mean():.0f}")
print(f"wall us: max={wall.max():.0f} mean={wall.mean():.0f} p50={np.median(wall):.0f} "
      f"start max={start.max():.1f}")
end = (P[:, 1] - P[:, 0].min()) / 100.0
q = np.percentile(end, [10, 50, 90, 99])
print(f"block end us: p10={q[0]:.0f} p50={q[1]:.0f} p90={q[2]:.0f} p99={q[3]:.0f} "
      f"max={end.max():.0f}; idle share of the span {(end.max() - end).mean() / end.max():.1%}")
print(f"nodes/block: max={P[:, 2].max()} mean={P[:, 2].mean():.1f} total={P[:, 2].sum()}; "
      f"rows/block: max={P[:, 3].max()} mean={P[:, 3].mean():.0f} total={P[:, 3].sum()}")
cyc = P[:, 4:9].sum(0)
names = ["hist", "scan(exact)", "partition", "rest", "scan(fp32)"]
print("cycle split:", {n: f"{100*c/cyc.sum():.1f}%" for n, c in zip(names, cyc)})
print(f"cycles per node: {cyc.sum() / P[:, 2].sum():.0f}; "
      f"hist cycles per row: {cyc[0] / P[:, 3].sum():.1f}")
i = int(np.argmax(wall))
print(f"slowest block: wall={wall[i]:.0f}us nodes={P[i, 2]} rows={P[i, 3]} "
      f"cycles={P[i, 4:9].tolist()}")
print(f"exact-rescored features per node: {P[:, 9].sum() / P[:, 2].sum():.2f}")
print({k: round(v * 1e3, 3) for k, v in r.timings.items()})
