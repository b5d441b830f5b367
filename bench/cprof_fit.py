"""cProfile of the host side of one flagship GPU fit (diagnostics)."""
import cProfile, io, os, pstats, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mpitree_amd.utils.datasets import make_classification
from mpitree_amd.core import fit as fitmod

X, y = make_classification(1_000_000, 64, seed=0, device="cuda")
for _ in range(2):
    fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None, min_samples_split=2, device="cuda")
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None, min_samples_split=2, device="cuda")
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
print(s.getvalue())
