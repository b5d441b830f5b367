import cProfile, pstats, sys, torch
sys.path.insert(0, '.')
from mpitree_amd import DecisionTreeClassifier
from mpitree_amd.utils.datasets import make_classification
X, y = make_classification(1_000_000, 64, seed=0)
clf = DecisionTreeClassifier(device="cuda")
clf.fit(X, y); torch.cuda.synchronize()
pr = cProfile.Profile(); pr.enable()
for _ in range(3): clf.fit(X, y)
torch.cuda.synchronize(); pr.disable()
pstats.Stats(pr).sort_stats('tottime').print_stats(25)
