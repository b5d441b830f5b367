"""Host-side (Python) profile of the flagship GPU fit: cProfile over warm fits.

Usage: python bench/host_prof.py [--fits 20] [--n 1000000] [--features 64]
"""
import argparse
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpitree_amd import DecisionTreeClassifier  # noqa: E402
from mpitree_amd.utils.datasets import make_classification  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--fits", type=int, default=20)
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--features", type=int, default=64)
a = ap.parse_args()
X, y = make_classification(a.n, a.features, seed=0, device=torch.device("cuda"))
est = DecisionTreeClassifier(device="cuda")
for _ in range(3):
    est.fit(X, y)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(a.fits):
    est.fit(X, y)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(30)
