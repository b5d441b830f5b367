"""Time the flagship fit under several environment settings in one process.

Usage: python bench/sweep_env.py MPITREE_FINISHER_ROWS=1024,2048,4096 [--reps 10]
       [--n 1000000] [--features 64] [--regression]
Each knob value is applied with ``os.environ`` before its fits (the knobs are
read per fit / per launch); prints one JSON line per setting with the median
and best ms per fit.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor  # noqa: E402
from mpitree_amd.utils.datasets import make_classification, make_regression  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("knobs", nargs="*", help="NAME=v1,v2,... (first knob varies)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--regression", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    if a.regression:
        X, y = make_regression(a.n, a.features, seed=0, device=dev)
        est = DecisionTreeRegressor(device="cuda")
    else:
        X, y = make_classification(a.n, a.features, seed=0, device=dev)
        est = DecisionTreeClassifier(device="cuda")
    settings = [[]]
    for k in a.knobs:
        name, vals = k.split("=", 1)
        settings = [s + [(name, v)] for s in settings for v in vals.split(",")]
    for s in settings:
        for name, v in s:
            os.environ[name] = v
        for _ in range(2):
            est.fit(X, y)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            est.fit(X, y)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        print(json.dumps({"setting": dict(s), "median_ms": round(ts[len(ts) // 2], 3),
                          "best_ms": round(ts[0], 3), "nodes": est.tree_arrays_.node_count}),
              flush=True)


if __name__ == "__main__":
    main()
