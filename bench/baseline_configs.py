#!/usr/bin/env python
"""Every BASELINE.json configuration, plus the reference's published sweep.

One JSON line per config (wall-clock per fit, samples/s, tree size):

  iris        Iris 150x4, single-process CPU fit (the native host builder)
  sweep       the notebook's published workload (experiments.ipynb:198-209):
              X = arange(n)[:, None], y = arange(n) (every sample its own
              class), n = 1..241 step 10; CPU, compared with time_data.csv
  sweep_gpu   the same workload fitted on one MI355X
  100k        100k x 32 synthetic classification, max_depth=12, 1 GPU
  1m          1M x 64 synthetic classification (flagship; bench.py), 1 GPU
  1m_exact    1M x 64 continuous (randn) features: every unique value a threshold
              (the reference's search; the presorted-list exact engine), 1 GPU
  100k_exact  100k x 32 continuous, max_depth=12, exact engine, 1 GPU
  1m_reg      1M x 64 regression tree (squared error), 1 GPU
  1m_exact_reg  1M x 64 continuous regression, exact thresholds (presorted lists), 1 GPU
  1m_q1024    1M x 64 continuous features, 1024 quantile bins (16-bit codes), 1 GPU
  1m_c64      1M x 64 classification with 64 classes, 1 GPU (feature-tiled finisher)
  200k_f512   200k x 512 classification, 1 GPU (feature-tiled finisher)
  1m_c300     1M x 64 classification with 300 classes (class-tiled level histograms,
              255-row finisher jobs), 1 GPU
  200k_f512_reg  200k x 512 regression (regression finisher past 256 features), 1 GPU
  10m         10M x 128 synthetic classification, 1 GPU (the 8-GPU
              data-parallel run is bench.py under torchrun)

Usage: python bench/baseline_configs.py [names...] [--reps R]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# published k=8 MPI times (ms) for n = 1, 11, ..., 241 (reference time_data.csv:3)
PUBLISHED_K8_MS = None


def _published():
    path = "/root/reference/time_data.csv"
    if not os.path.exists(path):
        return None
    rows = [list(map(float, line.split(","))) for line in open(path) if line.strip()]
    return {2: rows[0], 5: rows[1], 8: rows[2]} if len(rows) >= 3 else None


def _time(fn, reps, warmup=2, sync=None):
    for _ in range(warmup):
        fn()
    if sync:
        sync()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        if sync:
            sync()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)), float(np.min(ts))


def run_iris(reps):
    from sklearn.datasets import load_iris

    from mpitree_amd import DecisionTreeClassifier

    X, y = load_iris(return_X_y=True)
    out = []
    for md in (None, 3):
        est = DecisionTreeClassifier(max_depth=md, device="cpu")
        med, best = _time(lambda: est.fit(X, y), reps)
        out.append({"config": f"iris150x4_cpu_max_depth={md}", "ms_median": med * 1e3,
                    "ms_best": best * 1e3, "samples_per_sec": 150 / med,
                    "nodes": est.tree_arrays_.node_count,
                    "reference_ms": {None: 20.7, 3: 15.2}[md],
                    "engine": est.fit_stats_["engine"]})
    return out


def run_sweep(reps):
    from mpitree_amd import DecisionTreeClassifier

    pub = _published()
    out = []
    for i, n in enumerate(range(1, 242, 10)):
        X = np.arange(n).reshape(-1, 1)
        y = np.arange(n)
        est = DecisionTreeClassifier(device="cpu")
        med, best = _time(lambda: est.fit(X, y), reps)
        row = {"config": f"sweep_n={n}", "ms_median": med * 1e3, "ms_best": best * 1e3,
               "nodes": est.tree_arrays_.node_count}
        if pub:
            row["reference_k8_ms"] = pub[8][i]
            row["reference_k2_ms"] = pub[2][i]
        out.append(row)
    return out


def run_sweep_gpu(reps):
    """The published workload on one MI355X (device tensors in, tree out)."""
    import torch

    from mpitree_amd import DecisionTreeClassifier

    pub = _published()
    out = []
    for i, n in enumerate(range(1, 242, 10)):
        X = torch.arange(n, dtype=torch.float32, device="cuda").reshape(-1, 1)
        y = torch.arange(n, device="cuda")
        est = DecisionTreeClassifier(device="cuda")
        med, best = _time(lambda: est.fit(X, y), reps, sync=torch.cuda.synchronize)
        row = {"config": f"sweep_gpu_n={n}", "ms_median": med * 1e3, "ms_best": best * 1e3,
               "nodes": est.tree_arrays_.node_count, "engine": est.fit_stats_["engine"]}
        if pub:
            row["reference_k8_ms"] = pub[8][i]
        out.append(row)
    return out


def _gpu_fit(n, F, reps, md=None, regression=False, classes=2, seed=0, levels=256,
             max_bins=None):
    import torch

    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    if regression:
        X, y = make_regression(n, F, seed=seed, levels=levels)
        est = DecisionTreeRegressor(max_depth=md, device="cuda", max_bins=max_bins)
    else:
        X, y = make_classification(n, F, n_classes=classes, seed=seed, levels=levels)
        est = DecisionTreeClassifier(max_depth=md, device="cuda", max_bins=max_bins)
    med, best = _time(lambda: est.fit(X, y), reps, sync=torch.cuda.synchronize)
    st = est.fit_stats_
    return {"ms_median": med * 1e3, "ms_best": best * 1e3, "samples_per_sec": n / med,
            "nodes": st["node_count"], "depth": st["max_depth"], "engine": st["engine"],
            "timings_ms": {k: round(v * 1e3, 3) for k, v in st["timings"].items()}}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*",
                    default=["iris", "sweep", "sweep_gpu", "100k", "1m", "1m_exact",
                             "100k_exact", "1m_reg", "1m_exact_reg", "1m_q1024", "1m_c64",
                             "200k_f512", "1m_c300", "200k_f512_reg", "10m"])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args(argv)
    for name in a.names:
        if name == "iris":
            rows = run_iris(max(a.reps, 20))
        elif name == "sweep":
            rows = run_sweep(max(a.reps, 20))
        elif name == "sweep_gpu":
            rows = run_sweep_gpu(max(a.reps, 10))
        elif name == "100k":
            rows = [{"config": "100k x 32 classification, max_depth=12, 1 GPU",
                     **_gpu_fit(100_000, 32, a.reps, md=12)}]
        elif name == "1m":
            rows = [{"config": "1M x 64 classification, full depth, 1 GPU",
                     **_gpu_fit(1_000_000, 64, a.reps)}]
        elif name == "1m_exact":
            rows = [{"config": "1M x 64 continuous (randn) classification, exact thresholds, "
                               "full depth, 1 GPU",
                     **_gpu_fit(1_000_000, 64, max(2, a.reps // 2), levels=None)}]
        elif name == "100k_exact":
            rows = [{"config": "100k x 32 continuous (randn) classification, exact thresholds, "
                               "max_depth=12, 1 GPU",
                     **_gpu_fit(100_000, 32, a.reps, md=12, levels=None)}]
        elif name == "1m_reg":
            rows = [{"config": "1M x 64 regression (squared_error), full depth, 1 GPU",
                     **_gpu_fit(1_000_000, 64, a.reps, regression=True)}]
        elif name == "1m_exact_reg":
            rows = [{"config": "1M x 64 continuous (randn) regression, exact thresholds, "
                               "full depth, 1 GPU",
                     **_gpu_fit(1_000_000, 64, max(2, a.reps // 2), regression=True,
                                levels=None)}]
        elif name == "1m_q1024":
            rows = [{"config": "1M x 64 continuous (randn) classification, 1024 quantile bins "
                               "(16-bit codes), full depth, 1 GPU",
                     **_gpu_fit(1_000_000, 64, max(2, a.reps // 2), levels=None, max_bins=1024)}]
        elif name == "1m_c64":
            rows = [{"config": "1M x 64 classification, 64 classes, full depth, 1 GPU",
                     **_gpu_fit(1_000_000, 64, max(2, a.reps // 2), classes=64)}]
        elif name == "200k_f512":
            rows = [{"config": "200k x 512 classification, full depth, 1 GPU",
                     **_gpu_fit(200_000, 512, a.reps)}]
        elif name == "1m_c300":
            rows = [{"config": "1M x 64 classification, 300 classes, full depth, 1 GPU",
                     **_gpu_fit(1_000_000, 64, max(2, a.reps // 2), classes=300)}]
        elif name == "200k_f512_reg":
            rows = [{"config": "200k x 512 regression (squared_error), full depth, 1 GPU",
                     **_gpu_fit(200_000, 512, a.reps, regression=True)}]
        elif name == "10m":
            rows = [{"config": "10M x 128 classification, full depth, 1 GPU",
                     **_gpu_fit(10_000_000, 128, max(2, a.reps // 2))}]
        else:
            raise SystemExit(f"unknown config {name}")
        for r in rows:
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
