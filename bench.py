#!/usr/bin/env python
"""Headline benchmark: decision-tree fit on 1M x 64 synthetic data.

BASELINE.json metric: "tree fit wall-clock (s) + samples/sec, 1M x 64
synthetic at 1/2/4/8 GPUs". One *step* is one complete ``fit`` of a
``DecisionTreeClassifier`` (entropy, the reference's criterion and default
hyperparameters unless overridden) from raw device features to the finished
tree: input validation, label encoding, feature binning, level-wise growth,
subtree finishing, device assembly of every tree column (features, bins,
thresholds, child links, depths, node sizes, class counts, impurities) and
the host copy of those columns. ``fit`` returns a finished ``TreeArrays``:
no column is derived on the host after the timer stops (``"materialized":
true``).

``--continuous`` fits N(0, 1) features (every value distinct): the
reference's threshold semantics (every unique value a candidate) then run on
the presorted-list exact engine instead of the <= 256-value histogram engines.

Single GPU: ``python bench.py``. Multi-GPU (one process per GPU, RCCL):
``torchrun --nproc-per-node N bench.py --gpus N``, or ``python bench.py --gpus N``,
which starts the N rank processes itself (``torch.distributed.run`` as a child
process, before this process touches the GPU); ``--gpus`` must equal the
launcher's ``WORLD_SIZE`` and fewer visible GPUs than ``--gpus`` is an error
(never a silent one-rank run). Every rank holds the full
data (the reference's ParallelDecisionTreeClassifier contract) and the total
work is fixed, so scaling is "strong". ``--strategy auto`` (default) runs
subtree ownership: the device level loop replicated until a level holds >= 4N
units, then each rank grows only the subtrees the device planner assigned it
(LPT on rows; level loop and finisher, no per-level collective) and one RCCL
all-gather of finished position ranges completes the tree on every rank;
``--strategy feature`` runs the feature-parallel level loop (F/N features per
rank, one all-gather of split records per level); ``--strategy data`` runs
row-sharded histograms reduced per feature block to their owner ranks (BASELINE
config 4: ``--n 10000000 --features 128 --strategy data``). The JSON line reports the
level loop that actually ran (``config.level_loop``) and the bytes moved.

Every quantized-data run also times the same estimator on the continuous
companion data set (same shape and label model, N(0, 1) features: the
reference's every-unique-value threshold semantics on the presorted-list exact
engine) and reports it as ``continuous_ms_per_step`` next to the headline
(``--no-continuous`` skips it; ``--continuous`` makes it the headline).

``MPITREE_BENCH_BACKEND=gloo`` rehearses the multi-rank path with ranks
sharing the visible GPUs (collectives over gloo instead of RCCL).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch


# BASELINE.json's headline metric and the configurations it names
METRIC = "tree fit wall-clock (s) + samples/sec, 1M\u00d764 synthetic at 1/2/4/8 GPUs"
CONFIG = "1M\u00d764 synthetic, feature-parallel split search, RCCL all-reduce on 8\u00d7MI355X"
CONFIG_REG = "1M\u00d764 regression tree (MSE split criterion) on 8\u00d7MI355X"
CONFIG_10M = "10M\u00d7128 synthetic, data-parallel histogram all-reduce, 288 GB HBM sizing, 8 GPUs"

# what actually ran, by the level loop's reported mode (config.name)
MODE_TEXT = {
    "single-gpu": "one MI355X, no collectives",
    "subtree-owned": "subtree ownership: replicated levels until >= 2-4 units per rank, LPT "
                     "assignment, each rank writes its subtrees into one node-shared host "
                     "tree (one RCCL all-gather of segment counts)",
    "replicated": "replicated levels (too few units to switch), one RCCL all-gather of "
                  "finisher subtrees",
    "feature": "feature-parallel split search, one RCCL all-gather of split records per level",
    "data": "data-parallel row shards, histograms reduced per feature block to owner ranks "
            "over RCCL per level",
    "replicated-exact": "exact thresholds, replicated on every rank (fewer features than ranks)",
}


def _spawn_ranks(a, argv) -> int:
    """``--gpus N`` outside a launcher: run N rank processes under
    ``torch.distributed.run`` as children (this process never touches the GPU:
    counting devices does not initialise it) and return their exit code."""
    import socket
    import subprocess

    import torch

    have = torch.cuda.device_count()
    if os.environ.get("MPITREE_BENCH_BACKEND", "nccl") == "nccl" and have < a.gpus:
        sys.stderr.write(f"bench.py: --gpus {a.gpus} needs {a.gpus} visible GPUs, found {have}\n")
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", "--samples", dest="n", type=int, default=1_000_000,
                    help="rows (--samples under torchrun, whose parser takes --n)")
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--classes", type=int, default=2)
    ap.add_argument("--max-depth", type=int, default=-1, help="-1 = unlimited (reference default)")
    ap.add_argument("--criterion", default="entropy")
    ap.add_argument("--strategy", default="auto")
    ap.add_argument("--regression", action="store_true")
    ap.add_argument("--continuous", action="store_true",
                    help="N(0,1) features: exact thresholds over every unique value")
    ap.add_argument("--no-continuous", action="store_true",
                    help="skip the continuous companion timing (continuous_ms_per_step)")
    ap.add_argument("--max-bins", type=int, default=0,
                    help="> 0: quantile bins (e.g. 1024 with --continuous: 16-bit codes)")
    ap.add_argument("--profile-levels", action="store_true")
    argv = sys.argv[1:] if argv is None else list(argv)
    a = ap.parse_args(argv)
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(_spawn_ranks(a, argv))
    if int(os.environ.get("WORLD_SIZE", "1")) != a.gpus:
        ap.error(f"--gpus {a.gpus} but the launcher started WORLD_SIZE="
                 f"{os.environ.get('WORLD_SIZE')} ranks")

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from mpitree_amd import DecisionTreeClassifier, DecisionTreeRegressor
    from mpitree_amd import ParallelDecisionTreeClassifier, ParallelDecisionTreeRegressor
    from mpitree_amd.utils.datasets import make_classification, make_regression

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    backend = os.environ.get("MPITREE_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend != "nccl":  # rehearsal: ranks may share a GPU
        local %= max(1, torch.cuda.device_count())
        os.environ["LOCAL_RANK"] = str(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    md = None if a.max_depth < 0 else a.max_depth
    levels = None if a.continuous else 256
    if a.regression:
        X, y = make_regression(a.n, a.features, levels=levels, seed=0, device=dev)
        crit = "squared_error"
    else:
        X, y = make_classification(a.n, a.features, n_classes=a.classes, levels=levels, seed=0,
                                   device=dev)
        crit = a.criterion
    mb = {"max_bins": a.max_bins} if a.max_bins > 0 else {}
    if world > 1:
        import torch.distributed as dist

        from mpitree_amd.parallel.process_group import init_distributed

        init_distributed(backend=backend)
        cls = ParallelDecisionTreeRegressor if a.regression else ParallelDecisionTreeClassifier
        est = cls(max_depth=md, criterion=crit, device="cuda", strategy=a.strategy, **mb)
    else:
        dist = None
        cls = DecisionTreeRegressor if a.regression else DecisionTreeClassifier
        est = cls(max_depth=md, criterion=crit, device="cuda", **mb)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        est.fit(X, y)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        est.fit(X, y)
    barrier()
    dt = (time.perf_counter() - t0) / a.steps

    def reduce_max(v):
        if dist is None:
            return v
        t = torch.tensor([v], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    dt = reduce_max(dt)
    stats = est.fit_stats_
    ta = est.tree_arrays_
    cont = None
    if not a.continuous and not a.no_continuous and a.max_bins <= 0:
        # the same estimator and shape on continuous features (exact presorted-list
        # engine, the reference's threshold semantics), timed the same way
        gen = make_regression if a.regression else make_classification
        kw = {} if a.regression else {"n_classes": a.classes}
        Xc, yc = gen(a.n, a.features, levels=None, seed=1, device=dev, **kw)
        ksteps = max(1, min(a.steps, 10))
        est.fit(Xc, yc)  # warmup (setup buffers, level-loop workspace)
        barrier()
        t0 = time.perf_counter()
        for _ in range(ksteps):
            est.fit(Xc, yc)
        barrier()
        cont = {"ms_per_step": round(reduce_max((time.perf_counter() - t0) / ksteps) * 1e3, 3),
                "steps": ksteps, "tree_nodes": est.fit_stats_.get("node_count"),
                "engine": est.fit_stats_.get("engine"),
                "thresholds": est.fit_stats_.get("thresholds")}
        del Xc, yc
    # the fit returned finished columns (numpy arrays over host memory, no
    # lazily derived attributes): check it, outside the timed region
    cols = ("feature", "threshold", "threshold_bin", "left", "right", "depth", "n_samples",
            "impurity", "value" if a.regression else "count")
    materialized = all(isinstance(ta.__dict__.get(c), np.ndarray) for c in cols)
    mode = stats.get("mode", "single-gpu")
    if world > 1:
        parallelism = {"feature": f"fp{world}", "data": f"dp{world}",
                       "replicated": f"subtree{world}",
                       "subtree-owned": f"subtree{world}"}.get(mode, f"{a.strategy}{world}")
    else:
        parallelism = "single"
    if a.regression:
        baseline_cfg = CONFIG_REG
    elif a.n >= 10_000_000 and a.features >= 128:
        baseline_cfg = CONFIG_10M
    else:
        baseline_cfg = CONFIG
    shape = f"{a.n:,}\u00d7{a.features} synthetic" + (" regression" if a.regression else "")
    # what the process group saw: backend, ranks and their GPUs (all-gathered), so
    # a multi-GPU record proves N RCCL ranks on N distinct GPUs
    from mpitree_amd.parallel.process_group import rank_topology

    topo = rank_topology()
    mode_text = MODE_TEXT.get(mode, mode)
    if world > 1 and topo["dist_backend"] != "nccl":
        # rehearsal: collectives over gloo, ranks sharing the visible GPUs
        mode_text = mode_text.replace("RCCL", topo["dist_backend"])
        hw = (f"{world} {topo['dist_backend']} ranks sharing {topo['distinct_gpus']} "
              f"MI355X (rehearsal, not a multi-GPU run)")
    else:
        hw = f"{world}\u00d7MI355X"
    cfg_name = f"{shape}, {mode_text}, {hw}"
    if rank == 0:
        value = a.n / dt
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt * 1e3, 3),
            "continuous_ms_per_step": None if cont is None else cont["ms_per_step"],
            "fit_seconds": round(dt, 6),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "dtype_detail": "fp32 features (exact data-value thresholds), int32 histogram "
                            "counts, fp64 split criterion",
            "data": "synthetic (generated on device: "
                    + ("continuous N(0,1) features, every value a candidate threshold"
                       if a.continuous else "256-level quantized features")
                    + ", labels from a random linear + interaction score with Gaussian noise)",
            "materialized": materialized,
            "dist_backend": topo["dist_backend"],
            "world_size_seen": topo["world_size_seen"],
            "distinct_gpus": topo["distinct_gpus"],
            "rank_devices": [{"rank": r["rank"], "host": r["host"], "device": r["device"],
                              "pci": r["pci"]} for r in topo["ranks"]],
            "config": {
                "name": cfg_name,
                "baseline_config": baseline_cfg,
                "model": f"DecisionTree{'Regressor' if a.regression else 'Classifier'}"
                         f"(criterion={crit}, max_depth={md})",
                "n_samples": a.n,
                "n_features": a.features,
                "n_classes": None if a.regression else a.classes,
                "global_batch": a.n,
                "seq_len": a.features,
                "parallelism": parallelism,
                "strategy": a.strategy,
                "engine": stats.get("engine"),
                "level_loop": mode,
                "feature_block": stats.get("feature_block"),
                "comm_bytes": int(sum(stats.get("comm_bytes_per_level", [])))
                + int(stats.get("comm_bytes_exchange", 0)),
                "tree_nodes": stats.get("node_count"),
                "tree_depth": stats.get("max_depth"),
                "thresholds": (f"quantile ({a.max_bins} bins)" if a.max_bins > 0 else
                               stats.get("thresholds", "exact (<= 256 values per feature)")),
                "comm_bytes_per_level": stats.get("comm_bytes_per_level"),
                "peak_device_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 3),
            },
            "continuous": cont,
            "reference_note": "reference is infeasible at this size (BASELINE.md: >=775 CPU-h "
                              "for the root node alone); vs_baseline is null",
        }
        if a.profile_levels:
            out["timings"] = {k: round(v * 1e3, 3) for k, v in stats.get("timings", {}).items()}
            out["levels"] = stats.get("levels")
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
