"""Tree-identity diagnostic for the bench workload.

Fits the bench's synthetic data (``--n`` x ``--features``) on the GPU and
saves the tree columns to ``gpurun_out/diag_w{world}_r{rank}_i{k}.npz``; with
``--cpu`` also the native CPU builder's tree. Run once plainly and once
under torchrun (``MPITREE_BENCH_BACKEND=gloo`` shares one GPU) and compare
the files with ``--compare``.
"""

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FIELDS = ("feature", "threshold_bin", "left", "right", "n_samples", "depth")


def cols(ta):
    out = {k: np.asarray(getattr(ta, k)) for k in FIELDS}
    out["count"] = np.asarray(ta.count)
    return out


def compare(a, b):
    A, B = dict(np.load(a)), dict(np.load(b))
    na, nb = len(A["feature"]), len(B["feature"])
    print(f"{a}: {na} nodes, {b}: {nb} nodes")
    m = min(na, nb)
    for k in A:
        d = np.nonzero((A[k][:m] != B[k][:m]).reshape(m, -1).any(1))[0]
        if len(d):
            i = d[0]
            print(f"  first diff in {k} at node {i} ({len(d)} differing)")
            for kk in FIELDS:
                print(f"    {kk}: {A[kk][i]} vs {B[kk][i]}")
            print(f"    count: {A['count'][i]} vs {B['count'][i]}")
            return
    print("  identical" if na == nb else "  prefix identical")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        compare(*a.compare)
        return
    import torch

    from mpitree_amd import DecisionTreeClassifier, ParallelDecisionTreeClassifier
    from mpitree_amd.utils.datasets import make_classification

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    backend = os.environ.get("MPITREE_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    os.environ["LOCAL_RANK"] = str(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    X, y = make_classification(a.n, a.features, seed=0, device=dev)
    os.makedirs("gpurun_out", exist_ok=True)
    if world > 1:
        from mpitree_amd.parallel.process_group import init_distributed

        init_distributed(backend=backend)
        est = ParallelDecisionTreeClassifier(device="cuda")
    else:
        est = DecisionTreeClassifier(device="cuda")
    for it in range(a.repeat):
        est.fit(X, y)
        np.savez(f"gpurun_out/diag_w{world}_r{rank}_i{it}.npz", **cols(est.tree_arrays_))
        print(rank, it, est.tree_arrays_.node_count, est.fit_stats_.get("engine"), flush=True)
    if a.cpu and rank == 0:
        ref = DecisionTreeClassifier(device="cpu").fit(X.cpu().numpy(), y.cpu().numpy())
        np.savez("gpurun_out/diag_cpu.npz", **cols(ref.tree_arrays_))
        print("cpu", ref.tree_arrays_.node_count, flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
