"""Host profile (cProfile) of a collective fit on rank 0: ``bench.py``'s multi-rank
path -- the estimator's collective-fit wrapper, the communicator, the shared-tree
assembly -- under a launcher (ranks may share one GPU with the gloo backend).

    MPITREE_BENCH_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29650 bench/rank_host_prof.py [--fits 20]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fits", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/rank_host_prof.txt")
    a = ap.parse_args()
    import torch.distributed as dist

    from mpitree_amd import ParallelDecisionTreeClassifier
    from mpitree_amd.parallel.process_group import init_distributed
    from mpitree_amd.utils.datasets import make_classification

    backend = os.environ.get("MPITREE_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    X, y = make_classification(1_000_000, 64, n_classes=2, seed=0, device=dev)
    init_distributed(backend=backend)
    est = ParallelDecisionTreeClassifier(device="cuda")
    for _ in range(3):
        est.fit(X, y)
    dist.barrier()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.fits):
        est.fit(X, y)
    pr.disable()
    ms = (time.perf_counter() - t0) / a.fits * 1e3
    if dist.get_rank() == 0:
        with open(a.out, "w") as f:
            f.write(f"{ms:.3f} ms per fit (rank 0, {dist.get_world_size()} ranks, {backend})\n")
            for key in ("tottime", "cumulative"):
                sio = io.StringIO()
                pstats.Stats(pr, stream=sio).sort_stats(key).print_stats(40)
                f.write(f"==== by {key}\n{sio.getvalue()}\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
