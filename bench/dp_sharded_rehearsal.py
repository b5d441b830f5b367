"""Row-sharded data-parallel fit of continuous data (BASELINE config 4 shape):
each rank generates only its own shard of an N(0,1) matrix on its GPU, the
ranks agree on quantile bins from mergeable per-rank summaries
(``parallel/agreement.py``), and grow one tree with per-level histogram
reductions to each feature block's owner. Prints one JSON line per rank
(rank 0 adds the cross-rank digest check):

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29517 bench/dp_sharded_rehearsal.py \\
        --rows 10000000 --features 128

On one GPU the ranks share the card over gloo (``MPITREE_BENCH_BACKEND=gloo``,
the default here): a rehearsal of the RCCL path's bytes and memory, not of
xGMI timing.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000, help="rows over all ranks")
    ap.add_argument("--features", type=int, default=128)
    ap.add_argument("--max-bins", type=int, default=256)
    ap.add_argument("--fits", type=int, default=2)
    a = ap.parse_args()
    backend = os.environ.get("MPITREE_BENCH_BACKEND", "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
        os.environ["LOCAL_RANK"] = str(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from mpitree_amd import ParallelDecisionTreeClassifier
    from mpitree_amd.parallel.process_group import init_distributed
    from mpitree_amd.utils.datasets import make_classification
    from mpitree_amd.utils.observability import tree_digest

    init_distributed(backend=backend)
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    n_loc = a.rows // world
    # one generator per rank: a shard of the same distribution, different rows
    X, y = make_classification(n_loc, a.features, levels=None, seed=100 + rank, device=dev)
    torch.cuda.reset_peak_memory_stats(dev)
    est = ParallelDecisionTreeClassifier(strategy="data", device="cuda", max_bins=a.max_bins)
    times = []
    for _ in range(a.fits):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        est.fit(X, y, data_sharded=True)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    st = est.fit_stats_
    ta = est.tree_arrays_
    dig = torch.tensor([tree_digest(ta)], dtype=torch.int64)
    digs = [torch.zeros_like(dig) for _ in range(world)]
    dist.all_gather(digs, dig)
    out = dict(rank=rank, world=world, backend=backend, n_total=n_loc * world,
               n_local=n_loc, features=a.features, max_bins=a.max_bins,
               engine=st.get("engine"), mode=st.get("mode"), dp_reduce=st.get("dp_reduce"),
               levels=st.get("levels"), finisher_subtrees=st.get("finisher_subtrees"),
               nodes=ta.node_count, fit_s=[round(t, 3) for t in times],
               comm_bytes_per_level=st.get("comm_bytes_per_level"),
               comm_bytes_exchange=st.get("comm_bytes_exchange"),
               peak_device_mem_gb=round(torch.cuda.max_memory_allocated(dev) / 1e9, 3),
               train_acc=round(float((torch.as_tensor(est.predict(X), device=dev) == y)
                                     .double().mean()), 4),
               digests_equal=bool(all(int(d) == int(digs[0]) for d in digs)))
    print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
