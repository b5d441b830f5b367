"""Multi-process harness: run a function on N ranks (gloo on CPU, or RCCL with one GPU
per rank), rendezvous on 127.0.0.1."""

import os
import socket
import tempfile

import numpy as np
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, outdir, backend="gloo"):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    kw = {}
    if backend == "nccl":  # one GPU per rank (RCCL over xGMI)
        torch.cuda.set_device(rank)
        kw["device_id"] = torch.device("cuda", rank)
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    try:
        out = fn(rank, world, *args)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **out)
    finally:
        if dist.is_initialized():  # (a failed collective fit may have torn it down)
            dist.destroy_process_group()


def run_ranks(fn, world, *args, start_method="fork", backend="gloo"):
    """Run ``fn(rank, world, *args) -> dict[str, array]`` on ``world`` ranks."""
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_entry, args=(world, port, fn, args, d, backend), nprocs=world,
                           join=True, start_method=start_method)
        return [dict(np.load(os.path.join(d, f"r{r}.npz"), allow_pickle=False))
                for r in range(world)]
