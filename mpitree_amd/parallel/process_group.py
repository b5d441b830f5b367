"""Lazy ``torch.distributed`` bootstrap (RCCL over xGMI on MI355X, gloo on CPU).

The reference initialises MPI as a side effect of importing its estimator
module and captures ``COMM_WORLD``/rank/size as class attributes
(``mpitree/tree/decision_tree.py:313-317``). Here nothing happens at import:
the process group is created on the first collective ``fit`` (or explicitly
with :func:`init_distributed`), from the usual ``torchrun`` environment
(``RANK``, ``WORLD_SIZE``, ``LOCAL_RANK``, ``MASTER_ADDR``, ``MASTER_PORT``).
One process drives one GPU; the ``nccl`` backend name is RCCL on ROCm.
"""

from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

__all__ = [
    "init_distributed",
    "ensure_initialized",
    "world_group",
    "world_rank",
    "world_size",
    "local_rank",
    "comm_device",
]

DEFAULT_TIMEOUT = datetime.timedelta(seconds=int(os.environ.get("MPITREE_DIST_TIMEOUT", "600")))


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(backend: str | None = None, timeout=DEFAULT_TIMEOUT):
    """Initialise the default process group if needed; returns the world group."""
    if dist.is_available() and dist.is_initialized():
        return dist.group.WORLD
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local_rank())
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kwargs = {}
    if backend == "nccl":
        kwargs["device_id"] = torch.device("cuda", local_rank())
    dist.init_process_group(backend=backend, timeout=timeout, **kwargs)
    return dist.group.WORLD


def ensure_initialized(device: str = "auto"):
    """Create the process group on first use when launched with WORLD_SIZE > 1."""
    if dist.is_available() and dist.is_initialized():
        return dist.group.WORLD
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    use_gpu = device != "cpu" and torch.cuda.is_available()
    return init_distributed("nccl" if use_gpu else "gloo")


def world_group():
    return dist.group.WORLD if (dist.is_available() and dist.is_initialized()) else None


def world_rank() -> int:
    return dist.get_rank() if (dist.is_available() and dist.is_initialized()) else 0


def world_size() -> int:
    return dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1


def comm_device() -> torch.device:
    """Device that collective buffers must live on for the current backend."""
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")
