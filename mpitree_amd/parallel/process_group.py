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
    "rank_topology",
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


def _device_identity() -> dict:
    """This process's current GPU as the runtime sees it (None fields on CPU)."""
    out = {"device": None, "pci": None, "uuid": None, "name": None}
    if not torch.cuda.is_available():
        return out
    d = torch.cuda.current_device()
    pr = torch.cuda.get_device_properties(d)
    out["device"] = int(d)
    out["pci"] = "%04x:%02x:%02x" % (int(getattr(pr, "pci_domain_id", 0)),
                                     int(getattr(pr, "pci_bus_id", 0)),
                                     int(getattr(pr, "pci_device_id", 0)))
    out["uuid"] = str(getattr(pr, "uuid", ""))
    out["name"] = str(getattr(pr, "gcnArchName", pr.name))
    return out


def rank_topology() -> dict:
    """What the process group actually saw, for records that must prove it
    (bench.py): the backend, the world size and every rank's host, current
    device index and PCI address, all-gathered (a collective: every rank calls
    it). ``distinct_gpus`` counts different (host, PCI address) pairs -- N ranks
    of an RCCL run on N distinct GPUs show N; ranks sharing a card (gloo
    rehearsals) show fewer."""
    import socket

    me = dict(_device_identity(), rank=world_rank(), host=socket.gethostname())
    if not (dist.is_available() and dist.is_initialized()):
        ranks = [me]
        backend = "none"
    else:
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, me)
        backend = str(dist.get_backend())
    ids = {(r["host"], r["pci"]) for r in ranks if r["pci"] is not None}
    return {"dist_backend": backend, "world_size_seen": len(ranks),
            "distinct_gpus": len(ids), "ranks": ranks}
