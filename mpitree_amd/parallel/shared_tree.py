"""Node-local shared-host tree assembly for subtree-ownership fits.

The reference hands every rank the whole tree by pickling subtrees and
``allgather``-ing them (``mpitree/tree/decision_tree.py:340-362,446-477``). The
GPU ownership fit (``ops/device_grower.py``) used to do the device analogue: one
all-gather of every finished node over xGMI (144 MB for the 2M-node 1M x 64
regression tree), then every rank compacted the full position space and copied
the whole tree to host memory over its own PCIe link (2.2 ms at ~55 GB/s) -- a
cost that does not shrink with P.

When every rank of the group runs on one node, the ranks instead share one host
buffer per fit (a ``/dev/shm`` mapping registered with the HIP runtime, so a
kernel can store into it over PCIe):

1. each rank ranks its own position space (replicated prefix + its own
   segments; ``assemble.hip`` asm_rank) and counts the nodes of each of its
   segments (``shm_seg_count``); one all-gather of those counts (a few KB, RCCL);
2. every rank sorts the segments and derives each of its nodes' final id =
   local rank + nodes of other ranks' segments before it (``shm_seg_prefix``);
3. each rank's emit kernel writes its own nodes (rank 0 also the prefix) straight
   into the shared buffer (zero-copy), so each rank moves 1 / P of the tree over
   PCIe and no node crosses xGMI;
4. a flag barrier in the buffer's header; every rank returns numpy views of the
   same finished tree.

Buffers are pooled: a slot is reused only when no rank still references a tree
in it (each rank's free-slot mask travels in the count all-gather, so every rank
makes the same choice). ``MPITREE_SHM_TREE=0`` (or ranks on different hosts)
keeps the all-gather exchange.
"""

from __future__ import annotations

import hashlib
import mmap
import os
import socket
import sys
import time

import numpy as np

from .failure import ABORT, check_abort

__all__ = ["ShmTreePool", "pool_for", "HEADER", "GATHER_HDR", "shm_free_bytes"]

HEADER = 4096  # per-rank flag words (64 B apart), then the packed tree columns
GATHER_HDR = 3  # gathered row: {depth, free-slot mask, /dev/shm free bytes}, counts
MAX_SLOTS = 8
SHM_MARGIN = 64 << 20  # /dev/shm left free when a new slot is created


def _margin() -> int:
    return int(float(os.environ.get("MPITREE_SHM_MARGIN_MB", SHM_MARGIN >> 20)) * (1 << 20))
POLL_TIMEOUT_S = float(os.environ.get("MPITREE_POLL_TIMEOUT", "120"))


def _host_key() -> int:
    """Same value on every process of one machine (hostname + boot id)."""
    boot = ""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        pass
    h = hashlib.sha1((socket.gethostname() + "|" + boot).encode()).digest()
    return int.from_bytes(h[:7], "little")


def shm_free_bytes() -> int:
    """Bytes a new /dev/shm mapping can still take (a container's /dev/shm is
    often a 64 MB tmpfs; touching a page past it is a SIGBUS, not an error)."""
    try:
        st = os.statvfs("/dev/shm")
    except OSError:
        return 0
    return int(st.f_bavail) * int(st.f_frsize)


class _Slot:
    """One shared buffer: a /dev/shm mapping, pinned and mapped for the device."""

    def __init__(self, hip, name: str, nbytes: int):
        import _posixshmem

        fd = _posixshmem.shm_open(name, os.O_CREAT | os.O_RDWR, 0o600)
        try:
            os.ftruncate(fd, nbytes)  # (every rank: the same size)
            self.mm = mmap.mmap(fd, nbytes)
        finally:
            os.close(fd)
        self.name, self.nbytes, self.hip = name, nbytes, hip
        self.nd = np.frombuffer(self.mm, dtype=np.uint8)
        self.host = int(self.nd.ctypes.data)
        self.dev = int(hip.host_register(self.host, nbytes))
        self.linked = True

    def flags(self) -> np.ndarray:
        return self.nd[:HEADER].view(np.int64)

    def free(self) -> bool:
        # references: self.nd and getrefcount's argument (tree views add theirs)
        return sys.getrefcount(self.nd) <= 2

    def unlink(self):
        if self.linked:
            import _posixshmem

            try:
                _posixshmem.shm_unlink(self.name)
            except OSError:
                pass
            self.linked = False

    def close(self):
        self.unlink()
        try:
            self.hip.host_unregister(self.host)
        except Exception:  # pragma: no cover - (teardown)
            pass
        self.nd = None
        try:
            self.mm.close()
        except BufferError:  # pragma: no cover - a view survived: leave it mapped
            pass


class ShmTreePool:
    """The shared tree buffers of one communicator (same decisions on every rank)."""

    def __init__(self, comm, hip, uid: int):
        self.hip, self.uid = hip, int(uid)
        self.rank, self.P = int(comm.rank), int(comm.world_size)
        self.slots: dict[int, _Slot] = {}
        self.gen = 0
        self.epoch = 0
        if self.P > 62:
            raise ValueError("shared-host assembly: at most 62 ranks")

    def free_mask(self) -> int:
        """Slots this rank may overwrite (bit i: slot i exists and is unreferenced)."""
        m = 0
        for i, sl in self.slots.items():
            if sl.free():
                m |= 1 << i
        return m

    def choose(self, masks, need: int, exclude: _Slot | None = None,
               shm_free=None) -> _Slot | None:
        """The slot every rank uses for ``need`` bytes of tree: the smallest slot
        free on every rank that holds it, else a new one (a free too-small slot is
        replaced). ``masks``: every rank's :meth:`free_mask` (from the all-gather);
        ``shm_free``: every rank's :func:`shm_free_bytes` from the same gather --
        None (on every rank alike) when a new slot would not fit beside
        ``SHM_MARGIN`` in the smallest of them."""
        both = ~0
        for m in masks:
            both &= int(m)
        for i, sl in self.slots.items():
            if sl is exclude:
                both &= ~(1 << i)
        best = None
        for i, sl in self.slots.items():
            if (both >> i) & 1 and sl.nbytes - HEADER >= need:
                if best is None or sl.nbytes < self.slots[best].nbytes:
                    best = i
        if best is not None:
            return self.slots[best]
        size = HEADER + max(1 << 20, int(need * 1.25) + 4095) // 4096 * 4096
        if shm_free is not None and size + _margin() > min(int(v) for v in shm_free):
            return None
        idx = next((i for i in range(MAX_SLOTS) if i not in self.slots), None)
        if idx is None:  # replace the largest slot free everywhere (none: grow the pool)
            cand = [i for i in self.slots if (both >> i) & 1]
            if not cand:
                idx = max(self.slots) + 1
            else:
                idx = max(cand, key=lambda i: self.slots[i].nbytes)
                self.slots.pop(idx).close()
        self.gen += 1
        name = f"/mpitree-{self.uid:x}-{idx}-{self.gen}"
        if idx >= 62:
            raise RuntimeError("shared-host assembly: more than 62 trees of this "
                               "communicator are alive at once")
        # (a new mapping is zero-filled: no rank clears the flags, which a peer
        # may already have set)
        return self.slots.setdefault(idx, _Slot(self.hip, name, size))

    def take_next(self) -> _Slot | None:
        """The slot agreed for this fit at the end of the previous one (None: the
        first fit), so the emit kernel is enqueued without a host round trip. It
        is still free on every rank: a slot free at the last fit's all-gather can
        only become busy by receiving a tree, and only this pool places trees."""
        sl, self.next = getattr(self, "next", None), None
        return sl

    def plan_next(self, masks, current: _Slot, need: int, shm_free=None) -> None:
        """Agree on the next fit's slot now (the same masks on every rank), sized
        for a tree like this one (a larger one is re-emitted after the wait; None:
        /dev/shm is short, the next fit chooses after its wait)."""
        self.next = self.choose(masks, need, exclude=current, shm_free=shm_free)

    def barrier(self, slot: _Slot) -> None:
        """Every rank has written its nodes into ``slot`` (flag words in its header;
        the caller synchronised its stream first)."""
        self.epoch += 1
        ep = self.epoch
        f = slot.flags()
        f[self.rank * 8] = ep
        t_end = time.perf_counter() + POLL_TIMEOUT_S
        k = 0
        idx = np.arange(self.P) * 8
        while True:
            if (f[idx] == ep).all():
                break
            k += 1
            if (k & 0x3FF) == 0:
                if ABORT.is_set():
                    check_abort()
                if time.perf_counter() > t_end:
                    raise RuntimeError("shared-host tree assembly: a rank never finished "
                                       "writing its nodes")
                time.sleep(0)
        if self.rank == 0:
            slot.unlink()  # every rank has it mapped: the name is no longer needed


_POOLS: dict = {}  # process group -> (pool or False, weakref of the group)


def _group_key(comm):
    """The process group a communicator runs on (estimators build a new
    communicator per fit; the pool -- its registered buffers and the agreed
    next slot -- belongs to the group, so consecutive fits reuse it)."""
    group = getattr(comm, "group", None)
    try:
        import torch.distributed as dist

        if group is None and dist.is_initialized():
            group = dist.distributed_c10d._get_default_group()
    except Exception:  # pragma: no cover - (no torch.distributed)
        pass
    return (id(group), int(comm.world_size), int(comm.rank)), group


def _alive(entry, group) -> bool:
    """The cached pool belongs to this very group object (not a destroyed group
    whose id a new one reuses)."""
    ref = entry[1]
    return ref is None or ref() is group


def _ref(group):
    import weakref

    try:
        return weakref.ref(group)
    except TypeError:  # (no weak references: the id alone)
        return None


def pool_for(comm, hip):
    """The pool of the communicator's process group, or None when its ranks span
    hosts (or ``MPITREE_SHM_TREE=0``). Collective on the group's first use (one
    small all-gather); later fits -- each with a new communicator -- reuse it."""
    pool = getattr(comm, "_shm_pool", None)
    if pool is not None:  # (a communicator that carries its own, e.g. simulations)
        return pool or None
    if getattr(comm, "world_size", 1) <= 1 or not hasattr(comm, "_all_gather"):
        return None
    if os.environ.get("MPITREE_SHM_TREE", "1") == "0":
        return None
    key, group = _group_key(comm)
    entry = _POOLS.get(key)
    if entry is not None and _alive(entry, group):
        return entry[0] or None
    uid = int.from_bytes(os.urandom(6), "little")
    g = comm._all_gather(np.array([_host_key(), uid], dtype=np.int64)).reshape(-1, 2)
    if not (g[:, 0] == g[0, 0]).all() or not os.path.isdir("/dev/shm"):
        pool = False
    else:
        pool = ShmTreePool(comm, hip, int(g[0, 1]))
    _POOLS[key] = (pool, _ref(group) if group is not None else None)
    return pool or None
