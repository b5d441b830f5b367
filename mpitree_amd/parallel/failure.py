"""Failure containment for collective fits.

The reference has none: an exception inside one rank's subtree skips its
``allgather`` and ``Free`` and the other ranks block forever
(``mpitree/tree/decision_tree.py:446-477``). Here a rank that fails *inside*
a collective fit (a kernel error, a watchdog timeout, a host exception between
two collectives) must not leave its peers waiting in RCCL / gloo until the
process-group timeout. The protocol uses the c10d store (the rendezvous
key-value store every rank already holds) as an out-of-band channel:

1. The failing rank adds itself to the fit's failure counter
   (``mpitree/fit/<seq>/nfail``) and leaves its message under its rank.
2. Every rank runs a watchdog during a collective fit (one thread per process,
   re-armed per fit) that polls the counter (one store round trip per 0.2 s).
   A peer that sees a failure sets
   :data:`ABORT`; the host loops that wait on the device
   (``device_grower._wait_slot``, the level loops) raise
   :class:`CollectiveFitAborted` at their next check, so that peer fails too.
3. The failing rank waits up to ``MPITREE_FAIL_WAIT`` seconds (default 5) for
   every rank to fail. When they all do (an input error every rank raises at
   the same point, or peers that noticed :data:`ABORT`), nobody is inside a
   collective any more: the usual post-fit status all-gather runs and the
   process group stays usable.
4. Otherwise some peer is blocked inside a collective that will never
   complete: the failing rank aborts the process group. Its peers' gloo
   operations fail at once ("connection closed by peer"); an RCCL peer's
   watchdog aborts its own communicator after the same grace period, which
   releases its stream. Every rank then raises; the process group is gone
   (``ensure_initialized`` creates a new one on the next collective fit).

Fault injection for the tests: ``MPITREE_FAULT_RANK=k`` with
``MPITREE_FAULT_AT=level:L`` raises on rank k inside the level loops
(:func:`fault_point`).
"""

from __future__ import annotations

import os
import threading
import time

import torch.distributed as dist

from ..utils.observability import logger, maybe_inject_fault

__all__ = ["ABORT", "CollectiveFitAborted", "FitGuard", "check_abort", "fault_point"]

ABORT = threading.Event()  # set while a peer has failed the current collective fit
_SEQ = [0]  # collective fits started by this process (equal on every rank)


class CollectiveFitAborted(RuntimeError):
    """A peer rank failed the collective fit this rank was part of."""


def check_abort() -> None:
    """Raise :class:`CollectiveFitAborted` when a peer failed (cheap: an Event)."""
    if ABORT.is_set():
        raise CollectiveFitAborted("collective fit aborted: another rank failed")


def fault_point(comm, where: str) -> None:
    """Fault injection site inside a multi-rank loop (``MPITREE_FAULT_AT=where``)."""
    if getattr(comm, "world_size", 1) > 1:
        maybe_inject_fault(int(comm.rank), where)


def _store():
    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:  # pragma: no cover - no default group
        return None


class _Watcher:
    """The process's watchdog thread, started once and re-armed per collective
    fit: starting (and joining) a thread per fit cost ~0.34 ms of host time a
    fit, a sixth of a P = 8 flagship fit. It runs the armed guard's poll loop
    (``FitGuard._watch``) until that guard stops, then waits for the next."""

    def __init__(self):
        self.pid = os.getpid()
        self.lock = threading.Lock()
        self.armed = threading.Event()
        self.idle = threading.Event()
        self.idle.set()
        self.guard = None
        threading.Thread(target=self._run, name="mpitree-fit-watchdog", daemon=True).start()

    def _run(self):
        while True:
            self.armed.wait()
            with self.lock:
                self.armed.clear()
                g = self.guard
                if g is None:
                    continue
                self.idle.clear()
            try:
                g._watch()
            except Exception:  # pragma: no cover - (a watchdog never takes the process down)
                pass
            finally:
                self.idle.set()

    def arm(self, guard) -> bool:
        """Hand ``guard`` to the thread; False when the previous guard's loop is
        still busy after 10 s (a slow store call or a communicator abort): the
        caller then starts a fresh watcher rather than fit without one."""
        if not self.idle.wait(timeout=10):  # (the previous guard's loop has returned)
            return False
        with self.lock:
            self.guard = guard
            self.armed.set()
        return True

    def is_current(self, guard) -> bool:
        """Whether ``guard`` is still the armed guard (under the lock)."""
        with self.lock:
            return self.guard is guard

    def disarm(self, guard) -> None:
        """After ``guard._done`` is set: no further action on its behalf."""
        with self.lock:
            if self.guard is guard:
                self.guard = None
        self.idle.wait(timeout=10)


_WATCHER: list = [None]


def _watcher() -> _Watcher:
    w = _WATCHER[0]
    if w is None or w.pid != os.getpid():  # (first use, or a forked child)
        w = _WATCHER[0] = _Watcher()
    return w


def _arm_watcher(guard) -> _Watcher:
    """Arm the process's watcher for ``guard``; a watcher whose previous loop is
    stuck is abandoned (it can no longer act: its guard is not current) and a
    fresh thread takes the fit."""
    w = _watcher()
    if not w.arm(guard):
        logger.warning("fit watchdog busy with a previous fit: starting a fresh one")
        w = _WATCHER[0] = _Watcher()
        w.arm(guard)
    return w


class FitGuard:
    """Context of one collective fit on ``comm`` (see the module docstring)."""

    POLL_S = 0.2
    STORE_ERRORS = 5  # consecutive failed store polls read as a torn-down group

    def __init__(self, comm):
        self.comm = comm
        self.P = int(comm.world_size)
        self.rank = int(comm.rank)
        _SEQ[0] += 1
        self.pfx = f"mpitree/fit/{_SEQ[0]}"
        self.store = _store()
        self.wait_s = float(os.environ.get("MPITREE_FAIL_WAIT", "5"))
        self._done = threading.Event()
        self._thread = None
        self.aborted = False

    # ------------------------------------------------------------ store
    def _nfail(self) -> int:
        try:
            return int(self.store.add(self.pfx + "/nfail", 0))
        except Exception:  # the store went away with an aborted group
            return -1

    def _first_failure(self) -> str:
        for r in range(self.P):
            try:
                if self.store.check([f"{self.pfx}/msg/{r}"]):
                    return f"rank {r}: " + self.store.get(f"{self.pfx}/msg/{r}").decode()
            except Exception:
                break
        return "another rank failed"

    # --------------------------------------------------------- watchdog
    def _watch(self):
        seen = None
        errors = 0
        while not self._done.wait(self.POLL_S):
            n = self._nfail()
            if n == 0:
                errors = 0
                continue
            if n < 0:  # a store error: transient (retry), or the group is gone
                errors += 1
                if errors < self.STORE_ERRORS:
                    continue
            errors = 0
            if not self._live():  # (a previous fit's loop: never abort the next fit)
                return
            ABORT.set()  # host loops raise at their next check
            if seen is None:
                seen = time.monotonic()
            # still inside the fit well after the failing rank gave up waiting:
            # blocked on a device collective -- release it (RCCL communicator
            # abort; a gloo peer's socket closes on the failing rank's abort)
            if (time.monotonic() - seen > self.wait_s + 2.0 and dist.is_initialized()
                    and dist.get_backend() == "nccl"):
                logger.error("rank %d: aborting the RCCL communicator (peer failed)", self.rank)
                try:
                    dist.distributed_c10d._abort_process_group()
                except Exception:  # pragma: no cover
                    pass
                return

    def _live(self) -> bool:
        """This guard's fit is running and its watcher still serves it."""
        w = self._thread
        return not self._done.is_set() and w is not None and w.is_current(self)

    def __enter__(self):
        ABORT.clear()
        if self.store is not None and self.P > 1:
            self._thread = _arm_watcher(self)
        return self

    def stop(self) -> None:
        """End the watchdog's loop for this fit (idempotent)."""
        self._done.set()
        if self._thread is not None:
            self._thread.disarm(self)
            self._thread = None

    def __exit__(self, *exc):
        self.stop()
        ABORT.clear()
        return False

    def describe(self) -> str:
        """The first failing rank's message (for the peers' exceptions)."""
        return self._first_failure() if self.store is not None else "another rank failed"

    # ---------------------------------------------------------- failure
    def fail(self, error: BaseException) -> BaseException | None:
        """This rank failed inside the fit. Returns ``None`` when every rank
        failed (the caller runs the usual status all-gather: no rank is inside
        a collective), else the exception to raise after the process group was
        aborted."""
        if self.store is None:
            return error
        peer = isinstance(error, CollectiveFitAborted)
        try:
            if not peer:
                self.store.set(f"{self.pfx}/msg/{self.rank}", f"{type(error).__name__}: {error}")
            n = int(self.store.add(self.pfx + "/nfail", 1))
        except Exception:  # the group (and its store) is gone already
            n = -1
        t_end = time.monotonic() + self.wait_s
        while 0 <= n < self.P and time.monotonic() < t_end:
            if self._aborted_elsewhere():
                n = -1
                break
            time.sleep(0.01)
            n = self._nfail()
        if n == self.P:
            # every rank failed and agreed: nobody is inside a collective, and the
            # status all-gather that follows must not be aborted by the watchdog
            self.stop()
            ABORT.clear()
            return None
        msg = self._first_failure()
        try:
            self.store.set(self.pfx + "/aborted", "1")
        except Exception:
            pass
        self._abort_group()
        if peer or not isinstance(error, Exception):
            return CollectiveFitAborted(f"collective fit aborted ({msg}); the process group "
                                        "was torn down")
        return error

    def _aborted_elsewhere(self) -> bool:
        try:
            return bool(self.store.check([self.pfx + "/aborted"]))
        except Exception:
            return True

    def _abort_group(self):
        self.aborted = True
        logger.error("rank %d: collective fit failed; tearing down the process group", self.rank)
        if not dist.is_initialized():
            return
        try:
            if dist.get_backend() == "nccl":  # releases this rank's pending RCCL kernels
                dist.distributed_c10d._abort_process_group()
        except Exception:  # pragma: no cover - already torn down
            pass
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # pragma: no cover
            pass
