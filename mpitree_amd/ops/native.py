"""Loaders for the in-tree native extensions.

The GPU path never silently falls back to Python: if ``_hip`` cannot be
imported while a GPU fit is requested, :func:`hip` raises with the build
command to run.
"""

from __future__ import annotations

import importlib

_cache: dict = {}


def _load(name: str):
    if name not in _cache:
        try:
            _cache[name] = importlib.import_module(f"mpitree_amd.{name}")
        except ImportError as e:  # pragma: no cover - exercised when unbuilt
            _cache[name] = e
    mod = _cache[name]
    if isinstance(mod, Exception):
        raise ImportError(
            f"mpitree_amd native extension '{name}' is not built or failed to load ({mod}); "
            "run `python -m mpitree_amd.ops.build`"
        ) from mod
    return mod


def hip():
    """The gfx950 kernel module (raises if unavailable)."""
    return _load("_hip")


def cpu():
    """The native host builder module (raises if unavailable)."""
    return _load("_cpu")


def has_cpu() -> bool:
    try:
        cpu()
        return True
    except ImportError:
        return False


def has_hip() -> bool:
    try:
        hip()
        return True
    except ImportError:
        return False


def host_threads() -> int:
    """Host worker threads for native helpers: ``MPITREE_HOST_THREADS`` or the
    CPUs this process may run on, capped at 16 (one GPU's share of a node)."""
    import os

    env = os.environ.get("MPITREE_HOST_THREADS")
    if env:
        return max(1, int(env))
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):  # pragma: no cover - non-Linux
        n = os.cpu_count() or 1
    return max(1, min(16, n))
