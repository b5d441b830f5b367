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
