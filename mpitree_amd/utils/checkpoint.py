"""Checkpoint helpers around the reference's pickle format.

The reference has no save/load API: pickling the estimator *is* the
checkpoint. ``save``/``load`` keep that format; ``load`` never
unpickles arbitrary globals -- only the estimator/Node classes of this package
(under either module path), numpy array reconstruction and builtins.
"""

from __future__ import annotations

import io
import pickle

__all__ = ["save", "load", "dumps", "loads"]

_ALLOWED_MODULES = {
    "mpitree.tree.decision_tree",
    "mpitree.tree._base",
    "mpitree_amd.models.decision_tree",
    "mpitree_amd.models.node",
    "numpy",
    "numpy.core.multiarray",
    "numpy._core.multiarray",
    "numpy.core.numeric",
    "numpy._core.numeric",
    "builtins",
    "collections",
}
_ALLOWED_BUILTINS = {"dict", "list", "tuple", "set", "frozenset", "float", "int", "str",
                     "bool", "complex", "bytes", "bytearray", "slice", "range", "getattr",
                     "OrderedDict"}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if module not in _ALLOWED_MODULES:
            raise pickle.UnpicklingError(f"refusing to load global {module}.{name}")
        if module in ("builtins", "collections") and name not in _ALLOWED_BUILTINS:
            raise pickle.UnpicklingError(f"refusing to load global {module}.{name}")
        if module.startswith("mpitree"):
            import mpitree.tree  # noqa: F401  (registers the alias modules)
        return super().find_class(module, name)


def dumps(est) -> bytes:
    return pickle.dumps(est, protocol=pickle.HIGHEST_PROTOCOL)


def loads(data: bytes):
    return _SafeUnpickler(io.BytesIO(data)).load()


def save(est, path) -> None:
    with open(path, "wb") as f:
        f.write(dumps(est))


def load(path):
    with open(path, "rb") as f:
        return loads(f.read())
