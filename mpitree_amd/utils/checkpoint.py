"""Checkpoint helpers around the reference's pickle format.

The reference has no save/load API: pickling the estimator *is* the
checkpoint (``mpitree/tree/_base.py:16-57`` defines the pickled
``Node``/``BranchType``). ``save``/``load`` keep that format. ``load`` resolves
only an explicit allow-list of ``(module, name)`` globals: this package's
estimator / ``Node`` / ``BranchType`` classes (under the reference module
paths and the native ones), numpy's array and scalar reconstruction
(``_reconstruct``, ``_frombuffer``, ``ndarray``, ``dtype``, ``scalar``) and a
handful of inert builtin containers. Anything else -- ``numpy.savetxt``,
``os.system``, ``builtins.getattr``/``eval`` ... -- raises
``UnpicklingError`` before it is called.
"""

from __future__ import annotations

import io
import pickle

__all__ = ["save", "load", "dumps", "loads", "ALLOWED_GLOBALS"]

_ESTIMATORS = ("DecisionTreeClassifier", "ParallelDecisionTreeClassifier",
               "DecisionTreeRegressor", "ParallelDecisionTreeRegressor")
_NUMPY_CORE = ("numpy.core.multiarray", "numpy._core.multiarray")
_NUMPY_NUMERIC = ("numpy.core.numeric", "numpy._core.numeric")

ALLOWED_GLOBALS = frozenset(
    [(m, n) for m in ("mpitree.tree.decision_tree", "mpitree_amd.models.decision_tree")
     for n in _ESTIMATORS]
    + [(m, n) for m in ("mpitree.tree._base", "mpitree_amd.models.node")
       for n in ("Node", "BranchType")]
    + [(m, n) for m in _NUMPY_CORE for n in ("_reconstruct", "scalar")]
    + [(m, "_frombuffer") for m in _NUMPY_NUMERIC]
    + [("numpy", "ndarray"), ("numpy", "dtype")]
    # numpy >= 2 pickles dtypes of builtin scalar types via numpy.dtypes classes
    + [("numpy.dtypes", n) for n in ("Int64DType", "Int32DType", "Float64DType",
                                     "Float32DType", "BoolDType", "UInt8DType",
                                     "Int16DType", "UInt16DType", "UInt32DType",
                                     "UInt64DType", "Int8DType")]
    + [("builtins", n) for n in ("dict", "list", "tuple", "set", "frozenset", "float",
                                 "int", "str", "bool", "complex", "bytes", "bytearray")]
    + [("collections", "OrderedDict")]
    # protocol 2 spells bytes as _codecs.encode(str, "latin1") (a pure data transform)
    + [("_codecs", "encode")]
)


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) not in ALLOWED_GLOBALS:
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
