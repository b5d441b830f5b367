"""Load the reference implementation's *source* as an independent test oracle.

The reference (``/root/reference/mpitree/tree/{_base,decision_tree}.py``)
imports ``mpi4py`` in a class body and ``typing.override`` (Python 3.12).
Neither exists here, so :func:`load_reference` registers a single-rank
``mpi4py`` stub and a no-op ``typing.override`` shim, then executes the two
source files as the package ``_mpitree_ref.tree`` (a private name: our own
``mpitree`` alias package keeps its module path). Nothing is copied out of
the reference; the module objects are built from its files at test time.
Returns ``None`` when the reference checkout is absent (tests then skip).

``reference_pickle_env`` is the same loader run in a child process under
the reference's real module path ``mpitree.tree`` -- for producing and
consuming pickles that name the reference's globals.
"""

from __future__ import annotations

import importlib.util
import os
import sys
import types

REF_ROOT = os.environ.get("MPITREE_REFERENCE", "/root/reference")
_PKG = "_mpitree_ref"


def _stub_mpi4py():
    if "mpi4py" in sys.modules:
        return

    class _Comm:
        def Get_rank(self):
            return 0

        def Get_size(self):
            return 1

        def Split(self, color=0, key=0):
            return self

        def allgather(self, obj):
            return [obj]

        def Free(self):
            pass

    mpi = types.ModuleType("mpi4py.MPI")
    mpi.COMM_WORLD = _Comm()
    pkg = types.ModuleType("mpi4py")
    pkg.MPI = mpi
    sys.modules["mpi4py"] = pkg
    sys.modules["mpi4py.MPI"] = mpi


def _shim_override():
    import typing

    if not hasattr(typing, "override"):
        typing.override = lambda f: f


def reference_available() -> bool:
    return os.path.isfile(os.path.join(REF_ROOT, "mpitree", "tree", "decision_tree.py"))


def load_reference():
    """The reference's ``tree`` package (``DecisionTreeClassifier`` etc.), or None."""
    if not reference_available():
        return None
    key = f"{_PKG}.tree"
    if key in sys.modules:
        return sys.modules[key]
    _stub_mpi4py()
    _shim_override()
    tree_dir = os.path.join(REF_ROOT, "mpitree", "tree")
    top = types.ModuleType(_PKG)
    top.__path__ = []
    sys.modules[_PKG] = top
    pkg = types.ModuleType(key)
    pkg.__path__ = [tree_dir]
    sys.modules[key] = pkg
    for name in ("_base", "decision_tree"):
        spec = importlib.util.spec_from_file_location(f"{key}.{name}",
                                                      os.path.join(tree_dir, f"{name}.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = mod
        spec.loader.exec_module(mod)
        setattr(pkg, name, mod)
    pkg.DecisionTreeClassifier = pkg.decision_tree.DecisionTreeClassifier
    pkg.ParallelDecisionTreeClassifier = pkg.decision_tree.ParallelDecisionTreeClassifier
    pkg.Node = pkg._base.Node
    pkg.BranchType = pkg._base.BranchType
    return pkg


# A child process that imports the reference under its real module path
# (``mpitree.tree``), so pickles it writes / reads name the reference's globals.
CHILD_PRELUDE = f"""
import sys, types, typing
if not hasattr(typing, "override"):
    typing.override = lambda f: f
class _Comm:
    def Get_rank(self): return 0
    def Get_size(self): return 1
    def Split(self, color=0, key=0): return self
    def allgather(self, obj): return [obj]
    def Free(self): pass
_mpi = types.ModuleType("mpi4py.MPI"); _mpi.COMM_WORLD = _Comm()
_pkg = types.ModuleType("mpi4py"); _pkg.MPI = _mpi
sys.modules["mpi4py"] = _pkg; sys.modules["mpi4py.MPI"] = _mpi
sys.path.insert(0, {REF_ROOT!r})
import mpitree.tree
assert mpitree.tree.__file__.startswith({REF_ROOT!r}), mpitree.tree.__file__
"""
