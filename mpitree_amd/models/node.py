"""Linked tree-node view of a fitted tree (pickle-compatible with the reference).

The reference's public tree IR is a linked ``Node`` dataclass plus a
``BranchType`` glyph enum (reference: ``mpitree/tree/_base.py:16-101``).
Training here never builds ``Node`` objects: the builders emit flat arrays
(:class:`mpitree_amd.models.tree_arrays.TreeArrays`) and ``Node`` graphs are
materialised on demand for ``tree_``, ``export_text`` and pickling. Field
names, defaults, ``__lt__`` ordering side effects and the module path used in
pickles (``mpitree.tree._base``) match the reference so checkpoints move both
ways.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Optional

__all__ = ["BranchType", "Node"]


class BranchType(Enum):
    """Glyph drawn in front of a node by ``export_text``."""

    ROOT = "┌──"
    INTERIOR_LIKE = "├──"
    LEAF_LIKE = "└──"


@dataclass(kw_only=True)
class Node:
    """One node of a fitted tree.

    ``value`` is the split feature index for interior nodes and the class
    label (classifier) or mean target (regressor) for leaves. ``threshold``
    is the largest feature value routed left (``x <= threshold``), ``None``
    for leaves. ``count`` holds per-class sample counts (classifier) or the
    sample count (regressor).
    """

    value: Any
    threshold: Optional[float] = None
    depth: int = field(default_factory=int)
    count: Any = field(default_factory=list)
    parent: Optional["Node"] = field(default=None, repr=False)
    left: Optional["Node"] = field(default=None, repr=False)
    right: Optional["Node"] = field(default=None, repr=False)
    _btype: BranchType = field(default=BranchType.ROOT, repr=False)

    def __post_init__(self):
        if self.parent is not None:
            self.depth = self.parent.depth + 1

    def __lt__(self, other: "Node") -> bool:
        # ``sorted([left, right])`` evaluates ``right < left``. An interior
        # right child sorts first and is drawn "├──"; otherwise the left child
        # keeps first place. Both operands get their glyph assigned here, as in
        # the reference renderer contract (_base.py:63-75).
        if self.is_leaf:
            other._btype = BranchType.INTERIOR_LIKE
            self._btype = BranchType.LEAF_LIKE
            return False
        self._btype = BranchType.INTERIOR_LIKE
        other._btype = BranchType.LEAF_LIKE
        return True

    @property
    def is_leaf(self) -> bool:
        return self.left is None and self.right is None

    @property
    def children(self) -> list:
        return [] if self.is_leaf else [self.left, self.right]


# Pickles name the reference module paths so reference and mpitree_amd
# checkpoints are interchangeable (the ``mpitree`` package re-exports these).
BranchType.__module__ = "mpitree.tree._base"
Node.__module__ = "mpitree.tree._base"
