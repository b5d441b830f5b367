"""``Node``/``BranchType`` under the reference module path used in pickles."""

from mpitree_amd.models.node import BranchType, Node

__all__ = ["BranchType", "Node"]
