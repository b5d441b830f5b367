"""mpitree_amd: an MI355X-native parallel decision-tree trainer.

Public API (also importable as ``mpitree.tree``):

* :class:`DecisionTreeClassifier`, :class:`DecisionTreeRegressor`
* :class:`ParallelDecisionTreeClassifier`, :class:`ParallelDecisionTreeRegressor`
* :class:`Node`, :class:`BranchType` -- the linked tree view
* :class:`TreeArrays` -- the flat fitted-tree format

Importing has no side effects: no process group, no GPU initialisation.
"""

from .models.decision_tree import (
    DecisionTreeClassifier,
    DecisionTreeRegressor,
    ParallelDecisionTreeClassifier,
    ParallelDecisionTreeRegressor,
)
from .models.node import BranchType, Node
from .models.tree_arrays import TreeArrays

__version__ = "0.1.0"

__all__ = [
    "DecisionTreeClassifier",
    "DecisionTreeRegressor",
    "ParallelDecisionTreeClassifier",
    "ParallelDecisionTreeRegressor",
    "Node",
    "BranchType",
    "TreeArrays",
]
