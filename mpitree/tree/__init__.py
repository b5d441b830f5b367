"""Estimators under the reference's public path (``mpitree.tree``)."""

from mpitree_amd.models.decision_tree import (
    DecisionTreeClassifier,
    DecisionTreeRegressor,
    ParallelDecisionTreeClassifier,
    ParallelDecisionTreeRegressor,
)

__all__ = [
    "DecisionTreeClassifier",
    "ParallelDecisionTreeClassifier",
    "DecisionTreeRegressor",
    "ParallelDecisionTreeRegressor",
]
