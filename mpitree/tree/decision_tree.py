"""Estimator classes under the reference module path used in pickles."""

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
