"""Reference-compatible import path for the MI355X-native framework.

``from mpitree.tree import DecisionTreeClassifier`` works exactly as with
the reference package, and pickles written by either framework name these
module paths. The implementation lives in :mod:`mpitree_amd`.
"""
