"""Checkpoint format: cross-framework pickles and the restricted loader.

Reference format: pickling the estimator (globals
``mpitree.tree.decision_tree.*``, ``mpitree.tree._base.Node/BranchType`` and
numpy reconstruction; ``/root/reference/mpitree/tree/_base.py:16-57``).

* ``tests/fixtures/ref_iris2_depth{1,3}.pkl`` were written by the
  reference's own classes (its source run under ``tests/reference_oracle.py``'s
  mpi4py stub, Iris ``X[:, :2]``); the ``.txt`` next to each is the
  reference's ``export_text`` of that estimator. They load here through the
  restricted loader and render identically.
* The reverse direction runs the reference source in a child process and
  unpickles a tree fitted here.
* Malicious pickles (``numpy.savetxt``, ``numpy.load``, ``os.system``,
  ``builtins.getattr`` / ``eval``) are refused before anything runs.
"""

from __future__ import annotations

import os
import pickle
import subprocess
import sys

import numpy as np
import pytest

from mpitree_amd import DecisionTreeClassifier
from mpitree_amd.utils import checkpoint

from .reference_oracle import CHILD_PRELUDE, reference_available

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


@pytest.mark.parametrize("depth", [1, 3])
def test_reference_written_pickle_loads_and_renders(depth, iris2):
    X, y, iris = iris2
    blob = open(os.path.join(FIX, f"ref_iris2_depth{depth}.pkl"), "rb").read()
    if depth == 1:
        assert len(blob) == 759  # Iris max_depth=1 pickles to 759 B
    want = open(os.path.join(FIX, f"ref_iris2_depth{depth}.txt"), encoding="utf-8").read()
    clf = checkpoint.loads(blob)
    assert type(clf).__name__ == "DecisionTreeClassifier"
    names = dict(feature_names=iris.feature_names[:2], class_names=list(iris.target_names))
    assert clf.export_text(**names) == want
    # the same tree fitted here
    ours = DecisionTreeClassifier(max_depth=depth, device="cpu").fit(X, y)
    assert ours.export_text(**names) == want
    np.testing.assert_array_equal(clf.predict(X), ours.predict(X))
    np.testing.assert_array_equal(clf.predict_proba(X), ours.predict_proba(X))


@pytest.mark.skipif(not reference_available(), reason="reference checkout absent")
def test_our_pickle_loads_under_reference_classes(tmp_path, iris2):
    X, y, iris = iris2
    ours = DecisionTreeClassifier(max_depth=3, device="cpu").fit(X, y)
    p = tmp_path / "ours.pkl"
    ours.save(p)
    names = dict(feature_names=iris.feature_names[:2], class_names=list(iris.target_names))
    code = CHILD_PRELUDE + f"""
import pickle, numpy as np
from sklearn.datasets import load_iris
clf = pickle.load(open({str(p)!r}, "rb"))
assert type(clf).__module__ == "mpitree.tree.decision_tree", type(clf).__module__
iris = load_iris()
sys.stdout.write(clf.export_text(feature_names=iris.feature_names[:2],
                                 class_names=list(iris.target_names)))
sys.stdout.write("\\n@@" + ",".join(map(str, clf.predict(iris.data[:, :2]))))
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       env={**os.environ, "PYTHONPATH": ""}, timeout=120)
    assert r.returncode == 0, r.stderr
    text, pred = r.stdout.split("\n@@")
    assert text == ours.export_text(**names)
    np.testing.assert_array_equal(np.array(pred.split(","), dtype=np.int64), ours.predict(X))


class _Reduce:
    def __init__(self, fn, args):
        self.fn, self.args = fn, args

    def __reduce__(self):
        return (self.fn, self.args)


def _payloads(tmp_path):
    target = str(tmp_path / "pwned.txt")
    return target, [
        _Reduce(np.savetxt, (target, np.zeros(2))),
        _Reduce(np.load, (target,)),
        _Reduce(os.system, (f"touch {target}",)),
        _Reduce(eval, ("1+1",)),
        _Reduce(getattr, ("abc", "upper")),
        _Reduce(print, ("pwned",)),
    ]


def test_restricted_loader_refuses_code_execution(tmp_path):
    target, payloads = _payloads(tmp_path)
    for obj in payloads:
        for proto in (2, pickle.HIGHEST_PROTOCOL):
            blob = pickle.dumps(obj, protocol=proto)
            with pytest.raises(pickle.UnpicklingError):
                checkpoint.loads(blob)
    # nested inside an otherwise valid estimator state
    clf = DecisionTreeClassifier(max_depth=1, device="cpu").fit([[0.0], [1.0]], [0, 1])
    clf.fit_stats_["evil"] = payloads[0]
    with pytest.raises(pickle.UnpicklingError):
        checkpoint.loads(pickle.dumps(clf))
    assert not os.path.exists(target)


def test_restricted_loader_round_trips_every_protocol(iris2):
    X, y, _ = iris2
    clf = DecisionTreeClassifier(max_depth=4, device="cpu").fit(X, y)
    for proto in range(2, pickle.HIGHEST_PROTOCOL + 1):
        c2 = checkpoint.loads(pickle.dumps(clf, protocol=proto))
        assert c2.export_text() == clf.export_text()
        np.testing.assert_array_equal(c2.predict(X), clf.predict(X))
