"""Write tests/fixtures/reference_exact.json: continuous problems (> 256 unique
values per feature) fitted by the reference source itself (single-rank mpi4py
stub, tests/reference_oracle.py) on the CPU of this container. The GPU box has
no reference checkout, so the GPU exact engine is compared against these
recorded outputs (tests/test_gpu_kernels.py::test_gpu_exact_engine_matches_reference_source).

    python tools/make_reference_exact_fixtures.py
"""

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.reference_oracle import load_reference  # noqa: E402


def main():
    ref = load_reference()
    if ref is None:
        raise SystemExit("reference checkout absent")
    out = []
    for seed, (n, F, md) in enumerate([(400, 2, 4), (520, 3, 5), (640, 2, 6), (300, 3, None),
                                       (700, 2, 3)]):
        rng = np.random.default_rng(500 + seed)
        X = np.round(rng.normal(size=(n, F)), 6)
        s = X[:, 0] + 0.6 * X[:, F - 1] ** 2 + rng.normal(scale=0.6, size=n)
        y = np.digitize(s, np.quantile(s, [0.35, 0.7]))
        est = ref.DecisionTreeClassifier(max_depth=md).fit(X, y)
        out.append(dict(X=X.tolist(), y=y.tolist(), max_depth=md,
                        text=est.export_text(precision=17),
                        predict=np.asarray(est.predict(X)).tolist()))
    path = os.path.join(os.path.dirname(__file__), "..", "tests", "fixtures",
                        "reference_exact.json")
    with open(path, "w") as fh:
        json.dump(out, fh)
    print(f"wrote {len(out)} problems to {os.path.normpath(path)}")


if __name__ == "__main__":
    main()
