import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def iris2():
    from sklearn.datasets import load_iris

    iris = load_iris()
    return iris.data[:, :2], iris.target, iris


GOLDEN_DEPTH3 = """┌── sepal length (cm)
│  ├── sepal width (cm) [> 5.50]
│  │  ├── sepal length (cm) [> 3.60]
│  │  │  ├── setosa [<= 5.80]
│  │  │  └── virginica [> 5.80]
│  │  └── sepal length (cm) [<= 3.60]
│  │     ├── versicolor [<= 6.20]
│  │     └── virginica [> 6.20]
│  └── sepal width (cm) [<= 5.50]
│     ├── sepal length (cm) [> 2.70]
│     │  ├── setosa [<= 5.30]
│     │  └── setosa [> 5.30]
│     └── sepal length (cm) [<= 2.70]
│        ├── setosa [<= 4.90]
│        └── versicolor [> 4.90]"""

GOLDEN_DEPTH5 = """┌── sepal length (cm)
│  ├── sepal width (cm) [> 5.5]
│  │  ├── sepal length (cm) [> 3.6]
│  │  │  ├── setosa [<= 5.8]
│  │  │  └── virginica [> 5.8]
│  │  └── sepal length (cm) [<= 3.6]
│  │     ├── sepal length (cm) [> 6.2]
│  │     │  ├── sepal length (cm) [<= 7.0]
│  │     │  │  ├── virginica [<= 6.9]
│  │     │  │  └── versicolor [> 6.9]
│  │     │  └── virginica [> 7.0]
│  │     └── sepal length (cm) [<= 6.2]
│  │        ├── sepal width (cm) [> 5.7]
│  │        │  ├── versicolor [<= 2.9]
│  │        │  └── versicolor [> 2.9]
│  │        └── sepal width (cm) [<= 5.7]
│  │           ├── versicolor [<= 2.8]
│  │           └── versicolor [> 2.8]
│  └── sepal width (cm) [<= 5.5]
│     ├── sepal length (cm) [> 2.7]
│     │  ├── sepal width (cm) [> 5.3]
│     │  │  ├── versicolor [<= 3.0]
│     │  │  └── setosa [> 3.0]
│     │  └── setosa [<= 5.3]
│     └── sepal length (cm) [<= 2.7]
│        ├── sepal length (cm) [<= 4.9]
│        │  ├── sepal width (cm) [> 4.5]
│        │  │  ├── versicolor [<= 2.4]
│        │  │  └── virginica [> 2.4]
│        │  └── setosa [<= 4.5]
│        └── versicolor [> 4.9]"""
