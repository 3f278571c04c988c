import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
for p in (str(REPO), str(REPO / "tests"), str(REPO / "tests" / "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)
import _rgbd_import  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: CPU test that takes more than a few seconds")


GOLDEN = REPO / "tests" / "golden"


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
        return cache[name]
    return load
