import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs the HIP engine)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    here = os.path.join(ROOT, "tests", "golden")
    return {f[:-4]: np.load(os.path.join(here, f)) for f in os.listdir(here) if f.endswith(".npz")}
