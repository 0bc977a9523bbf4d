import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def blocks():
    with open(os.path.join(GOLDEN, "reference_blocks.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def tiles():
    return dict(np.load(os.path.join(GOLDEN, "tiles.npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


def f64(bits_list):
    return np.array(bits_list, dtype=np.uint64).view(np.float64)
