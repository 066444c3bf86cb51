import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "normalizing-flows-dpfs_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run on the GPU box")


def load_golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name)))


def group(fx, prefix):
    """Sub-dict of a golden fixture with ``prefix/`` stripped."""
    p = prefix + "/"
    return {k[len(p):]: v for k, v in fx.items() if k.startswith(p)}


@pytest.fixture(scope="session")
def golden():
    return load_golden
