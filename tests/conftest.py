import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "spartan-parallel_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def ctx():
    import spg

    c = spg.Context(0)
    yield c
    c.close()
