import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
ASSETS = os.path.join(ROOT, "assets")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def rt():
    return importlib.import_module("metal4-raytracing_amd")


@pytest.fixture(scope="session")
def orc():
    import oracle
    return oracle


@pytest.fixture(scope="session")
def assets():
    return ASSETS
