import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

PKG = "intensity_based_lidar_slam_for_me-_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def pkg():
    m = importlib.import_module(PKG)
    if os.environ.get("LISLAM_ALT_LIB"):  # developer A/B: a variant build of the library
        m.native.load(os.environ["LISLAM_ALT_LIB"])
    return m


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # the CPU restatement: checker only

    O.lib()
    return O


@pytest.fixture(scope="session")
def synth(pkg):
    return pkg.synth
