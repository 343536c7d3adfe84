import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the parity tests proper")
    config.addinivalue_line("markers", "slow: long CPU-side oracle runs")


@pytest.fixture(scope="session")
def ctx():
    from pcl_feature_extraction_amd import Context
    c = Context(0)
    yield c
    c.close()
