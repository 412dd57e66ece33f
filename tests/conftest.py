import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmcgpu on the GPU)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def built():
    """Build (idempotent) the oracle library and the product libraries."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True)
    return ROOT
