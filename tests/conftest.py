import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def hip_built():
    from pyspark_tf_gke_amd import _native

    _native.ensure_built()
    return _native.hip_lib()
