import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def golden():
    import workloads

    img = workloads.golden_image()
    off = workloads.read_points(os.path.join(workloads.GOLDEN, "kp_t16_n9_off.txt"))
    maxt = workloads.read_points(os.path.join(workloads.GOLDEN, "kp_t16_n9_maxt.txt"))
    return img, off, maxt
