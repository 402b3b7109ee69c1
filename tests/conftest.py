import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


_probe = {}


@pytest.fixture(autouse=True)
def _gpu_fault_probe(request):
    """After every GPU test: synchronize the device and run one copy-engine device-to-host
    copy (>= 64 KB: the runtime's staged SDMA path).  An asynchronous device error is then
    raised in the test that caused it -- the runtime reports some of them only at the next
    copy-engine transfer, i.e. in whichever test copies next."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch

    if not torch.cuda.is_available():
        return
    if "d" not in _probe:
        _probe["d"] = torch.zeros(1 << 17, dtype=torch.uint8, device="cuda")
        _probe["h"] = torch.empty(1 << 17, dtype=torch.uint8)
    torch.cuda.synchronize()
    _probe["h"].copy_(_probe["d"])
    torch.cuda.synchronize()


@pytest.fixture(scope="session")
def golden():
    import workloads

    img = workloads.golden_image()
    off = workloads.read_points(os.path.join(workloads.GOLDEN, "kp_t16_n9_off.txt"))
    maxt = workloads.read_points(os.path.join(workloads.GOLDEN, "kp_t16_n9_maxt.txt"))
    return img, off, maxt
