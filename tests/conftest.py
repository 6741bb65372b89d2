import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "disinfect-slam_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


_TORCH_HIP_READY = []


@pytest.fixture(autouse=True)
def _torch_hip_first(request):
    """GPU tests: torch ships its own HIP runtime (torch/lib/libamdhip64.so) beside the one the
    engine library links (/opt/rocm). Initialise torch's before the first GPU test creates an
    engine, so the tests that hand torch device tensors to the engine never depend on which of the
    two runtimes enumerated the device first."""
    if request.node.get_closest_marker("gpu") is not None and not _TORCH_HIP_READY:
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
        _TORCH_HIP_READY.append(True)
    yield
