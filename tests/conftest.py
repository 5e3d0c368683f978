import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (test infrastructure only)."""
    from tests import oracle_ctypes
    return oracle_ctypes.load()


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """torch ships its own HIP runtime next to the library's (/opt/rocm): on the GPU box torch's
    is brought up first in a GPU session, before any test's context, so a test that moves data
    with torch never meets a device the other runtime already configured (a run of the TCP / KAT
    files followed by a torch-using test saw 'No HIP GPUs are available' otherwise)"""
    if request.config.getoption("-m", default="") == "gpu":
        import torch
        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    yield
