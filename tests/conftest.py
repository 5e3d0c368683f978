import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")
    if getattr(config.option, "markexpr", "") == "gpu":
        # torch ships its own HIP runtime next to the library's (/opt/rocm). On the GPU boxes
        # torch's cannot open the device once the library's runtime has (a test module's
        # pv_device_count at collection is enough: 'No HIP GPUs are available'), while the other
        # order works. So torch's comes up first, before collection imports any test module.
        import torch
        try:
            if torch.cuda.device_count() > 0:
                torch.cuda.init()
        except RuntimeError as e:
            print(f"conftest: torch HIP runtime unavailable: {e}")


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (test infrastructure only)."""
    from tests import oracle_ctypes
    return oracle_ctypes.load()

