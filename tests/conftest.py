import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


@pytest.fixture(scope="session")
def cuda():
    """The GPU tests must run on a GPU: fail loudly instead of skipping, so a missing device or a
    missing libgsdr.so can never pass as green."""
    import torch

    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    import gsdr_amd  # noqa: F401  (raises if libgsdr.so is missing)

    return torch.device("cuda", 0)
