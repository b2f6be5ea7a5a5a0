import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cloudtik_amd import ops
    ops.require_native()  # GPU tests must exercise the HIP path, never a silent fallback
    return torch.device("cuda", 0)
