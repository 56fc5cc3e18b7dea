import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG_ROOT = os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd")
for p in (ROOT, PKG_ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP path")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a ROCm GPU (deselect with -m 'not gpu')")
    return torch.device("cuda:0")
