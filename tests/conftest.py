import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: CPU test that takes more than a few seconds")


@pytest.fixture(scope="session")
def hip():
    """The loaded native library; skips CPU-only sessions, fails loudly on a GPU box."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from denseclip_vit_multimodal_amd import _native
    return _native.lib()
