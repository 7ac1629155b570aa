import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _clear_interrupt_flag():
    """The interrupt flag is process-global (reference model_management.py:851-877): a test that
    POSTs /interrupt must not leak it into node calls made directly by later tests."""
    from comfy_gen_server_amd.runtime import device as dm
    dm.interrupt_current_processing(False)
    yield
    dm.interrupt_current_processing(False)
