import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="session")
def gpu():
    """GPU session: torch is imported first so the process has one HIP
    runtime (torch's), exactly as in bench.py."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import dccrg_amd

    dccrg_amd.lib()
    return torch
