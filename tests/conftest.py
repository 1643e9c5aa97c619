import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def dev():
    import torch
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _restore_threads():
    """CLI mains run in-process here; a tiny problem sets the intra-op pool to
    one thread for that (short-lived) tool process -- undo it per test."""
    import torch
    n = torch.get_num_threads()
    yield
    if torch.get_num_threads() != n:
        torch.set_num_threads(n)
