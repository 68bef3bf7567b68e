import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu():
        return
    skip = pytest.mark.skip(reason="no GPU on this host")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
