import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def pytest_collection_modifyitems(config, items):
    """torch bundles its own HIP runtime next to the one libzdl.so links (/opt/rocm). When
    both live in one process, torch's must initialise the device first, or torch later
    finds no GPU. Tests that hand torch tensors to the engine therefore get torch's CUDA
    initialised before any test of the session loads libzdl."""
    if not any(it.get_closest_marker("gpu") for it in items):
        return
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
