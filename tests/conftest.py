import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def gpu():
    """The product library on cuda:0; fails loudly (never skips to a CPU path) on a GPU box."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this container")
    import sketchml_amd
    return sketchml_amd
