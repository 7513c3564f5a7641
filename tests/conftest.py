import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "ab: a kernel form only the A/B build carries (measured slower than the "
                                       "default; run with SKML_LIB=sketchml_amd/lib_ab/libskml.so)")


@pytest.fixture(autouse=True)
def _ab_forms(request):
    """Tests of A/B-only kernel forms run against the A/B build only; with the product library
    they are skipped (its skml_debug_form refuses those forms)."""
    if request.node.get_closest_marker("ab") is not None:
        from sketchml_amd import _lib
        if not _lib.AB_BUILD:
            pytest.skip("A/B-only kernel form: needs SKML_LIB=sketchml_amd/lib_ab/libskml.so")


@pytest.fixture(scope="session")
def gpu():
    """The product library on cuda:0; fails loudly (never skips to a CPU path) on a GPU box."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this container")
    import sketchml_amd
    return sketchml_amd
