import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP library calls)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def hip():
    """The HIP C-ABI library, on a GPU box.  Fails loudly if it is missing."""
    import torch
    from confild_amd import _lib
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _lib.lib()
