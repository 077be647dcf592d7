import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a ROCm GPU (MI355X) and the built HIP extension')
    config.addinivalue_line('markers', 'slow: longer CPU tests')


@pytest.fixture(scope='session')
def gpu():
    import torch
    from medical_segmentation_pytorch_amd.ops import _ext
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    _ext.require()   # a GPU box without the extension is a FAILURE, not a skip
    return torch.device('cuda', 0)
