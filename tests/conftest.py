import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device) and libsiamese_hip.so')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


@pytest.fixture(scope='session')
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU test selected but no HIP device is visible')
    from graphembedding_amd.build import build_hip
    build_hip()
    return torch.device('cuda:0')
