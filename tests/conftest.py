import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
for p in (ROOT, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs on the GPU box)')


def pytest_collection_modifyitems(config, items):
    # On a host without a GPU, skip gpu tests when they are selected implicitly.
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)
