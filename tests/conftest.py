import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

INPUTS = os.path.join(ROOT, 'tests', 'golden', 'inputs')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a HIP device (MI355X) and the built libpycatkin_amd.so')


@pytest.fixture(scope='session')
def inputs():
    return INPUTS
