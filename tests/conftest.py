import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
os.environ.setdefault('TZ', 'UTC')
# the library honours its KW_TEST_* capacity overrides only with this gate (csrc/kwenv.hpp); the tests that
# use them set them per test, so the gate alone changes nothing
os.environ['KW_TEST_HOOKS'] = '1'
try:
    import time
    time.tzset()
except AttributeError:  # pragma: no cover
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libkwmatch.so")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope='session')
def golden():
    from tests import golden_data
    return golden_data
