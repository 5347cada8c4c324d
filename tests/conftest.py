import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# Reference data files. The mechanism library (test/lib/*) and the golden fixtures are
# copied under tests/golden/ (data only) so that nothing reads /root/reference at run time.
GOLDEN = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(GOLDEN, "lib")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libbrhip.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def pkg():
    import _pkgload
    return _pkgload.load()


@pytest.fixture(scope="session")
def orc():
    import oracle
    if not os.path.exists(oracle.LIB):
        oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
