import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: full-size (1M-frame) parity runs")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import csum_oracle
    return csum_oracle.load()
