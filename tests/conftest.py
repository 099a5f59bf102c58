import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libicw.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    O.load()
    return O


@pytest.fixture(scope="session")
def icw():
    from in_cwave_amd import lib as L
    L.load()
    return L
