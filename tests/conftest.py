import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE sizes)")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build(ref=False)
    return oracle


@pytest.fixture(scope="session")
def engine():
    import netflow_amd as nf
    if not os.path.exists(nf.LIB_PATH):
        nf.build()
    e = nf.Engine(0)  # raises loudly if there is no gfx950 device or the HIP library is missing
    yield e
    e.close()
