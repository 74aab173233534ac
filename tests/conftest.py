import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and the built libhbx.so")
    config.addinivalue_line("markers", "slow: long-running CPU oracle test")


@pytest.fixture(scope="session")
def hbx_ctx():
    from hbbft_amd.hbx import Context

    ctx = Context(0)
    yield ctx
    ctx.close()
