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


@pytest.fixture(autouse=True)
def _default_digests(request):
    """Every GPU test starts with the default digests (SHA-256 threshold hashing, afck Merkle)."""
    if "hbx_ctx" in request.fixturenames:
        ctx = request.getfixturevalue("hbx_ctx")
        ctx.set_digest(0)
        ctx.set_merkle_digest(0)
        ctx.set_verify_lanes(0)
        ctx.set_combine_lanes(0)
    yield
