import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpamg's HIP path)")


@pytest.fixture(scope="session")
def built():
    """Build libpamg.so and the oracle once per session (cheap when up to date)."""
    import __graft_entry__ as g
    g.build()
    return True


@pytest.fixture(scope="session")
def ctx(built):
    from parallel_amg_amd.partitioned import Context
    c = Context(0)
    yield c
