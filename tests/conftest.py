import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Load libpamg before any test module imports torch: libpamg then binds to /opt/rocm's HIP and
# RCCL instead of the copies bundled in the torch wheel (parallel_amg_amd/_lib.py,
# runtime_providers). Not built yet (fresh CPU checkout): the `built` fixture builds it.
if os.path.exists(os.path.join(ROOT, "parallel_amg_amd", "libpamg.so")):
    from parallel_amg_amd import _lib as _pamg_lib
    _pamg_lib.lib()


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
