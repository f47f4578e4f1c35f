import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "oracle", ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle1000():
    from pyoracle import Oracle
    return Oracle(1000)


@pytest.fixture(scope="session")
def oracle1200():
    from pyoracle import Oracle
    return Oracle(1200)


@pytest.fixture(scope="session")
def product():
    """librazor_fec.so (built in-tree if stale)."""
    from razor_amd import build
    build.build()
    from razor_amd.fec import native
    return native(1000)


@pytest.fixture(scope="session")
def product1200():
    from razor_amd import build
    build.build()
    from razor_amd.fec import native
    return native(1200)
