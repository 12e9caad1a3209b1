import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def ctx():
    from capsule_amd import packets

    c = packets.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def tctx():
    """A context of the test build (libcapsule_gpu_test.so: capi.hip with
    CGPU_TEST_HOOKS), for the tests that force rare paths through its
    environment hooks; the product library reads no environment."""
    from capsule_amd import packets

    c = packets.Context(0, test_hooks=True)
    yield c
    c.close()
