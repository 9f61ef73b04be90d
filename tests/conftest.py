import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP path); run with -m gpu")


@pytest.fixture(scope="session")
def sdk():
    """The product package (loaded from stable-diffusion-from-scratch_amd/ as ``sd_amd``)."""
    import sd_amd_loader
    return sd_amd_loader.load()
