import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # test infrastructure: the CPU restatement
sys.path.insert(0, os.path.join(ROOT, "tools"))  # synth: the bench's synthetic input streams


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def O():
    import oracle  # noqa: WPS433 (test-only import of the checker)

    oracle.lib()
    return oracle
