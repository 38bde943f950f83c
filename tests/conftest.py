import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # test infrastructure: the CPU restatement
sys.path.insert(0, os.path.join(ROOT, "tools"))  # synth: the bench's synthetic input streams

# Every GPU test runs its IPC rank processes on ONE GPU. libmpjx refuses such worlds by default (a
# platform fault lets kernels of processes sharing a GPU read a stale 2 MiB page after free/re-use,
# DESIGN.md §6); the test workers never free device memory while their world exists, so they opt in.
# test_ipc_refuses_oversubscribed_gpu sets it back to 0 to check the refusal.
os.environ.setdefault("MPJX_IPC_OVERSUBSCRIBE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def O():
    import oracle  # noqa: WPS433 (test-only import of the checker)

    oracle.lib()
    return oracle
