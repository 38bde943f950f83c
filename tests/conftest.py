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


# Test files whose GPU work runs only in child processes (IPC rank worlds, bench.py, the JNI driver,
# the C++ drivers). They run first, while the pytest process itself holds no GPU context: the full
# suite once took 96 s (and once > 180 s) for an 8-process IPC world that takes 4-5 s when run with
# its file alone (profiles/r05/README.md); the likely cause is the parent's own context, a ninth
# process on the card. With this order the full suite has run without such a stall (pass r05u).
CHILD_PROCESS_FILES = ("test_gpu_ipc.py", "test_gpu_bench.py", "test_gpu_jni.py", "test_gpu_cpp.py")


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=lambda it: 0 if os.path.basename(str(it.fspath)) in CHILD_PROCESS_FILES else 1)


@pytest.fixture(scope="session")
def O():
    import oracle  # noqa: WPS433 (test-only import of the checker)

    oracle.lib()
    return oracle
