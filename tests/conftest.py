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
# the C++ drivers, the RCCL stand-in drivers). Their worlds never share the card with a pytest process
# that holds a GPU context (DESIGN.md §6 "The P = 8 one-GPU stalls": round 5's two slow 8-process
# worlds both ran after the in-process suite had given the pytest process one; none has since): such a
# test is run in a fresh pytest process whenever this one has opened the GPU (pytest_pyfunc_call
# below), whatever the order the tests were collected in. They are also sorted first, so that in a
# whole-suite run this process has not opened the GPU yet and no test needs the re-run.
CHILD_PROCESS_FILES = ("test_gpu_ipc.py", "test_gpu_bench.py", "test_gpu_jni.py", "test_gpu_cpp.py",
                       "test_gpu_rccl_standin.py")


def pytest_collection_modifyitems(session, config, items):
    if not os.environ.get("MPJX_TEST_NO_SORT"):  # (MPJX_TEST_NO_SORT=1: collection order, to check the re-run)
        items.sort(key=lambda it: 0 if os.path.basename(str(it.fspath)) in CHILD_PROCESS_FILES else 1)


def holds_gpu_context():
    """This process has opened the GPU (the HIP / HSA runtime holds /dev/kfd or a /dev/dri node)."""
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                t = os.readlink(f"/proc/self/fd/{fd}")
            except OSError:
                continue
            if t == "/dev/kfd" or t.startswith("/dev/dri/"):
                return True
    except OSError:
        pass
    return False


@pytest.hookimpl(tryfirst=True)
def pytest_pyfunc_call(pyfuncitem):
    if (os.path.basename(str(pyfuncitem.fspath)) not in CHILD_PROCESS_FILES or os.environ.get("MPJX_TEST_FRESH_PARENT")
            or not holds_gpu_context()):
        return None
    import subprocess

    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-q", "-p", "no:cacheprovider", "--timeout", "150",
                        "--timeout-method", "thread", pyfuncitem.nodeid], cwd=ROOT, capture_output=True, text=True,
                       env=dict(os.environ, MPJX_TEST_FRESH_PARENT="1"), timeout=900)
    print(f"[run in a fresh pytest process: this one holds a GPU context]\n{r.stdout[-4000:]}")
    if os.environ.get("GRAFT_REPO_ROOT"):  # on the GPU box: a record of every re-run
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "fresh_parent_reruns.txt"), "a") as f:
            f.write(f"{pyfuncitem.nodeid} rc={r.returncode}\n")
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    return True


@pytest.fixture(scope="session")
def O():
    import oracle  # noqa: WPS433 (test-only import of the checker)

    oracle.lib()
    return oracle
