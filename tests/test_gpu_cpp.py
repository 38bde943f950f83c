"""GPU: the C++ host mirror (include/mpjx.hpp) running the reference's ccl known-answer tests
(test/mpi/ccl/*.java, ported in tests/cpp/ccl_tests.cpp) in multicore mode, device and host buffers."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_ccl_known_answer_tests():
    exe = os.path.join(ROOT, "tests", "cpp", "ccl_tests")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "mpjexpress_amd"), "tests"])
    r = subprocess.run([exe, "8"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "ALL CCL TESTS PASSED" in r.stdout


@pytest.mark.parametrize("P", [2, 4])
def test_cpp_ccl_known_answer_tests_ipc_processes(P):
    """The same KATs with P rank processes over the HIP-IPC direct engine (mpi::InitIPC)."""
    exe = os.path.join(ROOT, "tests", "cpp", "ccl_tests")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "mpjexpress_amd"), "tests"])
    r = subprocess.run([exe, "ipc", str(P)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MPJX_IPC_TIMEOUT_S="120"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "ALL CCL TESTS PASSED" in r.stdout
