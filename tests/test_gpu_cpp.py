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


def test_cpp_ccl_known_answer_tests_rccl_runtime():
    """The KATs through the RCCL engine's exchange path at world size 1, in a C++ process bound to
    /opt/rocm's HIP runtime and RCCL (what a JVM loading libmpjx binds; Python processes bind torch's
    bundled runtime)."""
    exe = os.path.join(ROOT, "tests", "cpp", "ccl_tests")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "mpjexpress_amd"), "tests"])
    r = subprocess.run([exe, "rccl"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MPJX_RCCL_TIMEOUT_S="120"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "ALL CCL TESTS PASSED" in r.stdout
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "/opt/rocm" in ldd and "torch" not in ldd, ldd


@pytest.mark.parametrize("sync", ["host", "device-shared"])
@pytest.mark.parametrize("P", [2, 4])
def test_cpp_ccl_known_answer_tests_ipc_processes(P, sync):
    """The same KATs with P rank processes over the HIP-IPC direct engine (mpi::InitIPC), with host
    or device (MPJX_IPC_SYNC=device-shared: device sync although the ranks share this GPU)
    synchronisation inside the calls."""
    exe = os.path.join(ROOT, "tests", "cpp", "ccl_tests")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "mpjexpress_amd"), "tests"])
    r = subprocess.run([exe, "ipc", str(P)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MPJX_IPC_TIMEOUT_S="120", MPJX_IPC_SYNC=sync))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "ALL CCL TESTS PASSED" in r.stdout


def test_ipc_preflight_tool_rank_processes():
    """tools/ipc_preflight — bench.py's child-process check of the HIP-IPC engine — passes with 3 rank
    processes on this GPU: push and pull Allreduce and a call over two staging windows, different
    data on every call, every element checked."""
    exe = os.path.join(ROOT, "tools", "ipc_preflight")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "mpjexpress_amd"), "tools"])
    uid = os.urandom(128).hex()
    env = dict(os.environ, MPJX_IPC_STAGE_MIB="4", MPJX_IPC_TIMEOUT_S="60")
    procs = [subprocess.Popen([exe, str(r), "3", "0", uid], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True, env=env) for r in range(3)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=120)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert all(p.returncode == 0 for p in procs), outs
    assert "ipc preflight ok: P=3" in outs[0]
    assert all("dsync ok" in o for o in outs), outs  # the device-synchronised second world


def test_cpp_jgf_reference_values_native_runtime():
    """The JGF SparseMatmult, MolDyn and RayTracer reference values through the C++ mirror in a native
    process bound to /opt/rocm's HIP runtime and RCCL (what a JVM loading libmpjx binds): host arrays,
    multicore ranks at P = 1, 2, 4, 8; P = 1 gives refval exactly, every P the oracle's order bit for bit,
    and the RayTracer's in-place Reduce(DOUBLE, SUM, 0) refval 2676692 at every P (tests/cpp/jgf_tests.cpp)."""
    exe = os.path.join(ROOT, "tests", "cpp", "jgf_tests")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "mpjexpress_amd"), "tests"])
    r = subprocess.run([exe, "1", "2", "4", "8"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ALL JGF TESTS PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
    assert r.stdout.count("RayTracer P=") == 4 and "checksum 2676692 refval 2676692" in r.stdout, r.stdout
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "/opt/rocm" in ldd and "torch" not in ldd, ldd
