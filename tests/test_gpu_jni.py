"""GPU: the JNI shim driven as a JVM drives it (VERDICT r4 "do this" #3), through the functional JNIEnv
stand-in (tests/jni/fakejvm.c) from a process that binds /opt/rocm's runtime (no torch), in one child
process (tests/jni_driver.py gpu):
  - one rank per JVM (RCCL world of one, calls through the exchange path; an IPC world of one;
    nativeDeviceCount — every native method of HipIntracomm.java is called): arrays pinned with
    GetPrimitiveArrayCritical and served as copies, so recv comes back only through mode 0 and send is
    released with JNI_ABORT; nonzero offsets; a 40 MiB call through the chunked host pipeline; Reduce /
    Scan / Reduce_scatter; direct buffers with the
    big-endian flags; a direct buffer too small; an invalid (op, type) pair -> mpi/MPIException;
  - long-lived rank threads: 8 calls each with new data through the thread's reused
    page-locked staging (host-direct and chunk-pipelined sizes), and the staging freed with the threads;
  - multicore (smpdev): 4 rank threads forming their worlds with nativeInitSmp; Allreduce / Reduce /
    Reduce_scatter (ragged) / Scan with rank-local offsets, MAXLOC on DOUBLE2 with a pair offset, direct
    big-endian buffers; an invalid pair on every rank; a too-short array on ONE rank, which raises the
    shim's message while the other ranks raise instead of hanging.
Every result bit for bit against the oracle (src/mpjdev/natmpjdev/lib/mpjdev_natmpjdev_Intracomm.c:410-627
is the reference entry point the shim replaces), no JNI rule broken, nothing written outside a window."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "jni", "libmpjx_jni_fake.so")


@pytest.mark.gpu
def test_jni_shim_on_gpu_through_fake_jvm():
    assert os.path.exists(SO), "tests/jni/libmpjx_jni_fake.so not built (make -C mpjexpress_amd tests)"
    env = dict(os.environ, MPJX_P1_EXCHANGE="1", MPJX_JNI_DRIVER_VERBOSE="1")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "jni_driver.py"), "gpu"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(d, indent=1))
    assert d["violations"] == [], d["violations"]
    bad = {k: v for k, v in d["cases"].items() if v != "ok"}
    assert not bad, bad
    assert len(d["cases"]) == 22, sorted(d["cases"])
