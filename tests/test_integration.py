"""CPU: the Java-side integration files, checked as far as this JDK-less image allows.

- integration/jni/mpi_HipIntracomm.c compiles with -Wall -Werror against include/mpjx.h and the
  subset of jni.h it uses (tests/jni/jni.h), and links against libmpjx: every libmpjx call it makes
  exists with the declared signature (tests/test_jni_fake.py and tests/test_gpu_jni.py execute it).
- Every `native` method of integration/java/mpi/HipIntracomm.java has a C definition with the JNI
  name and the JNI argument types its Java signature maps to (static -> jclass, instance ->
  jobject; int -> jint, long -> jlong, byte[] -> jbyteArray, int[] -> jintArray, Object -> jobject),
  and the shim defines nothing the class does not declare: a mismatch would otherwise surface only
  as an UnsatisfiedLinkError at a maintainer's site.
- HipIntracomm overrides what NativeIntracomm overrides to keep sub-communicators on its strategy
  (Split, Create, clone; src/mpi/NativeIntracomm.java:160-215) plus the four reductions.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "integration", "java", "mpi", "HipIntracomm.java")
SHIM = os.path.join(ROOT, "integration", "jni", "mpi_HipIntracomm.c")
LIB = os.path.join(ROOT, "mpjexpress_amd", "lib")

JNI_TYPES = {"int": "jint", "long": "jlong", "byte[]": "jbyteArray", "int[]": "jintArray", "Object": "jobject",
             "void": "void"}


def _java_natives():
    src = open(JAVA).read()
    out = {}
    for m in re.finditer(r"private\s+(static\s+)?native\s+(\w+(?:\[\])?)\s+(\w+)\(([^)]*)\);", src, re.S):
        static, ret, name, params = m.group(1), m.group(2), m.group(3), m.group(4)
        types = [" ".join(p.split()[:-1]) for p in params.split(",") if p.strip()]
        out[name] = (bool(static), ret, types)
    return out


def _c_entries():
    src = open(SHIM).read()
    out = {}
    for m in re.finditer(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+Java_mpi_HipIntracomm_(\w+)\(([^)]*)\)", src, re.S):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        types = [" ".join(p.replace("*", " * ").split()[:-1]).replace(" *", "*") for p in params.split(",")]
        out[name] = (ret, types)
    return out


def test_jni_shim_compiles_and_links(tmp_path):
    so = os.path.join(LIB, "libmpjx.so")
    if not os.path.exists(so):
        pytest.skip("libmpjx.so not built")
    out = tmp_path / "libmpjx_jni.so"
    cmd = ["gcc", "-std=c11", "-O2", "-fPIC", "-shared", "-Wall", "-Wextra", "-Werror",
           "-I" + os.path.join(ROOT, "tests", "jni"), "-I" + os.path.join(ROOT, "include"), SHIM,
           "-L" + LIB, "-lmpjx", "-Wl,--no-undefined", "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    nm = subprocess.run(["nm", "-D", "--defined-only", str(out)], capture_output=True, text=True).stdout
    for name in _java_natives():
        assert f"Java_mpi_HipIntracomm_{name}" in nm, name


def test_java_natives_match_jni_definitions():
    java, c = _java_natives(), _c_entries()
    assert set(java) == set(c), (sorted(set(java) ^ set(c)))
    for name, (static, ret, types) in java.items():
        cret, ctypes_ = c[name]
        assert cret == JNI_TYPES[ret], (name, ret, cret)
        assert ctypes_[0] == "JNIEnv*", (name, ctypes_)
        assert ctypes_[1] == ("jclass" if static else "jobject"), (name, "static" if static else "instance", ctypes_[1])
        assert ctypes_[2:] == [JNI_TYPES[t] for t in types], (name, types, ctypes_[2:])


def test_hipintracomm_keeps_subcommunicators_on_the_gpu_strategy():
    src = open(JAVA).read()
    for sig in (r"public IntracommImpl Split\(int color, int key\)", r"public IntracommImpl Create\(Group group\)",
                r"public Object clone\(\)", r"public void Reduce\(", r"public void Allreduce\(",
                r"public void Reduce_scatter\(", r"public void Scan\(", r"public void Free\(\)"):
        assert re.search(sig, src), sig
    # Split/Create results are HipIntracomm, each with a libmpjx world of its own
    assert src.count("new HipIntracomm(") >= 2
    assert "nativeInitSmp(id, rank, size, devices)" in src


def test_route_decides_from_shared_arguments_only():
    """HipIntracomm.route() must not let rank-local offsets pick the GPU or the Java
    path, or ranks of one call could split and deadlock. Offsets may only reach the collective
    agreement (agreeNoOffsets, a pure-Java Allreduce every rank of a faithful GPU-eligible call makes)."""
    src = open(JAVA).read()
    body = src[src.index("private boolean route("):]
    body = body[:body.index("\n  }\n")]
    uses = re.findall(r"\b(soff|roff)\b", body.split(")", 1)[1])
    assert uses == ["soff", "roff"], uses  # exactly one use each: agreeNoOffsets(soff, roff)
    assert "agreeNoOffsets(soff, roff)" in body
    assert "super.Allreduce(mine, 0, any, 0, 1, MPI.INT, MPI.MAX)" in src
