"""CPU: the C-ABI library loads, exports exactly what include/mpjx.h declares, and its host-side
logic (codes, worker table, argument validation) behaves without a GPU. No compute calls here."""
import ctypes
import os
import re
import subprocess

import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mpjx.h")


def header_functions():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^(?:int|const char \*)\s*\**(mpjx_[a-z_]+)\(", txt, re.M)))


def test_header_declares_the_path():
    fns = header_functions()
    for f in ("mpjx_combine", "mpjx_reduce", "mpjx_allreduce", "mpjx_reduce_scatter", "mpjx_scan",
              "mpjx_comm_init_rank", "mpjx_comm_init_smp", "mpjx_allreduce_host"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    from mpjexpress_amd import _lib

    L = _lib.lib()
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    for f in header_functions():
        assert f in exported, f
        assert hasattr(L, f)
    assert sorted(_lib.EXPORTS) == header_functions()  # the ctypes binding covers all of them


def test_library_is_gfx950_code_object():
    from mpjexpress_amd import _lib

    assert b"gfx950" in open(_lib.LIB_PATH, "rb").read()  # offload bundle for the MI355X target


def test_runtime_versions_report_the_bound_runtimes():
    """mpjx_runtime_versions: the HIP runtime / RCCL this process bound (bench.py records them), or
    MPJX_ERR_HIP without an answering HIP runtime; never a crash."""
    import ctypes

    from mpjexpress_amd import _lib

    L = _lib.lib()
    h, r = ctypes.c_int(0), ctypes.c_int(0)
    rc = L.mpjx_runtime_versions(ctypes.byref(h), ctypes.byref(r))
    assert rc in (0, -3), rc
    if rc == 0:
        assert h.value > 0 and r.value > 0
    assert L.mpjx_runtime_versions(None, None) in (0, -3)


def test_codes_and_sizes_match_reference():
    from mpjexpress_amd import _lib
    from mpjexpress_amd.mpi import MPI

    L = _lib.lib()
    assert L.mpjx_version() >= 100
    for t in range(1, 9):
        assert L.mpjx_type_size(t) == O.lib().ora_type_size(t)
    assert L.mpjx_type_size(9) == 0
    assert [MPI.MAX.opCode, MPI.MIN.opCode, MPI.SUM.opCode, MPI.PROD.opCode, MPI.LAND.opCode,
            MPI.BAND.opCode, MPI.LOR.opCode, MPI.BOR.opCode, MPI.LXOR.opCode, MPI.BXOR.opCode] == \
        list(range(1, 11))
    assert [MPI.BYTE.baseType, MPI.CHAR.baseType, MPI.SHORT.baseType, MPI.BOOLEAN.baseType,
            MPI.INT.baseType, MPI.LONG.baseType, MPI.FLOAT.baseType, MPI.DOUBLE.baseType] == \
        list(range(1, 9))


def test_worker_table_matches_oracle():
    from mpjexpress_amd import _lib

    L = _lib.lib()
    for op in range(1, 11):
        for t in range(1, 9):
            ok = L.mpjx_op_check(op, t) == 0
            assert ok == (O.check(op, t) == 0), (op, t)
    assert L.mpjx_op_check(3, 4) == -2
    assert b"MPI.SUM is invalid for MPI.BOOLEAN" in L.mpjx_last_error()
    assert L.mpjx_op_check(6, 8) == -2 and b"MPI.BAND is not valid for MPI.DOUBLE" in L.mpjx_last_error()


def test_argument_errors_without_gpu():
    from mpjexpress_amd import _lib

    L = _lib.lib()
    assert L.mpjx_combine(3, 8, None, None, 10, None) == -1  # NULL buffers
    assert L.mpjx_combine(3, 8, None, None, -1, None) == -1  # negative count
    assert L.mpjx_combine(3, 8, None, None, 0, None) == 0    # empty is a no-op
    assert L.mpjx_combine(3, 4, None, None, 1, None) == -2   # invalid (op, type) first
    assert L.mpjx_allreduce(None, None, None, 1, 8, 3, 0, None) == -1
    assert L.mpjx_strerror(-4) == b"RCCL error"


def test_no_device_is_loud():
    """On a machine without a GPU every device entry point fails with a status — never a silent
    CPU result (there is no CPU fallback in the product)."""
    from mpjexpress_amd import _lib

    L = _lib.lib()
    n = ctypes.c_int(-1)
    rc = L.mpjx_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("GPU present")
    comms = (ctypes.c_void_p * 2)()
    devs = (ctypes.c_int * 2)(0, 0)
    assert L.mpjx_comm_init_smp(comms, 2, devs) in (-5, -3)


def test_cpp_mirror_header_compiles_host_only(tmp_path):
    """include/mpjx.hpp is plain C++17 over the C ABI: it compiles and links with g++ alone."""
    src = tmp_path / "t.cpp"
    src.write_text('#include "mpjx.hpp"\nint main(){ std::vector<double> a(4), b(4);\n'
                   '  try { mpi::MPI::isOldSelected = false; (void)mpi::MPI::DOUBLE.Size(); }\n'
                   '  catch (const mpi::MPIException&) {} return 0; }\n')
    lib = os.path.join(ROOT, "mpjexpress_amd", "lib")
    subprocess.check_call(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                           str(tmp_path / "t"), f"-L{lib}", "-lmpjx", f"-Wl,-rpath,{lib}"])


def test_mpjbuf_section_header_parse():
    import numpy as np

    from mpjexpress_amd import _lib

    L = _lib.lib()
    vals = np.arange(5, dtype=">f8")  # big-endian doubles, as NIOBuffer writes them
    hdr = bytearray(8)  # 3 bytes of a previous section, padded to the 8-byte unit
    hdr += bytes([7, 0, 0, 0]) + (5).to_bytes(4, "big")
    buf = bytes(hdr) + vals.tobytes()
    b = ctypes.create_string_buffer(buf, len(buf))
    t, n, dp = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64()
    assert L.mpjx_mpjbuf_section(b, len(buf), 3, ctypes.byref(t), ctypes.byref(n), ctypes.byref(dp)) == 0
    assert (t.value, n.value, dp.value) == (8, 5, 16)  # DOUBLE, 5 elements, payload after header
    got = np.frombuffer(buf[dp.value:dp.value + 40], dtype=">f8")
    assert np.array_equal(got, vals)
    assert L.mpjx_mpjbuf_section(b, 20, 3, ctypes.byref(t), ctypes.byref(n), ctypes.byref(dp)) == -1  # overrun
    bad = bytearray(buf)
    bad[8] = 9  # BYTE_DYNAMIC: not a static primitive section
    bb = ctypes.create_string_buffer(bytes(bad), len(bad))
    assert L.mpjx_mpjbuf_section(bb, len(bad), 3, ctypes.byref(t), ctypes.byref(n), ctypes.byref(dp)) == -6


# (mpjbuf.Type code, capacity) of the one-section buffers of the reference's own buffer test, each
# holding 40 gathered elements: test/mpjdev/nbcomms/BufferTest3.java:61-97 ("(100*2)+section-
# overhead(8bytes)+NOPADDING"). A section image of exactly that capacity must parse to 40 elements
# with the payload right after the 8-byte header.
REF_BUFFER_TEST3 = [(0, 40 + 8, 1), (1, 80 + 8, 2), (4, 160 + 8, 4), (2, 80 + 8, 2), (3, 40 + 8, 1),
                    (5, 320 + 8, 8), (7, 320 + 8, 8), (6, 160 + 8, 4)]


def test_mpjbuf_section_capacities_of_reference_buffer_tests():
    from mpjexpress_amd import _lib

    L = _lib.lib()
    for code, cap, esz in REF_BUFFER_TEST3:
        img = bytes([code, 0, 0, 0]) + (40).to_bytes(4, "big") + bytes(40 * esz)
        assert len(img) == cap
        b = ctypes.create_string_buffer(img, len(img))
        t, n, dp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
        n = ctypes.c_int64()
        assert L.mpjx_mpjbuf_section(b, cap, 0, ctypes.byref(t), ctypes.byref(n), ctypes.byref(dp)) == 0
        assert (t.value, n.value, dp.value) == (code + 1, 40, 8)
        assert L.mpjx_type_size(t.value) == esz
        # one byte short of the reference's capacity: the payload would overrun
        assert L.mpjx_mpjbuf_section(b, cap - 1, 0, ctypes.byref(t), ctypes.byref(n), ctypes.byref(dp)) != 0


def test_rccl_standin_build_binds_only_its_own_rccl():
    """The RCCL stand-in test library (tests/rccl/libmpjx_rccl_standin.so, test infrastructure) is the SAME
    libmpjx objects linked against tests/rccl/rccl_standin.hip: it exports every C-ABI symbol of
    include/mpjx.h, no nccl* symbol (the stand-in's are hidden, so libmpjx binds them inside the library
    whatever librccl a process has loaded), needs no librccl, and leaves nothing undefined."""
    import subprocess

    so = os.path.join(ROOT, "tests", "rccl", "libmpjx_rccl_standin.so")
    if not os.path.exists(so):
        pytest.skip("stand-in not built (make -C mpjexpress_amd tests)")
    nm = subprocess.run(["nm", "-D", so], capture_output=True, text=True, check=True).stdout
    defined = {ln.split()[-1] for ln in nm.splitlines() if len(ln.split()) == 3 and ln.split()[1] in "TW"}
    undef = {ln.split()[-1] for ln in nm.splitlines() if ln.split()[0] == "U"}
    assert set(header_functions()) <= defined
    assert not any(s.startswith("nccl") for s in defined | undef)
    assert {"rsi_log", "rsi_log_clear", "rsi_is_standin", "rsi_fail_next"} <= defined
    ldd = subprocess.run(["ldd", so], capture_output=True, text=True).stdout
    assert "librccl" not in ldd
