"""ctypes binding of libmpjx.so (include/mpjx.h).

The library is built in-tree (mpjexpress_amd/lib/libmpjx.so, `make -C mpjexpress_amd`). There is no
CPU fallback: if the library is missing or cannot load, every entry point raises.
"""
import ctypes
import os

# torch (when present) must be loaded BEFORE libmpjx: both resolve libamdhip64.so.7 / librccl.so.1 by
# soname, and loading torch first makes libmpjx bind to the HIP runtime torch already mapped instead
# of mapping a second copy from /opt/rocm.
try:  # pragma: no cover - environment dependent
    import torch  # noqa: F401
except Exception:  # noqa: BLE001
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPJX_LIB_PATH: another build of the same library (A/B timing of two builds in one GPU job)
LIB_PATH = os.environ.get("MPJX_LIB_PATH") or os.path.join(_HERE, "lib", "libmpjx.so")

_lib = None


class MPJXError(RuntimeError):
    """Raised for a non-zero libmpjx status (maps to mpi.MPIException on the Java side)."""

    def __init__(self, status, fn, detail):
        self.status = status
        super().__init__(f"{fn}: {strerror(status)} ({status}): {detail}")


def _declare(L):
    c_int, c_i64, vp, c_uint = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint
    pi64 = ctypes.POINTER(ctypes.c_int64)
    sig = {
        "mpjx_version": ([], c_int),
        "mpjx_runtime_versions": ([ctypes.POINTER(c_int), ctypes.POINTER(c_int)], c_int),
        "mpjx_strerror": ([c_int], ctypes.c_char_p),
        "mpjx_last_error": ([], ctypes.c_char_p),
        "mpjx_type_size": ([c_int], c_int),
        "mpjx_op_check": ([c_int, c_int], c_int),
        "mpjx_device_count": ([ctypes.POINTER(c_int)], c_int),
        "mpjx_combine": ([c_int, c_int, vp, vp, c_i64, vp], c_int),
        "mpjx_combine_multi": ([c_int, c_int, c_int, c_int, ctypes.POINTER(vp), ctypes.POINTER(vp), c_i64,
                                c_int, c_uint, vp], c_int),
        "mpjx_mpjbuf_section": ([vp, c_i64, c_i64, ctypes.POINTER(c_int), pi64, pi64], c_int),
        "mpjx_mpjbuf_combine": ([c_int, c_int, vp, vp, c_i64, c_i64, vp, c_uint, vp], c_int),
        "mpjx_get_unique_id": ([ctypes.c_char_p], c_int),
        "mpjx_comm_init_rank": ([ctypes.POINTER(vp), c_int, ctypes.c_char_p, c_int, c_int], c_int),
        "mpjx_comm_init_smp": ([ctypes.POINTER(vp), c_int, ctypes.POINTER(c_int)], c_int),
        "mpjx_comm_init_smp_rank": ([ctypes.POINTER(vp), c_int, ctypes.c_char_p, c_int, ctypes.POINTER(c_int)],
                                    c_int),
        "mpjx_comm_init_ipc": ([ctypes.POINTER(vp), c_int, ctypes.c_char_p, c_int, c_int], c_int),
        "mpjx_comm_destroy": ([vp], c_int),
        "mpjx_comm_rank": ([vp, ctypes.POINTER(c_int)], c_int),
        "mpjx_comm_size": ([vp, ctypes.POINTER(c_int)], c_int),
        "mpjx_comm_device": ([vp, ctypes.POINTER(c_int)], c_int),
        "mpjx_comm_stream": ([vp, ctypes.POINTER(vp)], c_int),
        "mpjx_comm_synchronize": ([vp], c_int),
        "mpjx_barrier": ([vp], c_int),
        "mpjx_comm_phase_timing": ([vp, c_int], c_int),
        "mpjx_comm_last_phases": ([vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(c_int)], c_int),
        "mpjx_comm_pipeline_trace": ([vp, ctypes.POINTER(ctypes.c_float), c_int, ctypes.POINTER(c_int)], c_int),
        "mpjx_reduce": ([vp, vp, vp, c_i64, c_int, c_int, c_int, c_uint, vp], c_int),
        "mpjx_allreduce": ([vp, vp, vp, c_i64, c_int, c_int, c_uint, vp], c_int),
        "mpjx_reduce_scatter": ([vp, vp, vp, pi64, c_int, c_int, c_uint, vp], c_int),
        "mpjx_scan": ([vp, vp, vp, c_i64, c_int, c_int, c_uint, vp], c_int),
        "mpjx_bcast": ([vp, vp, c_i64, c_int, c_int, vp], c_int),
        "mpjx_gather": ([vp, vp, vp, c_i64, c_int, c_int, vp], c_int),
        "mpjx_scatter": ([vp, vp, vp, c_i64, c_int, c_int, vp], c_int),
        "mpjx_reduce_host": ([vp, vp, vp, c_i64, c_int, c_int, c_int, c_uint], c_int),
        "mpjx_allreduce_host": ([vp, vp, vp, c_i64, c_int, c_int, c_uint], c_int),
        "mpjx_reduce_scatter_host": ([vp, vp, vp, pi64, c_int, c_int, c_uint], c_int),
        "mpjx_scan_host": ([vp, vp, vp, c_i64, c_int, c_int, c_uint], c_int),
        "mpjx_host_alloc": ([ctypes.POINTER(vp), c_i64], c_int),
        "mpjx_host_free": ([vp], c_int),
        "mpjx_comm_last_host_form": ([vp, ctypes.POINTER(c_int)], c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return sig


EXPORTS = None


def lib():
    """Load libmpjx.so (once). Raises if it is not built — there is no fallback path."""
    global _lib, EXPORTS
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libmpjx.so not found at {LIB_PATH}: build it with `make -C mpjexpress_amd` "
                "(or __graft_entry__.build()); the HIP path has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        EXPORTS = sorted(_declare(L))
        _lib = L
    return _lib


def strerror(status):
    return lib().mpjx_strerror(status).decode()


def check(status, fn):
    if status != 0:
        detail = lib().mpjx_last_error().decode(errors="replace")
        raise MPJXError(status, fn, detail)
    return status


def call(name, *args):
    return check(getattr(lib(), name)(*args), name)
