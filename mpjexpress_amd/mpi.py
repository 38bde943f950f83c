"""mpiJava-1.2 style host mirror of the reduction path, over libmpjx's C ABI.

Mirrors the reference's public surface for this path so that tests and callers read like the
reference's own programs (e.g. test/mpi/ccl/allreduce.java):

    MPI.SUM, MPI.DOUBLE, ...                     src/mpi/MPI.java:117-126, src/mpi/Datatype.java:57-66
    comm.Reduce(send, soff, recv, roff, count, datatype, op, root)      src/mpi/Intracomm.java:740-760
    comm.Allreduce(send, soff, recv, roff, count, datatype, op)          src/mpi/Intracomm.java:787-793
    comm.Reduce_scatter(send, soff, recv, roff, recvcounts, datatype, op) src/mpi/Intracomm.java:833-840
    comm.Scan(send, soff, recv, roff, count, datatype, op)               src/mpi/Intracomm.java:879-885
    comm.Bcast(buf, off, count, datatype, root), comm.Barrier(), comm.Rank(), comm.Size()

Buffers are device-resident torch tensors (the device path) or numpy arrays (the host-resident
path, as Java heap arrays are). Offsets and counts are in elements. Calls block until the result is
in the receive buffer, like the Java methods. Errors raise MPIException (src/mpi/MPIException.java:42).
`MPI.isOldSelected` mirrors conf `mpjexpress.mpi.old.collectives` (src/mpi/MPI.java:70,266).
"""
import ctypes
import threading

import numpy as np

from . import _lib

FLAG_OLD_COLLECTIVES = 0x1
FLAG_FAITHFUL = 0x2


class MPIException(RuntimeError):
    pass


class Datatype:
    def __init__(self, base_type, name, np_dtype, torch_dtype_name):
        self.baseType = base_type
        self.name = name
        self.np_dtype = np.dtype(np_dtype)
        self.torch_dtype_name = torch_dtype_name
        self.byteSize = self.np_dtype.itemsize

    def Size(self):
        return 1

    def __repr__(self):
        return f"MPI.{self.name}"


class Op:
    def __init__(self, code, name):
        self.opCode = code
        self.name = name

    def __repr__(self):
        return f"MPI.{self.name}"


class MPI:
    BYTE = Datatype(1, "BYTE", np.int8, "int8")
    CHAR = Datatype(2, "CHAR", np.uint16, "uint16")
    SHORT = Datatype(3, "SHORT", np.int16, "int16")
    BOOLEAN = Datatype(4, "BOOLEAN", np.uint8, "uint8")
    INT = Datatype(5, "INT", np.int32, "int32")
    LONG = Datatype(6, "LONG", np.int64, "int64")
    FLOAT = Datatype(7, "FLOAT", np.float32, "float32")
    DOUBLE = Datatype(8, "DOUBLE", np.float64, "float64")

    MAX = Op(1, "MAX")
    MIN = Op(2, "MIN")
    SUM = Op(3, "SUM")
    PROD = Op(4, "PROD")
    LAND = Op(5, "LAND")
    BAND = Op(6, "BAND")
    LOR = Op(7, "LOR")
    BOR = Op(8, "BOR")
    LXOR = Op(9, "LXOR")
    BXOR = Op(10, "BXOR")

    isOldSelected = False  # conf mpjexpress.mpi.old.collectives
    COMM_WORLD = None


DATATYPES = [MPI.BYTE, MPI.CHAR, MPI.SHORT, MPI.BOOLEAN, MPI.INT, MPI.LONG, MPI.FLOAT, MPI.DOUBLE]
OPS = [MPI.MAX, MPI.MIN, MPI.SUM, MPI.PROD, MPI.LAND, MPI.BAND, MPI.LOR, MPI.BOR, MPI.LXOR, MPI.BXOR]


def _wrap(fn, *args):
    try:
        _lib.call(fn, *args)
    except _lib.MPJXError as e:
        raise MPIException(str(e)) from None


def _is_torch(buf):
    t = getattr(_lib, "torch", None)
    return t is not None and isinstance(buf, t.Tensor)


def _dev_ptr(buf, off, dt, need):
    """Device address of element `off` of a contiguous torch tensor, checking type and extent."""
    if not buf.is_cuda:
        raise MPIException("torch tensor buffers must be on a GPU device")
    if not buf.is_contiguous():
        raise MPIException("buffer must be contiguous")
    if buf.element_size() != dt.byteSize:
        raise MPIException(f"buffer element size {buf.element_size()} does not match {dt}")
    if off < 0 or off + need > buf.numel():
        raise MPIException(f"offset {off} + count {need} exceeds buffer length {buf.numel()}")
    return buf.data_ptr() + off * dt.byteSize


def _host_ptr(buf, off, dt, need):
    if not isinstance(buf, np.ndarray) or not buf.flags.c_contiguous:
        raise MPIException("host buffers must be C-contiguous numpy arrays")
    if buf.dtype.itemsize != dt.byteSize:
        raise MPIException(f"buffer dtype {buf.dtype} does not match {dt}")
    if off < 0 or off + need > buf.size:
        raise MPIException(f"offset {off} + count {need} exceeds buffer length {buf.size}")
    return buf.ctypes.data + off * dt.byteSize


class Intracomm:
    """One rank's view of a communicator (src/mpi/Intracomm.java)."""

    def __init__(self, handle, faithful=False):
        self._h = ctypes.c_void_p(handle)
        self.faithful = faithful
        r, s, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _wrap("mpjx_comm_rank", self._h, ctypes.byref(r))
        _wrap("mpjx_comm_size", self._h, ctypes.byref(s))
        _wrap("mpjx_comm_device", self._h, ctypes.byref(d))
        self._rank, self._size, self.device = r.value, s.value, d.value

    # -- mpiJava accessors
    def Rank(self):
        return self._rank

    def Size(self):
        return self._size

    @property
    def handle(self):
        return self._h

    def flags(self):
        f = FLAG_OLD_COLLECTIVES if MPI.isOldSelected else 0
        return f | (FLAG_FAITHFUL if self.faithful else 0)

    def Barrier(self):
        _wrap("mpjx_barrier", self._h)

    def Free(self):
        if self._h:
            _wrap("mpjx_comm_destroy", self._h)
            self._h = ctypes.c_void_p(None)

    def _sync_in(self, *bufs):
        if any(_is_torch(b) for b in bufs):
            _lib.torch.cuda.synchronize(self.device)

    def _sync_out(self):
        _wrap("mpjx_comm_synchronize", self._h)

    # -- reductions
    def Reduce(self, sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op, root):
        is_root = self._rank == root
        if _is_torch(sendbuf):
            self._sync_in(sendbuf)
            sp = _dev_ptr(sendbuf, sendoffset, datatype, count)
            rp = _dev_ptr(recvbuf, recvoffset, datatype, count) if is_root else None
            _wrap("mpjx_reduce", self._h, sp, rp, count, datatype.baseType, op.opCode, root,
                  self.flags(), None)
            self._sync_out()
        else:
            sp = _host_ptr(sendbuf, sendoffset, datatype, count)
            rp = _host_ptr(recvbuf, recvoffset, datatype, count) if is_root else None
            _wrap("mpjx_reduce_host", self._h, sp, rp, count, datatype.baseType, op.opCode, root,
                  self.flags())

    def Allreduce(self, sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op):
        if _is_torch(sendbuf):
            self._sync_in(sendbuf, recvbuf)
            sp = _dev_ptr(sendbuf, sendoffset, datatype, count)
            rp = _dev_ptr(recvbuf, recvoffset, datatype, count)
            _wrap("mpjx_allreduce", self._h, sp, rp, count, datatype.baseType, op.opCode,
                  self.flags(), None)
            self._sync_out()
        else:
            sp = _host_ptr(sendbuf, sendoffset, datatype, count)
            rp = _host_ptr(recvbuf, recvoffset, datatype, count)
            _wrap("mpjx_allreduce_host", self._h, sp, rp, count, datatype.baseType, op.opCode,
                  self.flags())

    def Reduce_scatter(self, sendbuf, sendoffset, recvbuf, recvoffset, recvcounts, datatype, op):
        counts = list(recvcounts)[: self._size]
        if len(counts) < self._size:
            raise MPIException("recvcounts shorter than the communicator")
        rc = (ctypes.c_int64 * self._size)(*counts)
        total, mine = sum(counts), counts[self._rank]
        if _is_torch(sendbuf):
            self._sync_in(sendbuf, recvbuf)
            sp = _dev_ptr(sendbuf, sendoffset, datatype, total)
            rp = _dev_ptr(recvbuf, recvoffset, datatype, mine)
            _wrap("mpjx_reduce_scatter", self._h, sp, rp, rc, datatype.baseType, op.opCode,
                  self.flags(), None)
            self._sync_out()
        else:
            sp = _host_ptr(sendbuf, sendoffset, datatype, total)
            rp = _host_ptr(recvbuf, recvoffset, datatype, mine)
            _wrap("mpjx_reduce_scatter_host", self._h, sp, rp, rc, datatype.baseType, op.opCode,
                  self.flags())

    def Scan(self, sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op):
        if _is_torch(sendbuf):
            self._sync_in(sendbuf, recvbuf)
            sp = _dev_ptr(sendbuf, sendoffset, datatype, count)
            rp = _dev_ptr(recvbuf, recvoffset, datatype, count)
            _wrap("mpjx_scan", self._h, sp, rp, count, datatype.baseType, op.opCode, self.flags(),
                  None)
            self._sync_out()
        else:
            sp = _host_ptr(sendbuf, sendoffset, datatype, count)
            rp = _host_ptr(recvbuf, recvoffset, datatype, count)
            _wrap("mpjx_scan_host", self._h, sp, rp, count, datatype.baseType, op.opCode,
                  self.flags())

    def Bcast(self, buf, offset, count, datatype, root):
        if not _is_torch(buf):
            raise MPIException("Bcast is provided for device-resident buffers")
        self._sync_in(buf)
        p = _dev_ptr(buf, offset, datatype, count)
        _wrap("mpjx_bcast", self._h, p, count, datatype.baseType, root, None)
        self._sync_out()


def combine(op, datatype, inout, inp, count=None, stream=None):
    """inout[i] = inp[i] (op) inout[i] on device tensors (one typed Op.perform)."""
    n = inout.numel() if count is None else count
    a = _dev_ptr(inout, 0, datatype, n)
    b = _dev_ptr(inp, 0, datatype, n)
    _wrap("mpjx_combine", op.opCode, datatype.baseType, a, b, n, stream)


def smp_world(nranks, devices=None, faithful=False):
    """Multicore mode: `nranks` ranks that are threads of this process (smpdev)."""
    devices = list(devices) if devices is not None else [0] * nranks
    arr = (ctypes.c_void_p * nranks)()
    devs = (ctypes.c_int * nranks)(*devices)
    _wrap("mpjx_comm_init_smp", arr, nranks, devs)
    return [Intracomm(arr[r], faithful=faithful) for r in range(nranks)]


def run_multicore(comms, fn):
    """Run fn(comm) on one thread per rank, as MulticoreStarter does
    (src/runtime/starter/MulticoreStarter.java:309-322); returns per-rank results, re-raises errors."""
    out, err = [None] * len(comms), [None] * len(comms)

    def body(r):
        try:
            if _lib.torch is not None:
                _lib.torch.cuda.set_device(comms[r].device)
            out[r] = fn(comms[r])
        except BaseException as e:  # noqa: BLE001
            err[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(len(comms))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return out


def unique_id():
    buf = ctypes.create_string_buffer(128)
    _wrap("mpjx_get_unique_id", buf)
    return buf.raw


def Init(rank, size, device, uid):
    """One process per GPU over RCCL: every rank passes the same 128-byte unique id (from rank 0's
    unique_id(), shared out of band, e.g. torch.distributed.broadcast_object_list)."""
    h = ctypes.c_void_p()
    _wrap("mpjx_comm_init_rank", ctypes.byref(h), size, uid, rank, device)
    MPI.COMM_WORLD = Intracomm(h.value)
    return MPI.COMM_WORLD
