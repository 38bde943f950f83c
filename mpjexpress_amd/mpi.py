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
import os
import struct
import threading

import numpy as np

from . import _lib

FLAG_OLD_COLLECTIVES = 0x1
FLAG_FAITHFUL = 0x2
FLAG_BLOCKING = 0x10  # the mpiJava calls are blocking: return complete (include/mpjx.h)


class MPIException(RuntimeError):
    pass


class Datatype:
    """A basic type, or a (value, index) pair type MPI.SHORT2..DOUBLE2 = Contiguous(2, base)
    (src/mpi/MPI.java:110-114). `code` is what crosses the C ABI (0x100 | base for pairs); offsets
    are in base elements (Java array indices), counts in datatype elements (pairs for *2 types)."""

    def __init__(self, base_type, name, np_dtype, torch_dtype_name, size=1):
        self.baseType = base_type
        self.name = name
        self.np_dtype = np.dtype(np_dtype)
        self.torch_dtype_name = torch_dtype_name
        self.size = size
        self.code = base_type if size == 1 else (0x100 | base_type)
        self.baseSize = self.np_dtype.itemsize
        self.byteSize = self.baseSize * size

    def Size(self):
        return self.size

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
    SHORT2 = Datatype(3, "SHORT2", np.int16, "int16", 2)
    INT2 = Datatype(5, "INT2", np.int32, "int32", 2)
    LONG2 = Datatype(6, "LONG2", np.int64, "int64", 2)
    FLOAT2 = Datatype(7, "FLOAT2", np.float32, "float32", 2)
    DOUBLE2 = Datatype(8, "DOUBLE2", np.float64, "float64", 2)

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
    MAXLOC = Op(11, "MAXLOC")
    MINLOC = Op(12, "MINLOC")

    isOldSelected = False  # conf mpjexpress.mpi.old.collectives
    COMM_WORLD = None


DATATYPES = [MPI.BYTE, MPI.CHAR, MPI.SHORT, MPI.BOOLEAN, MPI.INT, MPI.LONG, MPI.FLOAT, MPI.DOUBLE]
OPS = [MPI.MAX, MPI.MIN, MPI.SUM, MPI.PROD, MPI.LAND, MPI.BAND, MPI.LOR, MPI.BOR, MPI.LXOR, MPI.BXOR,
       MPI.MAXLOC, MPI.MINLOC]
PAIR_TYPES = {0x103: MPI.SHORT2, 0x105: MPI.INT2, 0x106: MPI.LONG2, 0x107: MPI.FLOAT2, 0x108: MPI.DOUBLE2}


def datatype(code):
    """Datatype for a C-ABI type code (1..8, or 0x100 | base for the pair types)."""
    return PAIR_TYPES[code] if code in PAIR_TYPES else DATATYPES[code - 1]


def _wrap(fn, *args):
    try:
        _lib.call(fn, *args)
    except _lib.MPJXError as e:
        raise MPIException(str(e)) from None


def _is_torch(buf):
    t = getattr(_lib, "torch", None)
    return t is not None and isinstance(buf, t.Tensor)


def _dev_ptr(buf, off, dt, need):
    """Device address of base element `off` of a contiguous torch tensor of the datatype's base
    type, checking type and extent (`need` datatype elements)."""
    if not buf.is_cuda:
        raise MPIException("torch tensor buffers must be on a GPU device")
    if not buf.is_contiguous():
        raise MPIException("buffer must be contiguous")
    if buf.element_size() != dt.baseSize:
        raise MPIException(f"buffer element size {buf.element_size()} does not match {dt}")
    if off < 0 or off + need * dt.size > buf.numel():
        raise MPIException(f"offset {off} + count {need} exceeds buffer length {buf.numel()}")
    return buf.data_ptr() + off * dt.baseSize


def _host_ptr(buf, off, dt, need):
    """Host address of base element `off` (numpy arrays of the base type, or of structured pairs)."""
    if not isinstance(buf, np.ndarray) or not buf.flags.c_contiguous:
        raise MPIException("host buffers must be C-contiguous numpy arrays")
    if buf.dtype.itemsize not in (dt.baseSize, dt.byteSize):
        raise MPIException(f"buffer dtype {buf.dtype} does not match {dt}")
    nbase = buf.size * (buf.dtype.itemsize // dt.baseSize)
    if off < 0 or off + need * dt.size > nbase:
        raise MPIException(f"offset {off} + count {need} exceeds buffer length {nbase}")
    return buf.ctypes.data + off * dt.baseSize


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
        return f | (FLAG_FAITHFUL if self.faithful else 0) | FLAG_BLOCKING

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

    # -- communicator constructors: a new libmpjx world per sub-communicator, of the parent's engine
    # kind ("smp": rank threads of this process; "rccl": one process per GPU over RCCL; "ipc": processes
    # mapping each other's buffers). NativeIntracomm.java:160-215 keeps Split/Create on its strategy.
    _kind = "smp"

    def _world_base(self):
        """128 random bytes drawn by rank 0 and broadcast (device Bcast) to every rank."""
        torch = _lib.torch
        dev = torch.device("cuda", self.device)
        base = torch.zeros(128, dtype=torch.int8, device=dev)
        if self._rank == 0:
            base.copy_(torch.frombuffer(bytearray(os.urandom(128)), dtype=torch.int8))
        self.Bcast(base, 0, 128, MPI.BYTE, 0)
        return bytes(base.cpu().numpy().view(np.uint8))

    def _world_id(self, members):
        """Collective: the 128-byte id of this rank's new world (None outside every new group). Multicore
        worlds derive theirs from one shared random base (made unique per group by _sub_world); the
        process engines take their group leader's: an RCCL unique id (mpjx_get_unique_id, whose
        bootstrap root lives in the leader's process) or random bytes (IPC), gathered to every rank."""
        if self._kind == "smp":
            return self._world_base()
        leader = members[0] if members else None
        mine = bytes(128)
        if self._rank == leader:
            mine = unique_id() if self._kind == "rccl" else os.urandom(128)
        table = self._all_bytes(mine)
        return table[leader] if members else None

    def _sub_world(self, members, tag, base):
        """The world of `members` (parent ranks, in new-rank order) on their devices."""
        if self._rank not in members:
            return None
        h = ctypes.c_void_p()
        me = members.index(self._rank)
        if self._kind == "rccl":
            _wrap("mpjx_comm_init_rank", ctypes.byref(h), len(members), base, me, self.device)
        elif self._kind == "ipc":
            _wrap("mpjx_comm_init_ipc", ctypes.byref(h), len(members), base, me, self.device)
        else:
            uid = bytearray(base)
            for i, b in enumerate(struct.pack("<q", tag)):
                uid[i] ^= b
            devs = (ctypes.c_int * len(members))(*[self._devices[m] for m in members])
            _wrap("mpjx_comm_init_smp_rank", ctypes.byref(h), len(members), bytes(uid), me, devs)
        c = Intracomm(h.value, faithful=self.faithful)
        c._kind = self._kind
        c._devices = [self._devices[m] for m in members]
        return c

    def _all_ints(self, vals):
        """Every rank's int32 row (gathered to rank 0 on the device, then broadcast)."""
        torch = _lib.torch
        dev = torch.device("cuda", self.device)
        k, P = len(vals), self._size
        mine = torch.tensor(vals, dtype=torch.int32, device=dev)
        table = torch.zeros(k * P, dtype=torch.int32, device=dev)
        Gather(self, mine, 0, k, table, 0, k, MPI.INT, 0)
        self.Bcast(table, 0, k * P, MPI.INT, 0)
        return table.cpu().numpy().reshape(P, k)

    def _all_bytes(self, b):
        """Every rank's byte string of len(b) (all equal), gathered and broadcast on the device."""
        torch = _lib.torch
        dev = torch.device("cuda", self.device)
        k, P = len(b), self._size
        mine = torch.frombuffer(bytearray(b), dtype=torch.int8).to(dev)
        table = torch.zeros(k * P, dtype=torch.int8, device=dev)
        Gather(self, mine, 0, k, table, 0, k, MPI.BYTE, 0)
        self.Bcast(table, 0, k * P, MPI.BYTE, 0)
        t = table.cpu().numpy().view(np.uint8).reshape(P, k)
        return [bytes(t[r]) for r in range(P)]

    def Split(self, color, key):
        """Intracomm.Split (src/mpi/PureIntracomm.java:201-280; NativeIntracomm.java:160-170 keeps the
        result on its strategy, as this does): ranks of one color form a communicator ordered by key,
        ties by parent rank; a negative color (MPI.UNDEFINED) gets None. Collective."""
        t = self._all_ints([color, key, self.device])
        self._devices = [int(d) for d in t[:, 2]]
        members = None
        if color >= 0:
            members = sorted((r for r in range(self._size) if t[r, 0] == color), key=lambda r: (t[r, 1], r))
        base = self._world_id(members)
        if color < 0:
            return None
        return self._sub_world(members, int(color), base)

    def Create(self, group):
        """Intracomm.Create (src/mpi/PureIntracomm.java:302-309; NativeIntracomm.java:200-215): `group`
        lists the parent ranks of the new communicator in new-rank order (mpi.Group's members, the same
        on every rank); ranks outside it get None. Collective."""
        members = [int(m) for m in group]
        t = self._all_ints([self.device])
        self._devices = [int(d) for d in t[:, 0]]
        base = self._world_id(members if self._rank in members else None)
        return self._sub_world(members, -1, base)

    # -- reductions
    def Reduce(self, sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op, root):
        """recvbuf is significant at the root; with faithful=True every rank's recvbuf is left as
        PureIntracomm leaves it (MST: the rank's sub-tree partial, FT: its own send copy)."""
        is_root = self._rank == root
        if _is_torch(sendbuf):
            self._sync_in(sendbuf)
            sp = _dev_ptr(sendbuf, sendoffset, datatype, count)
            rp = _dev_ptr(recvbuf, recvoffset, datatype, count) if (is_root or self.faithful) else None
            _wrap("mpjx_reduce", self._h, sp, rp, count, datatype.code, op.opCode, root,
                  self.flags(), None)
            self._sync_out()
        else:
            sp = _host_ptr(sendbuf, sendoffset, datatype, count)
            rp = _host_ptr(recvbuf, recvoffset, datatype, count) if (is_root or self.faithful) else None
            _wrap("mpjx_reduce_host", self._h, sp, rp, count, datatype.code, op.opCode, root,
                  self.flags())

    def Allreduce(self, sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op):
        if _is_torch(sendbuf):
            self._sync_in(sendbuf, recvbuf)
            sp = _dev_ptr(sendbuf, sendoffset, datatype, count)
            rp = _dev_ptr(recvbuf, recvoffset, datatype, count)
            _wrap("mpjx_allreduce", self._h, sp, rp, count, datatype.code, op.opCode,
                  self.flags(), None)
            self._sync_out()
        else:
            sp = _host_ptr(sendbuf, sendoffset, datatype, count)
            rp = _host_ptr(recvbuf, recvoffset, datatype, count)
            _wrap("mpjx_allreduce_host", self._h, sp, rp, count, datatype.code, op.opCode,
                  self.flags())

    def Reduce_scatter(self, sendbuf, sendoffset, recvbuf, recvoffset, recvcounts, datatype, op):
        counts = list(recvcounts)[: self._size]
        if len(counts) < self._size:
            raise MPIException("recvcounts shorter than the communicator")
        rc = (ctypes.c_int64 * self._size)(*counts)
        total, mine = sum(counts), counts[self._rank]  # datatype elements
        if _is_torch(sendbuf):
            self._sync_in(sendbuf, recvbuf)
            sp = _dev_ptr(sendbuf, sendoffset, datatype, total)
            rp = _dev_ptr(recvbuf, recvoffset, datatype, mine)
            _wrap("mpjx_reduce_scatter", self._h, sp, rp, rc, datatype.code, op.opCode,
                  self.flags(), None)
            self._sync_out()
        else:
            sp = _host_ptr(sendbuf, sendoffset, datatype, total)
            rp = _host_ptr(recvbuf, recvoffset, datatype, mine)
            _wrap("mpjx_reduce_scatter_host", self._h, sp, rp, rc, datatype.code, op.opCode,
                  self.flags())

    def Scan(self, sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op):
        if _is_torch(sendbuf):
            self._sync_in(sendbuf, recvbuf)
            sp = _dev_ptr(sendbuf, sendoffset, datatype, count)
            rp = _dev_ptr(recvbuf, recvoffset, datatype, count)
            _wrap("mpjx_scan", self._h, sp, rp, count, datatype.code, op.opCode, self.flags(),
                  None)
            self._sync_out()
        else:
            sp = _host_ptr(sendbuf, sendoffset, datatype, count)
            rp = _host_ptr(recvbuf, recvoffset, datatype, count)
            _wrap("mpjx_scan_host", self._h, sp, rp, count, datatype.code, op.opCode,
                  self.flags())

    def Gather(self, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root):
        Gather(self, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root)

    def Scatter(self, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root):
        Scatter(self, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root)

    def Bcast(self, buf, offset, count, datatype, root):
        if not _is_torch(buf):
            raise MPIException("Bcast is provided for device-resident buffers")
        self._sync_in(buf)
        p = _dev_ptr(buf, offset, datatype, count)
        _wrap("mpjx_bcast", self._h, p, count, datatype.code, root, None)
        self._sync_out()


def _gs(fn, comm, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root, send_all):
    if not (_is_torch(sendbuf) or _is_torch(recvbuf)):
        raise MPIException(f"{fn} is provided for device-resident buffers")
    if sendcount != recvcount:
        raise MPIException("sendcount must equal recvcount")
    comm._sync_in(*(b for b in (sendbuf, recvbuf) if b is not None))
    is_root = comm.Rank() == root
    n_send = sendcount * (comm.Size() if (send_all and is_root) else 1)
    n_recv = recvcount * (comm.Size() if (not send_all and is_root) else 1)
    sp = _dev_ptr(sendbuf, sendoffset, datatype, n_send) if (is_root or not send_all) else None
    rp = _dev_ptr(recvbuf, recvoffset, datatype, n_recv) if (is_root or send_all) else None
    _wrap(fn, comm.handle, sp, rp, sendcount, datatype.code, root, None)
    comm._sync_out()


def Gather(comm, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root):
    """Intracomm.Gather (src/mpi/PureIntracomm.java:782-1053) on device buffers, equal counts."""
    _gs("mpjx_gather", comm, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root, False)


def Scatter(comm, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root):
    """Intracomm.Scatter (src/mpi/PureIntracomm.java:1055-1171) on device buffers, equal counts."""
    _gs("mpjx_scatter", comm, sendbuf, sendoffset, sendcount, recvbuf, recvoffset, recvcount, datatype, root, True)


def combine(op, datatype, inout, inp, count=None, stream=None):
    """inout[i] = inp[i] (op) inout[i] on device tensors (one typed Op.perform)."""
    n = inout.numel() // datatype.size if count is None else count
    a = _dev_ptr(inout, 0, datatype, n)
    b = _dev_ptr(inp, 0, datatype, n)
    _wrap("mpjx_combine", op.opCode, datatype.code, a, b, n, stream)


def smp_world(nranks, devices=None, faithful=False):
    """Multicore mode: `nranks` ranks that are threads of this process (smpdev)."""
    devices = list(devices) if devices is not None else [0] * nranks
    arr = (ctypes.c_void_p * nranks)()
    devs = (ctypes.c_int * nranks)(*devices)
    _wrap("mpjx_comm_init_smp", arr, nranks, devs)
    comms = [Intracomm(arr[r], faithful=faithful) for r in range(nranks)]
    for c in comms:
        c._devices = list(devices)
    return comms


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
    MPI.COMM_WORLD._kind = "rccl"
    return MPI.COMM_WORLD


def InitIPC(rank, size, device, uid):
    """Processes of one node mapping each other's device buffers through HIP IPC (no RCCL): every
    rank passes the same 128-byte id (e.g. rank 0's unique_id(), or any bytes unique to the world)."""
    h = ctypes.c_void_p()
    _wrap("mpjx_comm_init_ipc", ctypes.byref(h), size, uid, rank, device)
    MPI.COMM_WORLD = Intracomm(h.value)
    MPI.COMM_WORLD._kind = "ipc"
    return MPI.COMM_WORLD
