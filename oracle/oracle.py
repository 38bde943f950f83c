"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes/numpy front end of oracle/mpjx_oracle.c, the plain-C restatement of MPJ Express 0.44's
reduction path (typed Op bodies, PureIntracomm MST/FT/BKT/Scan algorithms). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the product package
(mpjexpress_amd) never does.

Parity pinning: reference known-answer tests test/mpi/ccl/*.java (INT SUM/PROD) via
tests/golden/; the remaining (op, type) rows are pinned by source reading only.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libmpjx_oracle.so")

# mpi.Datatype base types (src/mpi/Datatype.java:57-66) and mpjdev.Constants op codes
# (src/mpjdev/Constants.java:53-62).
BYTE, CHAR, SHORT, BOOLEAN, INT, LONG, FLOAT, DOUBLE = range(1, 9)
MAX, MIN, SUM, PROD, LAND, BAND, LOR, BOR, LXOR, BXOR = range(1, 11)
MAXLOC, MINLOC = 11, 12
SHORT2, INT2, LONG2, FLOAT2, DOUBLE2 = 0x103, 0x105, 0x106, 0x107, 0x108
PAIR_BASE = {SHORT2: SHORT, INT2: INT, LONG2: LONG, FLOAT2: FLOAT, DOUBLE2: DOUBLE}
FLAG_OLD = 1
FLAG_FAITHFUL = 2

NP_DTYPE = {
    BYTE: np.int8, CHAR: np.uint16, SHORT: np.int16, BOOLEAN: np.uint8,
    INT: np.int32, LONG: np.int64, FLOAT: np.float32, DOUBLE: np.float64,
}
# pair types: one element = (value, index), as structured numpy records of the base type
for _p, _b in PAIR_BASE.items():
    NP_DTYPE[_p] = np.dtype([("v", NP_DTYPE[_b]), ("l", NP_DTYPE[_b])])
TYPE_NAMES = {BYTE: "BYTE", CHAR: "CHAR", SHORT: "SHORT", BOOLEAN: "BOOLEAN", INT: "INT",
              LONG: "LONG", FLOAT: "FLOAT", DOUBLE: "DOUBLE", SHORT2: "SHORT2", INT2: "INT2",
              LONG2: "LONG2", FLOAT2: "FLOAT2", DOUBLE2: "DOUBLE2"}
OP_NAMES = {MAX: "MAX", MIN: "MIN", SUM: "SUM", PROD: "PROD", LAND: "LAND", BAND: "BAND",
            LOR: "LOR", BOR: "BOR", LXOR: "LXOR", BXOR: "BXOR", MAXLOC: "MAXLOC", MINLOC: "MINLOC"}

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        vp, i, u, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_int64
        pp = ctypes.POINTER(ctypes.c_void_p)
        L.ora_type_size.argtypes = [i]
        L.ora_check.argtypes = [i, i]
        L.ora_apply.argtypes = [i, i, vp, vp, i64, i64]
        L.ora_apply.restype = None
        L.ora_reduce.argtypes = [i, u, pp, i, pp, i, i, i, i, i]
        L.ora_allreduce.argtypes = [i, u, pp, i, pp, i, i, i, i]
        L.ora_reduce_scatter.argtypes = [i, u, pp, i, pp, i, ctypes.POINTER(ctypes.c_int), i, i]
        L.ora_scan.argtypes = [i, u, pp, i, pp, i, i, i, i]
        L.ora_bcast.argtypes = [i, u, pp, i, i, i, i]
        L.ora_time_combine.argtypes = [i, i, i64, i]
        L.ora_time_combine.restype = ctypes.c_double
        L.ora_time_allreduce_mst.argtypes = [i, i64, i, i]
        L.ora_time_allreduce_mst.restype = ctypes.c_double
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.ora_jrandom_seed.argtypes = [u64p, i64]
        L.ora_jrandom_seed.restype = None
        L.ora_jrandom_next_int.argtypes = [u64p]
        L.ora_jrandom_next_int.restype = ctypes.c_int32
        L.ora_jrandom_next_double.argtypes = [u64p]
        L.ora_jrandom_next_double.restype = ctypes.c_double
        L.ora_jgf_sparse_gen.argtypes = [i64, i, i, i, vp, vp, vp, vp]
        L.ora_jgf_sparse_rep.argtypes = [vp, vp, vp, vp, vp, i, i]
        L.ora_jgf_sparse_rep.restype = None
        L.ora_jgf_ytotal.argtypes = [vp, vp, i]
        L.ora_jgf_ytotal.restype = ctypes.c_double
        L.ora_md_new.argtypes = [i]
        L.ora_md_new.restype = vp
        L.ora_md_free.argtypes = [vp]
        L.ora_md_free.restype = None
        L.ora_md_mdsize.argtypes = [vp]
        L.ora_md_forces.argtypes = [vp, i, i, vp, vp, vp, vp, vp]
        L.ora_md_forces.restype = None
        L.ora_md_finish.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int32]
        L.ora_md_finish.restype = None
        L.ora_md_ek.argtypes = [vp]
        L.ora_md_ek.restype = ctypes.c_double
        L.ora_md_interactions.argtypes = [vp]
        L.ora_md_interactions.restype = ctypes.c_int32
        L.ora_java_log.argtypes = [ctypes.c_double]
        L.ora_java_log.restype = ctypes.c_double
        L.ora_jgf_raytracer_rows.argtypes = [i, vp]
        L.ora_jgf_raytracer_partial.argtypes = [vp, i, i, i]
        L.ora_jgf_raytracer_partial.restype = ctypes.c_int64
        _lib = L
    return _lib


def check(op, type_):
    return lib().ora_check(op, type_)


def valid_pairs():
    """The 46 typed (op, type) classes of the reference (ops 1-10 on base types)."""
    return [(op, t) for op in range(1, 11) for t in range(1, 9) if check(op, t) == 0]


def loc_pairs():
    """MAXLOC / MINLOC on the five pair types."""
    return [(op, t) for op in (MAXLOC, MINLOC) for t in PAIR_BASE]


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def apply(op, type_, acc, inp):
    """acc[i] = inp[i] (op) acc[i] in place (the typed perform loop body)."""
    assert acc.dtype == np.dtype(NP_DTYPE[type_]) and inp.dtype == acc.dtype and acc.flags.c_contiguous
    lib().ora_apply(op, type_, acc.ctypes.data, inp.ctypes.data, 0, acc.size)
    return acc


def _prep(sends, type_):
    sends = [np.ascontiguousarray(s, dtype=NP_DTYPE[type_]).copy() for s in sends]
    return sends


def reduce(sends, count, type_, op, root, flags=0, soff=0, roff=0, recv_len=None):
    sends = _prep(sends, type_)
    P = len(sends)
    n = recv_len if recv_len is not None else max(soff, roff) + count
    recvs = [np.zeros(n, dtype=NP_DTYPE[type_]) for _ in range(P)]
    rc = lib().ora_reduce(P, flags, _ptrs(sends), soff, _ptrs(recvs), roff, count, type_, op, root)
    if rc:
        raise ValueError(f"ora_check={rc}")
    return recvs


def allreduce(sends, count, type_, op, flags=0, soff=0, roff=0):
    sends = _prep(sends, type_)
    P = len(sends)
    recvs = [np.zeros(max(soff, roff) + count, dtype=NP_DTYPE[type_]) for _ in range(P)]
    rc = lib().ora_allreduce(P, flags, _ptrs(sends), soff, _ptrs(recvs), roff, count, type_, op)
    if rc:
        raise ValueError(f"ora_check={rc}")
    return recvs


def reduce_scatter(sends, recvcounts, type_, op, flags=0, soff=0, roff=0):
    sends = _prep(sends, type_)
    P = len(sends)
    # the reference's FT path reduces the whole vector into recvbuf first: size it for sum(recvcounts)
    recvs = [np.zeros(max(soff, roff) + max(1, sum(recvcounts)), dtype=NP_DTYPE[type_]) for _ in range(P)]
    rcs = (ctypes.c_int * P)(*recvcounts)
    rc = lib().ora_reduce_scatter(P, flags, _ptrs(sends), soff, _ptrs(recvs), roff, rcs, type_, op)
    if rc:
        raise ValueError(f"ora_check={rc}")
    return [r[roff:roff + recvcounts[i]] for i, r in enumerate(recvs)], sends


def scan(sends, count, type_, op, flags=0, soff=0, roff=0):
    sends = _prep(sends, type_)
    P = len(sends)
    recvs = [np.zeros(max(soff, roff) + count, dtype=NP_DTYPE[type_]) for _ in range(P)]
    rc = lib().ora_scan(P, flags, _ptrs(sends), soff, _ptrs(recvs), roff, count, type_, op)
    if rc:
        raise ValueError(f"ora_check={rc}")
    return recvs


def time_combine(op, type_, n, reps):
    return lib().ora_time_combine(op, type_, n, reps)


def time_allreduce_mst(P, n, reps, pin=True):
    return lib().ora_time_allreduce_mst(P, n, reps, 1 if pin else 0)


class JavaRandom:
    """java.util.Random (48-bit LCG per the Java API specification), as oracle/jgf_sparsematmult.c."""

    def __init__(self, seed):
        self._s = ctypes.c_uint64()
        lib().ora_jrandom_seed(ctypes.byref(self._s), seed)

    def nextInt(self):
        return lib().ora_jrandom_next_int(ctypes.byref(self._s))

    def nextDouble(self):
        return lib().ora_jrandom_next_double(ctypes.byref(self._s))


# JGF SparseMatmult, test/jgf_mpj_benchmarks/section2/sparsematmult/JGFSparseMatmultBench.java:33-38,148
JGF_SEED = 10101010
JGF_SIZES = {"A": (50000, 50000, 250000), "B": (100000, 100000, 500000), "C": (500000, 500000, 2500000)}
JGF_REFVAL = {"A": 75.02484945753453, "B": 150.0130719633895, "C": 749.5245870753752}
JGF_ITERS = 200


class JgfSparse:
    """The benchmark's inputs (x, row, col, val in draw order) and its per-rank work split."""

    def __init__(self, size="A"):
        self.M, self.N, self.nz = JGF_SIZES[size]
        self.x = np.zeros(self.N, np.float64)
        self.row = np.zeros(self.nz, np.int32)
        self.col = np.zeros(self.nz, np.int32)
        self.val = np.zeros(self.nz, np.float64)
        rc = lib().ora_jgf_sparse_gen(JGF_SEED, self.M, self.N, self.nz, self.x.ctypes.data,
                                      self.row.ctypes.data, self.col.ctypes.data, self.val.ctypes.data)
        if rc:
            raise ValueError("a drawn index is negative: the reference would throw")

    def share(self, rank, P):
        """[lo, hi) of the nonzeros rank `rank` owns (JGFSparseMatmultBench.java:73-80,116-128)."""
        p = (self.nz + P - 1) // P
        rem = p - (p * P - self.nz)
        cnt = rem if (rank == P - 1 and p * (rank + 1) > self.nz) else p
        return rank * p, rank * p + cnt

    def rep(self, p_y, rank, P):
        """One rep of SparseMatmult.java:241-244 on rank's share: p_y[row[i]] += x[col[i]] * val[i]."""
        lo, hi = self.share(rank, P)
        lib().ora_jgf_sparse_rep(p_y.ctypes.data, self.x.ctypes.data, self.row.ctypes.data,
                                 self.col.ctypes.data, self.val.ctypes.data, lo, hi)

    def ytotal(self, y):
        """SparseMatmult.java:255-259: sum of y[buf_row[i]] over all nonzeros in draw order."""
        y = np.ascontiguousarray(y, np.float64)
        return lib().ora_jgf_ytotal(y.ctypes.data, self.row.ctypes.data, self.nz)


def jgf_sparse_matmult(P, flags=0, size="A", iters=JGF_ITERS, return_y=False):
    """SparseMatmult.test with P simulated ranks and the oracle's Allreduce(DOUBLE, SUM): returns
    rank 0's ytotal (and every rank's final y with return_y)."""
    J = JgfSparse(size)
    p_y = [np.zeros(J.M, np.float64) for _ in range(P)]
    y = None
    for _ in range(iters):
        for r in range(P):
            J.rep(p_y[r], r, P)
        y = allreduce(p_y, J.M, DOUBLE, SUM, flags)
    return (J.ytotal(y[0]), y) if return_y else J.ytotal(y[0])


# JGF MolDyn, test/jgf_mpj_benchmarks/section3/moldyn/JGFMolDynBench.java:72 (size A, B)
MD_REFVAL = {"A": 1731.4306625334357, "B": 7397.392307839352}


class MolDyn:
    """One rank's MolDyn state (oracle/jgf_moldyn.c). step_forces() runs a move up to the Allreduces
    and returns (xf, yf, zf, ev[epot, vir], inter[1]) — the buffers md.java reduces in place;
    step_finish() takes them back reduced."""

    def __init__(self, size="A"):
        self._h = lib().ora_md_new({"A": 0, "B": 1}[size])
        self.n = lib().ora_md_mdsize(self._h)
        self.moves = lib().ora_md_moves()

    def step_forces(self, rank, P):
        xf, yf, zf = (np.zeros(self.n) for _ in range(3))
        ev = np.zeros(2)
        inter = np.zeros(1, np.int32)
        lib().ora_md_forces(self._h, rank, P, xf.ctypes.data, yf.ctypes.data, zf.ctypes.data, ev.ctypes.data,
                            inter.ctypes.data)
        return xf, yf, zf, ev, inter

    def step_finish(self, xf, yf, zf, ev, inter):
        lib().ora_md_finish(self._h, xf.ctypes.data, yf.ctypes.data, zf.ctypes.data, ev.ctypes.data, int(inter[0]))

    @property
    def ek(self):
        return lib().ora_md_ek(self._h)

    @property
    def interactions(self):
        return lib().ora_md_interactions(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ora_md_free(self._h)
            self._h = None


def jgf_moldyn(P, flags=0, size="A"):
    """md.runiters() with P simulated ranks, the oracle's Allreduce(SUM) for the three force arrays,
    epot / vir (DOUBLE, two calls of one element in the reference) and interactions (INT). Returns
    (rank 0's ek, every rank's interaction count)."""
    ranks = [MolDyn(size) for _ in range(P)]
    for _ in range(ranks[0].moves):
        parts = [m.step_forces(r, P) for r, m in enumerate(ranks)]
        red = [allreduce([p[k] for p in parts], parts[0][k].size, DOUBLE if k < 4 else INT, SUM, flags)
               for k in range(3)]
        ep = allreduce([p[3][:1] for p in parts], 1, DOUBLE, SUM, flags)
        vi = allreduce([p[3][1:] for p in parts], 1, DOUBLE, SUM, flags)
        it = allreduce([p[4] for p in parts], 1, INT, SUM, flags)
        for r, m in enumerate(ranks):
            m.step_finish(red[0][r], red[1][r], red[2][r], np.array([ep[r][0], vi[r][0]]), it[r])
    return ranks[0].ek, [m.interactions for m in ranks]


# JGF RayTracer, test/jgf_mpj_benchmarks/section3/raytracer/JGFRayTracerBench.java:50,87-88 and
# RayTracer.java:85,275-279: the pixel checksum reduced with an in-place Reduce(DOUBLE, SUM, root 0)
RT_SIZES = {"A": 150, "B": 500}
RT_REFVAL = {"A": 2676692, "B": 29827635}
_rt_rows = {}


def jgf_raytracer_rows(size="A"):
    """Every row's checksum contribution of the size x size picture (oracle/jgf_raytracer.c); cached."""
    if size not in _rt_rows:
        n = RT_SIZES[size]
        rows = np.zeros(n, np.int64)
        if lib().ora_jgf_raytracer_rows(n, rows.ctypes.data) != 0:
            raise RuntimeError("ora_jgf_raytracer_rows failed")
        _rt_rows[size] = rows
    return _rt_rows[size]


def jgf_raytracer_partials(P, size="A"):
    """tmp_checksum[0] of every rank at P ranks: (double) of its rows' checksum (RayTracer.java:240, 275)."""
    rows = jgf_raytracer_rows(size)
    return [np.array([float(lib().ora_jgf_raytracer_partial(rows.ctypes.data, rows.size, r, P))]) for r in range(P)]


def jgf_raytracer(P, flags=0, size="A"):
    """render() with P simulated ranks and the oracle's Reduce(DOUBLE, SUM, root 0) of the partial
    checksums: rank 0's checksum = (long) tmp_checksum[0] (RayTracer.java:276-279)."""
    red = reduce(jgf_raytracer_partials(P, size), 1, DOUBLE, SUM, 0, flags=flags)
    return int(red[0][0])
