"""GPU parity of Reduce / Allreduce / Reduce_scatter / Scan / Bcast through libmpjx.

Ranks run as threads of this process on the one GPU (multicore mode, the reference's smpdev), so
P > 1 exercises the full exchange -> P-way combine -> exchange engine on a single MI355X. Results
are compared bit-exactly with the oracle's restatement of the reference algorithms
(src/mpi/PureIntracomm.java), including float/double — the GPU evaluates the same combine order.
"""
import contextlib
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from util import make_input, same_bits

pytestmark = pytest.mark.gpu

PS = [1, 2, 3, 4, 5, 8]


@contextlib.contextmanager
def old_collectives(on):
    from mpjexpress_amd.mpi import MPI

    prev = MPI.isOldSelected
    MPI.isOldSelected = on
    try:
        yield
    finally:
        MPI.isOldSelected = prev


def _world(P, faithful=False):
    from mpjexpress_amd import mpi

    return mpi.smp_world(P, [0] * P, faithful=faithful)


def _free(comms):
    for c in comms:
        c.Free()


def _t(a):
    """numpy -> device tensor; (value, index) pair records go as their interleaved base type."""
    import torch

    if a.dtype.names:
        a = a.view(a.dtype[0])
    return torch.from_numpy(a).cuda()


def _np(t, like):
    """device tensor -> numpy in the dtype of `like` (pair records re-assembled)."""
    a = t.cpu().numpy()
    return a.view(like.dtype) if like.dtype.names else a


def run(kind, P, op, type_, n=None, recvcounts=None, root=0, flags=0, inputs=None):
    """Run one collective on P smp ranks; return (gpu results per rank, oracle results per rank)."""
    from mpjexpress_amd import mpi

    dt, opx = mpi.datatype(type_), mpi.OPS[op - 1]
    total = sum(recvcounts) if recvcounts is not None else n
    sends = inputs or [make_input(type_, total, 7919 * (r + 1) + total, op=op) for r in range(P)]
    comms = _world(P, faithful=bool(flags & O.FLAG_FAITHFUL))
    try:
        def body(c):
            r = c.Rank()
            s = _t(sends[r])
            if kind == "reduce_scatter":
                out = _t(np.zeros(max(1, recvcounts[r]), sends[r].dtype))
                c.Reduce_scatter(s, 0, out, 0, recvcounts, dt, opx)
                return _np(out, sends[r])[: recvcounts[r]]
            out = _t(np.zeros(max(1, n), sends[r].dtype))
            if kind == "reduce":
                c.Reduce(s, 0, out, 0, n, dt, opx, root)
            elif kind == "allreduce":
                c.Allreduce(s, 0, out, 0, n, dt, opx)
            elif kind == "scan":
                c.Scan(s, 0, out, 0, n, dt, opx)
            return _np(out, sends[r])[:n]

        with old_collectives(bool(flags & O.FLAG_OLD)):
            got = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    if kind == "reduce":
        exp = O.reduce(sends, n, type_, op, root, flags=flags)
    elif kind == "allreduce":
        exp = O.allreduce(sends, n, type_, op, flags=flags)
    elif kind == "scan":
        exp = O.scan(sends, n, type_, op, flags=flags)
    else:
        exp, _ = O.reduce_scatter(sends, list(recvcounts), type_, op, flags=flags)
    exp = [e[: (recvcounts[r] if recvcounts is not None else n)] for r, e in enumerate(exp)]
    return got, exp


def _assert(kind, got, exp, op, type_, only=None, ctx=""):
    for r in range(len(got)):
        if only is not None and r != only:
            continue
        assert same_bits(type_, op, got[r], exp[r]), f"{kind} rank {r} {O.OP_NAMES[op]} {O.TYPE_NAMES[type_]} {ctx}"


# ---- the reference's own known-answer tests (test/mpi/ccl/*.java), run on the GPU path ----------

@pytest.mark.parametrize("P", PS)
def test_ccl_allreduce_kat(P):
    """test/mpi/ccl/allreduce.java:73-86: out[i] = i on every rank, expect in[k] == k * tasks."""
    from mpjexpress_amd.mpi import MPI

    comms = _world(P)

    def body(c):
        tasks = c.Size()
        j = 1
        while j <= 10000:
            out = _t(np.arange(j, dtype=np.int32))
            inn = _t(np.zeros(10000, np.int32))
            c.Allreduce(out, 0, inn, 0, j, MPI.INT, MPI.SUM)
            c.Barrier()
            got = inn.cpu().numpy()[:j]
            assert np.array_equal(got, np.arange(j, dtype=np.int32) * tasks), f"bad answer j={j}"
            j *= 10

    try:
        from mpjexpress_amd import mpi
        mpi.run_multicore(comms, body)
    finally:
        _free(comms)


@pytest.mark.parametrize("P", PS)
def test_ccl_reduce_scan_reduce_scatter_kat(P):
    """test/mpi/ccl/reduce.java:73-87 (root = tasks/2), reduce2.java (PROD, checked at P == 2),
    scan.java:73-85, reduce_scatter.java:81-96 (recvcounts = 10 each)."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    comms = _world(P)

    def body(c):
        me, tasks = c.Rank(), c.Size()
        root = tasks // 2
        j = 1
        while j <= 10000:
            out = _t(np.arange(j, dtype=np.int32))
            inn = _t(np.zeros(10000, np.int32))
            c.Reduce(out, 0, inn, 0, j, MPI.INT, MPI.SUM, root)
            if me == root:
                assert np.array_equal(inn.cpu().numpy()[:j], np.arange(j) * tasks)
            c.Reduce(out, 0, inn, 0, j, MPI.INT, MPI.PROD, root)
            if me == root and tasks == 2:
                assert np.array_equal(inn.cpu().numpy()[:j], np.arange(j) ** 2)
            c.Scan(out, 0, inn, 0, j, MPI.INT, MPI.SUM)
            assert np.array_equal(inn.cpu().numpy()[:j], np.arange(j) * (me + 1))
            j *= 10
        j = 10
        out = _t(np.arange(j * tasks, dtype=np.int32))
        inn = _t(np.zeros(j, np.int32))
        c.Reduce_scatter(out, 0, inn, 0, [j] * tasks, MPI.INT, MPI.SUM)
        assert np.array_equal(inn.cpu().numpy(), tasks * (me * j + np.arange(j)))

    try:
        mpi.run_multicore(comms, body)
    finally:
        _free(comms)


# ---- randomized parity over the (op, type) matrix ----------------------------------------------------

PAIRS = O.valid_pairs() if hasattr(O, "valid_pairs") else []


@pytest.mark.parametrize("P", PS)
@pytest.mark.parametrize("op,type_", PAIRS)
def test_allreduce_all_pairs(P, op, type_):
    got, exp = run("allreduce", P, op, type_, n=1037)
    _assert("allreduce", got, exp, op, type_)


@pytest.mark.parametrize("P", [2, 3, 5, 8])
@pytest.mark.parametrize("op,type_", [(O.SUM, O.DOUBLE), (O.PROD, O.FLOAT), (O.MAX, O.DOUBLE),
                                      (O.MIN, O.FLOAT), (O.BXOR, O.INT), (O.LAND, O.BOOLEAN),
                                      (O.SUM, O.CHAR), (O.MAX, O.BYTE)])
def test_reduce_every_root(P, op, type_):
    for root in range(P):
        got, exp = run("reduce", P, op, type_, n=777, root=root)
        _assert("reduce", got, exp, op, type_, only=root, ctx=f"root={root}")


@pytest.mark.parametrize("P", PS)
@pytest.mark.parametrize("op,type_", [(O.SUM, O.DOUBLE), (O.SUM, O.FLOAT), (O.MAX, O.FLOAT),
                                      (O.BAND, O.INT), (O.BXOR, O.INT), (O.PROD, O.LONG),
                                      (O.LOR, O.BOOLEAN), (O.MIN, O.SHORT)])
def test_scan_pairs(P, op, type_):
    got, exp = run("scan", P, op, type_, n=2049)
    _assert("scan", got, exp, op, type_)


@pytest.mark.parametrize("P", PS)
@pytest.mark.parametrize("op,type_", [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.BAND, O.INT),
                                      (O.BXOR, O.INT), (O.SUM, O.BYTE), (O.LXOR, O.BOOLEAN)])
def test_reduce_scatter_ragged(P, op, type_):
    rng = np.random.default_rng(P)
    for rc in ([64] * P, list(rng.integers(0, 300, P)), [0] * (P - 1) + [5]):
        got, exp = run("reduce_scatter", P, op, type_, recvcounts=[int(x) for x in rc])
        _assert("reduce_scatter", got, exp, op, type_, ctx=f"rc={rc}")


@pytest.mark.parametrize("P", [2, 3, 4, 8])
@pytest.mark.parametrize("kind", ["reduce", "allreduce", "reduce_scatter", "scan"])
def test_old_collectives_orders(P, kind):
    """conf mpjexpress.mpi.old.collectives=true: FT_Reduce / FT_Allreduce (a different fold order
    on every rank) / FT_Reduce_scatter — float results must still match bit for bit."""
    for op, type_ in [(O.SUM, O.DOUBLE), (O.SUM, O.FLOAT), (O.MAX, O.DOUBLE), (O.PROD, O.FLOAT)]:
        if kind == "reduce_scatter":
            got, exp = run(kind, P, op, type_, recvcounts=[100] * P, flags=O.FLAG_OLD)
        else:
            got, exp = run(kind, P, op, type_, n=1500, root=P - 1, flags=O.FLAG_OLD)
        _assert(kind, got, exp, op, type_, only=(P - 1 if kind == "reduce" else None))


@pytest.mark.parametrize("P", [2, 3, 4, 5, 8])
def test_faithful_defects(P):
    """FAITHFUL flag: BOR/BXOR never combine (A3) and the P>=3 bucket Reduce_scatter (A9)."""
    for op, type_ in [(O.BOR, O.INT), (O.BXOR, O.LONG)]:
        for kind in ("allreduce", "scan"):
            got, exp = run(kind, P, op, type_, n=300, flags=O.FLAG_FAITHFUL)
            _assert(kind, got, exp, op, type_, ctx="faithful")
        got, exp = run("reduce", P, op, type_, n=300, root=P // 2, flags=O.FLAG_FAITHFUL)
        _assert("reduce", got, exp, op, type_, only=P // 2, ctx="faithful")
    for op, type_ in [(O.SUM, O.INT), (O.PROD, O.INT), (O.MAX, O.DOUBLE), (O.MIN, O.FLOAT),
                      (O.BAND, O.INT), (O.BXOR, O.INT), (O.SUM, O.DOUBLE)]:
        got, exp = run("reduce_scatter", P, op, type_, recvcounts=[40] * P, flags=O.FLAG_FAITHFUL)
        _assert("reduce_scatter", got, exp, op, type_, ctx="faithful")


def test_p_greater_than_8_compositions():
    """P > 8 ranks (multicore on one GPU): the chunked fold and the recursive MST composition."""
    for P in (9, 13):
        for op, type_ in [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT)]:
            got, exp = run("allreduce", P, op, type_, n=5000)
            _assert("allreduce", got, exp, op, type_, ctx=f"P={P}")
            got, exp = run("reduce", P, op, type_, n=3000, root=P - 2)
            _assert("reduce", got, exp, op, type_, only=P - 2, ctx=f"P={P}")
            got, exp = run("scan", P, op, type_, n=999)
            _assert("scan", got, exp, op, type_, ctx=f"P={P}")
            got, exp = run("allreduce", P, op, type_, n=2000, flags=O.FLAG_OLD)
            _assert("allreduce-old", got, exp, op, type_, ctx=f"P={P}")


@pytest.mark.parametrize("engine", ["direct", "copy", "oneshot"])
def test_smp_direct_and_copy_engines(engine, monkeypatch):
    """Multicore mode reduces in place across ranks (the kernel reads every rank's send block and
    writes every rank's recv block); MPJX_SMP_COPY=1 selects the exchange engine's PLAN (the one the RCCL
    engine runs) with device copies as its transport, not RCCL itself — with MPJX_ONESHOT_KIB=0 the two-exchange plan at every size, by default the small-vector
    one-shot (all-gather + local combine) for Allreduce/Scan. All must match the oracle bit for bit,
    including P > 8 and ragged blocks."""
    copy = engine != "direct"
    if copy:
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    if engine == "copy":
        monkeypatch.setenv("MPJX_ONESHOT_KIB", "0")
    for P in (2, 3, 9):
        for op, type_ in [(O.SUM, O.DOUBLE), (O.BXOR, O.SHORT), (O.MIN, O.FLOAT)]:
            for flags in (0, O.FLAG_OLD):
                got, exp = run("allreduce", P, op, type_, n=4099, flags=flags)
                _assert("allreduce", got, exp, op, type_, ctx=f"P={P} copy={copy} flags={flags}")
                got, exp = run("reduce", P, op, type_, n=777, root=P - 1, flags=flags)
                _assert("reduce", got, exp, op, type_, only=P - 1, ctx=f"P={P} copy={copy}")
            got, exp = run("scan", P, op, type_, n=1001)
            _assert("scan", got, exp, op, type_, ctx=f"P={P} copy={copy}")
            got, exp = run("reduce_scatter", P, op, type_, recvcounts=[17 * (r % 3) + 5 for r in range(P)])
            _assert("reduce_scatter", got, exp, op, type_, ctx=f"P={P} copy={copy}")


def config0_inputs(pattern, P=4, n=(1 << 20) // 8):
    """BASELINE configs[0] (Allreduce SUM double[] 1 MiB, 4 ranks): SURVEY §8d C1 streams (uniform
    [-1, 1), splitmix64 seed 0x4D504A00 + 1000*1 + rank, the bench's generator) or the reference
    microbenchmark's own pattern A[i] = 1/(i+1) on every rank
    (test/microbenchmarkmpiJava/allreduce/Allreduce.java:48-62)."""
    import synth

    if pattern == "uniform":
        return [synth.uniform_np(np.arange(n, dtype=np.uint64), synth.seed(1, r)) for r in range(P)]
    return [1.0 / (np.arange(n, dtype=np.float64) + 1.0) for _ in range(P)]


@pytest.mark.parametrize("pattern", ["uniform", "reference"])
@pytest.mark.parametrize("engine", ["direct", "exchange", "oneshot"])
def test_config0_allreduce_sum_double_1mib_p4(engine, pattern, monkeypatch):
    """configs[0] at its own shape — Allreduce SUM double 1 MiB on 4 ranks (multicore mode, the
    reference's CPU configuration) — on every multicore engine, bit-exact against the oracle's
    MST_Reduce(0) + Bcast restatement (src/mpi/PureIntracomm.java:2168-2185)."""
    if engine != "direct":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    monkeypatch.setenv("MPJX_ONESHOT_KIB", "2048" if engine == "oneshot" else "0")
    n = (1 << 20) // 8
    sends = config0_inputs(pattern)
    got, exp = run("allreduce", 4, O.SUM, O.DOUBLE, n=n, inputs=sends)
    _assert("allreduce", got, exp, O.SUM, O.DOUBLE, ctx=f"configs[0] {engine} {pattern}")
    if pattern == "reference":  # every rank holds the same A: the sum is 4A, exactly (power of two)
        assert np.array_equal(got[0], 4.0 * sends[0])


@pytest.mark.parametrize("P", [3, 9])
def test_smp_in_place_every_order(P):
    """In-place Allreduce (new and old orders) and in-place Scan: in multicore mode a rank's recv block
    is also an input other ranks' results depend on, so writes must follow all reads."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    n = 3000
    sends = [make_input(O.DOUBLE, n, 555 + r, specials=False) for r in range(P)]
    exp_new = O.allreduce(sends, n, O.DOUBLE, O.SUM)
    exp_old = O.allreduce(sends, n, O.DOUBLE, O.SUM, flags=O.FLAG_OLD)
    exp_scan = O.scan(sends, n, O.DOUBLE, O.SUM)
    comms = _world(P)

    def body(c):
        r = c.Rank()
        a, b, d = _t(sends[r].copy()), _t(sends[r].copy()), _t(sends[r].copy())
        c.Allreduce(a, 0, a, 0, n, MPI.DOUBLE, MPI.SUM)
        c.Scan(d, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
        MPI.isOldSelected = True  # per-rank FT orders; all ranks set it before the call
        try:
            c.Barrier()
            c.Allreduce(b, 0, b, 0, n, MPI.DOUBLE, MPI.SUM)
            c.Barrier()
        finally:
            MPI.isOldSelected = False
        return a.cpu().numpy(), b.cpu().numpy(), d.cpu().numpy()

    try:
        out = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    for r in range(P):
        assert np.array_equal(out[r][0].view(np.uint64), exp_new[r].view(np.uint64)), r
        assert np.array_equal(out[r][1].view(np.uint64), exp_old[r].view(np.uint64)), r
        assert np.array_equal(out[r][2].view(np.uint64), exp_scan[r].view(np.uint64)), r


def test_in_place_allreduce_and_bcast():
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    P, n = 4, 10000
    sends = [make_input(O.DOUBLE, n, 31 + r, specials=False) for r in range(P)]
    exp = O.allreduce(sends, n, O.DOUBLE, O.SUM)
    comms = _world(P)

    def body(c):
        b = _t(sends[c.Rank()].copy())
        c.Allreduce(b, 0, b, 0, n, MPI.DOUBLE, MPI.SUM)
        res = b.cpu().numpy()
        x = _t(sends[c.Rank()].copy())
        c.Bcast(x, 0, n, MPI.DOUBLE, 2)
        return res, x.cpu().numpy()

    try:
        out = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    for r in range(P):
        assert np.array_equal(out[r][0].view(np.uint64), exp[r].view(np.uint64))
        assert np.array_equal(out[r][1], sends[2])


def test_offsets_and_host_buffers():
    """Element offsets into device buffers and the host-resident (Java heap array) variants."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    P, n, so, ro = 3, 1234, 5, 11
    sends = [make_input(O.FLOAT, n + so, 77 + r) for r in range(P)]
    exp_all = O.allreduce([s[so:] for s in sends], n, O.FLOAT, O.MAX)
    exp_scan = O.scan([s[so:] for s in sends], n, O.FLOAT, O.SUM)
    comms = _world(P)

    def body(c):
        r = c.Rank()
        s = _t(sends[r])
        d = _t(np.zeros(n + ro, np.float32))
        c.Allreduce(s, so, d, ro, n, MPI.FLOAT, MPI.MAX)
        hs, hr = sends[r].copy(), np.zeros(n + ro, np.float32)
        c.Scan(hs, so, hr, ro, n, MPI.FLOAT, MPI.SUM)
        return d.cpu().numpy()[ro:], hr[ro:]

    try:
        out = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    for r in range(P):
        assert same_bits(O.FLOAT, O.MAX, out[r][0], exp_all[r])
        assert same_bits(O.FLOAT, O.SUM, out[r][1], exp_scan[r])


def test_rccl_single_rank_comm():
    """One-process-per-GPU communicator (RCCL) at world size 1 on the box's single GPU."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    c = mpi.Init(0, 1, 0, mpi.unique_id())
    try:
        x = make_input(O.DOUBLE, 4096, 5, specials=False)
        s, d = _t(x), _t(np.zeros_like(x))
        c.Allreduce(s, 0, d, 0, x.size, MPI.DOUBLE, MPI.SUM)
        assert np.array_equal(d.cpu().numpy(), x)
        c.Barrier()
    finally:
        c.Free()


def test_rccl_transport_calls_at_world_size_1():
    """MPJX_P1_EXCHANGE=1 routes a 1-rank RCCL Allreduce through the full exchange path, so the
    ncclAllToAll / ncclAllToAllv / ncclAllGather calls used at N>1 run on this one-GPU box — and the
    chunk pipeline's second lane (ncclCommSplit) with it."""
    import subprocess
    import sys

    code = r'''
import numpy as np, torch, sys
sys.path.insert(0, "oracle")
from mpjexpress_amd import mpi
from mpjexpress_amd.mpi import MPI
c = mpi.Init(0, 1, 0, mpi.unique_id())
for n in (4096, 4099, 1 << 20):   # equal 256-B blocks -> AllToAll; ragged -> AllToAllv
    x = np.random.default_rng(n).uniform(-1, 1, n)
    s = torch.from_numpy(x).cuda(); d = torch.zeros_like(s)
    c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
    assert np.array_equal(d.cpu().numpy(), x), n
    b = s.clone(); c.Allreduce(b, 0, b, 0, n, MPI.DOUBLE, MPI.MAX)
    assert np.array_equal(b.cpu().numpy(), x), n
# skewed input slots (MPJX_SLOT_SKEW): equal blocks go through ncclAllToAllv instead of ncclAllToAll
import os
os.environ["MPJX_SLOT_SKEW"] = "4096"
for n in (4096, 1 << 20):
    x = np.random.default_rng(n + 1).uniform(-1, 1, n)
    s = torch.from_numpy(x).cuda(); d = torch.zeros_like(s)
    c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
    assert np.array_equal(d.cpu().numpy(), x), ("skew", n)
os.environ.pop("MPJX_SLOT_SKEW")
# the chunk pipeline: exchange #1 on the call's stream, all-gathers on a second RCCL communicator
# (ncclCommSplit) on the gather stream; 1 MiB chunks, ragged last chunk, twice (the lane is reused)
import os
os.environ["MPJX_PIPE_CHUNK_MIB"] = "1"
for n in ((8 << 20) // 8 + 5, (3 << 20) // 8):
    x = np.random.default_rng(n).uniform(-1, 1, n)
    s = torch.from_numpy(x).cuda(); d = torch.zeros_like(s)
    c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
    assert np.array_equal(d.cpu().numpy(), x), ("pipelined", n)
c.Free()
print("ok")
'''
    import os

    env = dict(os.environ, MPJX_P1_EXCHANGE="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_rccl_native_allreduce_routing_world_size_1():
    """MPJX_RCCL_NATIVE=1: an Allreduce whose result cannot depend on the combine
    order runs as ONE ncclAllReduce — byte/int/long SUM, PROD, MAX, MIN at any P; double SUM and PROD
    at P <= 2 (the reference's order there is one commutative operation per element, x1 (op) x0,
    PureIntracomm.java:1943-1992) — and everything else keeps the exchange engine: float (RCCL's binary32
    subnormal handling unverified), float MAX/MIN (Java's NaN and +-0 rule is order-dependent), 16-bit
    types (RCCL carries none), pair types, big-endian operands. At world size 1 with MPJX_P1_EXCHANGE=1 the RCCL calls run on this one-GPU box; the
    engine that ran is read from the phase marks (6 = ncclAllReduce, 1 = exchange). The arithmetic of a
    P = 2 ncclAllReduce is checked where it can run: tools/rccl_preflight's rccl_native variant and the
    N = 2 bench line (full-result checksum) on a multi-GPU node."""
    import subprocess
    import sys

    code = r'''
import ctypes, numpy as np, torch, sys
from mpjexpress_amd import mpi, _lib
from mpjexpress_amd.mpi import MPI
L = _lib.lib()
c = mpi.Init(0, 1, 0, mpi.unique_id())
h = c.handle
_lib.check(L.mpjx_comm_phase_timing(h, 1), "phase")
def engine():
    ms = (ctypes.c_float * 3)(); e = ctypes.c_int()
    _lib.check(L.mpjx_comm_last_phases(h, ms, ctypes.byref(e)), "phases")
    return e.value
rng = np.random.default_rng(5)
cases = [(MPI.DOUBLE, MPI.SUM, 6), (MPI.DOUBLE, MPI.PROD, 6), (MPI.FLOAT, MPI.SUM, 1), (MPI.INT, MPI.SUM, 6),
         (MPI.LONG, MPI.PROD, 6), (MPI.BYTE, MPI.MAX, 6), (MPI.INT, MPI.MIN, 6),
         (MPI.DOUBLE, MPI.MAX, 1), (MPI.FLOAT, MPI.MIN, 1), (MPI.SHORT, MPI.SUM, 1), (MPI.CHAR, MPI.SUM, 1),
         (MPI.INT, MPI.BXOR, 1), (MPI.BOOLEAN, MPI.LAND, 1)]
n = 300007
for dt, op, want in cases:
    x = (rng.uniform(-1, 1, n) if np.dtype(dt.np_dtype).kind == "f" else rng.integers(-100, 100, n)).astype(dt.np_dtype)
    if dt is MPI.BOOLEAN:
        x = (x != 0).astype(np.uint8)
    s = torch.from_numpy(x).cuda(); d = torch.zeros_like(s)
    c.Allreduce(s, 0, d, 0, n, dt, op)
    got = engine()
    assert got == want, (dt, op, got, want)
    assert np.array_equal(d.cpu().numpy().view(np.uint8), x.view(np.uint8)), (dt, op)
# in place, and the big-endian flags keep the exchange engine (the swap lives in the combine kernels)
x = rng.uniform(-1, 1, n); b = torch.from_numpy(x).cuda()
c.Allreduce(b, 0, b, 0, n, MPI.DOUBLE, MPI.SUM)
assert engine() == 6 and np.array_equal(b.cpu().numpy(), x)
s = torch.from_numpy(x.astype(">f8").view(np.float64)).cuda(); d = torch.zeros_like(s)
_lib.check(L.mpjx_allreduce(h, s.data_ptr(), d.data_ptr(), n, 8, 3, 0x4 | 0x8, None), "be")
torch.cuda.synchronize()
assert engine() == 1 and np.array_equal(d.cpu().numpy(), s.cpu().numpy())
import os
# the routing is the communicator's, read at init (ADVICE r5): changing the variable later changes nothing
os.environ["MPJX_RCCL_NATIVE"] = "0"
s = torch.from_numpy(x).cuda(); d = torch.zeros_like(s)
c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
assert engine() == 6
c.Free()
# a new communicator with the variable off: the exchange engine
c = mpi.Init(0, 1, 0, mpi.unique_id()); h = c.handle
_lib.check(L.mpjx_comm_phase_timing(h, 1), "phase")
c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
assert engine() == 1
c.Free()
os.environ["MPJX_RCCL_NATIVE_P2"] = "1"  # the P = 2 form: this world has one rank, so not taken
c = mpi.Init(0, 1, 0, mpi.unique_id()); h = c.handle
_lib.check(L.mpjx_comm_phase_timing(h, 1), "phase")
c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
assert engine() == 1 and np.array_equal(d.cpu().numpy(), x)
c.Free()
print("ok")
'''
    import os

    env = dict(os.environ, MPJX_P1_EXCHANGE="1", MPJX_RCCL_NATIVE="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr



def test_rccl_timeout_aborts_instead_of_hanging():
    """MPJX_RCCL_TIMEOUT_S: a blocking wait on an RCCL communicator polls ncclCommGetAsyncError and
    gives up after the limit — the communicator is aborted and later calls on it fail with
    MPJX_ERR_RCCL instead of the rank hanging on a dead peer. Forced here with a 50 us limit, shorter
    than one 1 GiB exchange-path Allreduce at world size 1 (MPJX_P1_EXCHANGE=1)."""
    import subprocess
    import sys

    code = r'''
import os, torch
from mpjexpress_amd import _lib, mpi
L = _lib.lib()
c = mpi.Init(0, 1, 0, mpi.unique_id())
n = (1 << 30) // 8
s = torch.ones(n, dtype=torch.float64, device="cuda"); d = torch.empty_like(s)
torch.cuda.synchronize()
os.environ["MPJX_RCCL_TIMEOUT_S"] = "0.00005"
rc = L.mpjx_allreduce(c.handle, s.data_ptr(), d.data_ptr(), n, 8, 3, 0, None)
w = L.mpjx_comm_synchronize(c.handle)
msg = L.mpjx_last_error().decode()
rc2 = L.mpjx_allreduce(c.handle, s.data_ptr(), d.data_ptr(), 16, 8, 3, 0, None)
msg2 = L.mpjx_last_error().decode()
print(rc, w, rc2)
print(msg)
print(msg2)
L.mpjx_comm_destroy(c.handle)
torch.cuda.synchronize()
print("done")
'''
    import os

    env = dict(os.environ, MPJX_P1_EXCHANGE="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "done" in r.stdout, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    i = next(k for k, ln in enumerate(lines) if ln.replace("-", "").replace(" ", "").isdigit())
    rc, w, rc2 = map(int, lines[i].split())
    assert rc == 0 and w == -4 and "MPJX_RCCL_TIMEOUT_S" in lines[i + 1], r.stdout
    assert rc2 == -4 and "aborted" in lines[i + 2], r.stdout

def test_host_pipeline_multichunk():
    """Host-resident Allreduce / Reduce / Scan large enough to be chunk-pipelined (16 MiB chunks,
    ragged last chunk) in multicore mode, bit-exact vs the oracle."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    P, n = 3, 5 * (1 << 20) + 12345  # ~40 MiB of doubles -> 3 chunks
    sends = [make_input(O.DOUBLE, n, 900 + r, specials=False) for r in range(P)]
    exp_ar = O.allreduce(sends, n, O.DOUBLE, O.SUM)
    exp_sc = O.scan(sends, n, O.DOUBLE, O.SUM)
    exp_rd = O.reduce(sends, n, O.DOUBLE, O.MAX, 1)[1]
    comms = _world(P)

    def body(c):
        r = c.Rank()
        a, b, d = np.zeros(n), np.zeros(n), np.zeros(n)
        c.Allreduce(sends[r], 0, a, 0, n, MPI.DOUBLE, MPI.SUM)
        c.Scan(sends[r], 0, b, 0, n, MPI.DOUBLE, MPI.SUM)
        c.Reduce(sends[r], 0, d, 0, n, MPI.DOUBLE, MPI.MAX, 1)
        return a, b, d

    try:
        out = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    for r in range(P):
        assert np.array_equal(out[r][0].view(np.uint64), exp_ar[r].view(np.uint64))
        assert np.array_equal(out[r][1].view(np.uint64), exp_sc[r].view(np.uint64))
    assert np.array_equal(out[1][2].view(np.uint64), exp_rd.view(np.uint64))


@pytest.mark.parametrize("mix", ["all_direct", "mixed", "direct_off", "chunk_edge", "once_on", "mixed_rank0_staged"])
def test_host_direct_form_multicore(mix, monkeypatch):
    """The *_host calls' host-direct form (round 5): multicore mode, every rank on one device, a call of
    one host-pipeline chunk, page-locked buffers from mpjx_host_alloc — the P-way kernel reads and writes
    the host buffers itself (no staging). `mixed`: ranks 1 and 3 pass pageable arrays (staged) while
    ranks 0 and 2 go direct, in the same collective calls; `direct_off`: MPJX_HOST_DIRECT=0; `chunk_edge`:
    mixed, with 1 MiB host chunks, at exactly one chunk (direct) and one element more (every rank
    pipelines: two chunks). Allreduce, Reduce (root 3, and a faithful Reduce writing every rank's
    recvbuf), Scan and a ragged Reduce_scatter, at 1001 elements and 1 MiB, all bit-exact vs the oracle.
    The form each rank took is read back (mpjx_comm_last_host_form). `once_on`: MPJX_HOST_ONCE=1, the
    host-direct Allreduce writes its result across the link once (into the first
    host-direct rank's recvbuf; the others copy it host-to-host inside the call; off by default, slower
    per call); `mixed_rank0_staged`: odd ranks direct, so the launching rank 0 is staged."""
    import ctypes

    from mpjexpress_amd import _lib, mpi
    from mpjexpress_amd.mpi import MPI

    if mix == "direct_off":
        monkeypatch.setenv("MPJX_HOST_DIRECT", "0")
    if mix == "once_on":
        monkeypatch.setenv("MPJX_HOST_ONCE", "1")
    sizes = (1001, (1 << 20) // 8)
    if mix == "chunk_edge":
        monkeypatch.setenv("MPJX_HOST_CHUNK_MIB", "1")
        sizes = ((1 << 20) // 8, (1 << 20) // 8 + 1)
    L = _lib.lib()
    P = 4
    keep = []

    def pinned(a):
        p = ctypes.c_void_p()
        _lib.check(L.mpjx_host_alloc(ctypes.byref(p), a.nbytes), "mpjx_host_alloc")
        keep.append(p)
        v = np.frombuffer((ctypes.c_uint8 * a.nbytes).from_address(p.value), dtype=a.dtype, count=a.size)
        v[:] = a
        return v

    comms = _world(P)
    try:
        for n in sizes:
            sends = [make_input(O.DOUBLE, n, 2100 + r + n, specials=False) for r in range(P)]
            rc = [n // 7, n // 3, 0, n - n // 7 - n // 3]
            exp_ar = O.allreduce(sends, n, O.DOUBLE, O.SUM)
            exp_sc = O.scan(sends, n, O.DOUBLE, O.SUM)
            exp_rd = O.reduce(sends, n, O.DOUBLE, O.SUM, 3)[3]
            exp_fr = O.reduce(sends, n, O.DOUBLE, O.SUM, 0, flags=O.FLAG_FAITHFUL)
            exp_rs, _ = O.reduce_scatter(sends, rc, O.DOUBLE, O.MIN)

            def body(c):
                r = c.Rank()
                direct = (r % 2 == 1) if mix == "mixed_rank0_staged" else (
                    mix not in ("mixed", "chunk_edge") or r % 2 == 0)

                def buf(a):
                    return pinned(a) if direct else a.copy()
                s = buf(sends[r])
                a, b, d, f = buf(np.zeros(n)), buf(np.zeros(n)), buf(np.zeros(n)), buf(np.zeros(n))
                e = buf(np.zeros(max(1, rc[r])))
                c.Allreduce(s, 0, a, 0, n, MPI.DOUBLE, MPI.SUM)
                form = ctypes.c_int()
                _lib.check(L.mpjx_comm_last_host_form(c.handle, ctypes.byref(form)), "host_form")
                one_chunk = n * 8 <= (1 << 20) or mix != "chunk_edge"
                want = 2 if direct and mix != "direct_off" and one_chunk else 1
                assert form.value == want, (mix, n, r, form.value, want)
                c.Scan(s, 0, b, 0, n, MPI.DOUBLE, MPI.SUM)
                c.Reduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM, 3)
                c.faithful = True
                c.Reduce(s, 0, f, 0, n, MPI.DOUBLE, MPI.SUM, 0)
                c.faithful = False
                c.Reduce_scatter(s, 0, e, 0, rc, MPI.DOUBLE, MPI.MIN)
                return a.copy(), b.copy(), d.copy(), f.copy(), e[:rc[r]].copy()

            out = mpi.run_multicore(comms, body)
            for r in range(P):
                assert np.array_equal(out[r][0].view(np.uint64), exp_ar[r].view(np.uint64)), (mix, n, r, "ar")
                assert np.array_equal(out[r][1].view(np.uint64), exp_sc[r].view(np.uint64)), (mix, n, r, "scan")
                assert np.array_equal(out[r][3].view(np.uint64), exp_fr[r].view(np.uint64)), (mix, n, r, "faithful")
                assert np.array_equal(out[r][4].view(np.uint64), exp_rs[r].view(np.uint64)), (mix, n, r, "rs")
            assert np.array_equal(out[3][2].view(np.uint64), exp_rd.view(np.uint64)), (mix, n, "reduce")
    finally:
        _free(comms)
        for p in keep:
            L.mpjx_host_free(p)


def _straddling_range(keep, nbytes):
    """A host range [p, p + nbytes) that starts in one page-locked, identity-mapped allocation, runs through
    PAGEABLE memory and ends in another page-locked allocation: three MiB of one anonymous mapping with the
    first and last MiB registered separately (hipHostRegister), p half a MiB into the first. Its first and
    last bytes are both page-locked at the same device address — what round 5's check sampled — but its
    middle is not mapped for the device: a kernel storing there faults. (Two mpjx_host_alloc blocks are
    never adjacent: hipHostMalloc leaves at least 1 MiB unmapped between them, profiles/r06/probe_host_f.jsonl,
    so a range spanning two of them holds unmapped bytes and is no buffer at all.) Returns p, or None when
    the runtime does not report the registered extents as the probe saw them (then nothing is launched)."""
    import ctypes
    import mmap

    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipPointerGetAttribute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    hip.hipGetLastError.restype = ctypes.c_int
    mib = 1 << 20
    assert nbytes <= 2 * mib
    m = mmap.mmap(-1, 3 * mib)
    base = ctypes.addressof(ctypes.c_char.from_buffer(m))
    regs = []
    for h in (base, base + 2 * mib):
        if hip.hipHostRegister(ctypes.c_void_p(h), mib, 0) != 0:
            break
        regs.append(h)
    keep.append(("unregister", hip, regs, m))
    if len(regs) != 2:
        return None
    RANGE_START, RANGE_SIZE = 11, 12  # HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, _RANGE_SIZE (driver_types.h)

    def extent(p):
        st, sz = ctypes.c_void_p(), ctypes.c_size_t()
        ok = hip.hipPointerGetAttribute(ctypes.byref(st), RANGE_START, ctypes.c_void_p(p)) == 0 and \
            hip.hipPointerGetAttribute(ctypes.byref(sz), RANGE_SIZE, ctypes.c_void_p(p)) == 0
        hip.hipGetLastError()
        return (st.value, sz.value) if ok else None
    if extent(base + mib // 2) != (base, mib) or extent(base + 2 * mib) != (base + 2 * mib, mib) or \
            extent(base + mib + 4096) is not None:
        return None
    return base + mib - nbytes // 2


def test_host_direct_range_spanning_two_allocations():
    """the host-direct form's range check covers the WHOLE range. A rank's recvbuf (in the
    Allreduce) and sendbuf (in the Scan) that start in one page-locked registration, cross pageable memory
    and end in another pass a first-and-last-byte check, but are not one allocation: libmpjx must take the
    staged form for that rank (never launch a kernel on the range — its middle is not mapped for the device)
    and stay bit-exact, its host copies split at the allocation boundaries (host_copy), while the other
    ranks keep the host-direct form in the same calls."""
    import ctypes

    from mpjexpress_amd import _lib
    from mpjexpress_amd.mpi import MPI

    L = _lib.lib()
    P, n = 4, (1 << 20) // 8 + 4099  # 1 MiB + 32 KiB: crosses the pageable middle MiB at both ends
    keep = []
    comms = _world(P)
    try:
        rspan, sspan = _straddling_range(keep, n * 8), _straddling_range(keep, n * 8)
        if rspan is None or sspan is None:
            pytest.skip("the runtime does not report registered extents as probe_host saw them: nothing launched")
        sends = [make_input(O.DOUBLE, n, 4100 + r, specials=False) for r in range(P)]
        exp_ar = O.allreduce(sends, n, O.DOUBLE, O.SUM)
        exp_sc = O.scan(sends, n, O.DOUBLE, O.MAX)

        def pinned(a):
            p = ctypes.c_void_p()
            _lib.check(L.mpjx_host_alloc(ctypes.byref(p), a.nbytes), "mpjx_host_alloc")
            keep.append(p)
            v = np.frombuffer((ctypes.c_uint8 * a.nbytes).from_address(p.value), dtype=a.dtype, count=a.size)
            v[:] = a
            return v

        def at(addr):
            return np.frombuffer((ctypes.c_uint8 * (n * 8)).from_address(addr), dtype=np.float64, count=n)

        def body(c):
            r = c.Rank()
            s, out = pinned(sends[r]), pinned(np.zeros(n))
            forms = []
            try:
                for call in ("ar", "scan"):
                    if r == 0 and call == "ar":
                        s_, o_ = s, at(rspan)  # recvbuf straddles
                    elif r == 0:
                        s_, o_ = at(sspan), out  # sendbuf straddles
                        s_[:] = sends[0]
                    else:
                        s_, o_ = s, out
                    o_[:] = -7.0
                    if call == "ar":
                        c.Allreduce(s_, 0, o_, 0, n, MPI.DOUBLE, MPI.SUM)
                    else:
                        c.Scan(s_, 0, o_, 0, n, MPI.DOUBLE, MPI.MAX)
                    f = ctypes.c_int()
                    _lib.check(L.mpjx_comm_last_host_form(c.handle, ctypes.byref(f)), "host_form")
                    forms.append((f.value, o_.copy()))
            except BaseException:
                # a rank whose call failed after the collective leaves its peers waiting in the next one:
                # a call with bad arguments marks the world failed, so they fail instead of hanging
                L.mpjx_allreduce(c.handle, None, None, 1, 8, 3, 0, None)
                raise
            return forms

        out = mpi_run(comms, body)
        for r in range(P):
            (fa, ra), (fs, rs) = out[r]
            want = 1 if r == 0 else 2
            assert fa == want and fs == want, (r, fa, fs)
            assert np.array_equal(ra.view(np.uint64), exp_ar[r].view(np.uint64)), (r, "allreduce")
            assert np.array_equal(rs.view(np.uint64), exp_sc[r].view(np.uint64)), (r, "scan")
    finally:
        _free(comms)
        for k in keep:
            if isinstance(k, tuple):
                _, hip, regs, m = k
                for h in regs:
                    hip.hipHostUnregister(ctypes.c_void_p(h))
            else:
                L.mpjx_host_free(k)


def mpi_run(comms, body):
    from mpjexpress_amd import mpi

    return mpi.run_multicore(comms, body)


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("mem", ["pageable", "pinned", "pinned_in", "registered", "inplace"])
def test_host_pipeline_pinned_and_pageable(P, mem, monkeypatch):
    """The host pipeline's two drain paths: a page-locked destination copied back from the issuing
    thread, a pageable one by the drain thread; page-locked (hipHostMalloc'd by torch, or caller memory
    hipHostRegister'ed) and pageable sources; pageable in-place (send == recv). 1 MiB chunks over a
    ragged ~9.5 MiB vector (10 chunks, a short last one). Bit-exact vs the oracle."""
    import torch

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    monkeypatch.setenv("MPJX_HOST_CHUNK_MIB", "1")
    n = (19 << 19) // 8 + 1001
    sends = [make_input(O.DOUBLE, n, 1300 + r, specials=False) for r in range(P)]
    exp_ar = O.allreduce(sends, n, O.DOUBLE, O.SUM)
    exp_sc = O.scan(sends, n, O.DOUBLE, O.SUM)
    exp_rd = O.reduce(sends, n, O.DOUBLE, O.MAX, P - 1)[P - 1]
    comms = _world(P)

    registered = []

    def host(a, pinned):
        if not pinned:
            return a.copy()
        if mem == "registered":  # the caller's own memory, page-locked with hipHostRegister
            b = a.copy()
            assert torch._C._cudart.cudaHostRegister(b.ctypes.data, b.nbytes, 0) == 0
            registered.append(b)
            return b
        t = torch.from_numpy(a).pin_memory()  # page-locked: the direct path
        return t.numpy()

    def body(c):
        r = c.Rank()
        pin_in = mem in ("pinned", "pinned_in", "registered")
        pin_out = mem in ("pinned", "registered")
        outs = []
        for call in ("ar", "sc", "rd"):
            s = host(sends[r], pin_in)
            d = s if mem == "inplace" else host(np.zeros(n), pin_out)
            if call == "ar":
                c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
            elif call == "sc":
                c.Scan(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
            else:
                c.Reduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.MAX, P - 1)
            outs.append(d.copy())
        return outs

    try:
        out = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
        for b in registered:
            torch._C._cudart.cudaHostUnregister(b.ctypes.data)
    for r in range(P):
        assert np.array_equal(out[r][0].view(np.uint64), exp_ar[r].view(np.uint64)), (r, mem)
        assert np.array_equal(out[r][1].view(np.uint64), exp_sc[r].view(np.uint64)), (r, mem)
    assert np.array_equal(out[P - 1][2].view(np.uint64), exp_rd.view(np.uint64)), mem


@pytest.mark.parametrize("P", [2, 3, 8])
def test_pipelined_allreduce_chunks(P, monkeypatch):
    """Chunked Allreduce (combine of chunk k on a second stream, overlapping chunk k+1's exchange):
    1 MiB chunks over a ragged ~9 MiB vector, out-of-place and in-place, bit-exact vs the oracle."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    monkeypatch.setenv("MPJX_PIPE_CHUNK_MIB", "1")
    monkeypatch.setenv("MPJX_SMP_COPY", "1")  # the exchange-based engine (multicore otherwise goes direct)
    n = (9 << 20) // 8 + 333
    for op, t, dt in [(O.SUM, O.DOUBLE, MPI.DOUBLE), (O.MAX, O.FLOAT, MPI.FLOAT)]:
        sends = [make_input(t, n, 4242 + r, specials=(t == O.FLOAT)) for r in range(P)]
        exp = O.allreduce(sends, n, t, op)
        comms = _world(P)

        def body(c):
            r = c.Rank()
            s = _t(sends[r])
            d = _t(np.zeros_like(sends[r]))
            c.Allreduce(s, 0, d, 0, n, dt, mpi.OPS[op - 1])
            c.Allreduce(s, 0, s, 0, n, dt, mpi.OPS[op - 1])  # in place
            return d.cpu().numpy(), s.cpu().numpy()

        try:
            out = mpi.run_multicore(comms, body)
        finally:
            _free(comms)
        for r in range(P):
            assert same_bits(t, op, out[r][0], exp[r]), (P, op, r)
            assert same_bits(t, op, out[r][1], exp[r]), (P, op, r, "in-place")


@pytest.mark.parametrize("engine", ["direct", "exchange", "pipelined"])
def test_config3_allreduce_sum_double_256mib_p8(engine, monkeypatch):
    """BASELINE configs[2] at full size on one GPU: Allreduce SUM double, 256 MiB per rank, 8 ranks
    (multicore), SURVEY 8(d) splitmix64 inputs; the direct engine, the exchange engine's plan on device
    copies (MPJX_SMP_COPY=1: the RCCL engine's exchange -> combine -> all-gather with SmpTransport as the
    transport — RcclTransport's own P > 1 calls run only on a multi-GPU node: tools/rccl_preflight and
    bench.py) and its 64 MiB chunk pipeline. Bit-exact against the oracle's MST(0) order on every rank."""
    import sys

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import synth

    if engine != "direct":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
        monkeypatch.setenv("MPJX_PIPE_CHUNK_MIB", "64" if engine == "pipelined" else "0")
    P, n = 8, (256 << 20) // 8
    sends = [synth.uniform_np(np.arange(n), synth.seed(3, r)) for r in range(P)]
    exp = O.allreduce(sends, n, O.DOUBLE, O.SUM)[0]
    comms = _world(P)

    def body(c):
        s = _t(sends[c.Rank()])
        d = torch_empty_like(s)
        c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
        return d.cpu().numpy()

    try:
        out = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    for r in range(P):
        assert np.array_equal(out[r].view(np.uint64), exp.view(np.uint64)), r


def torch_empty_like(t):
    import torch

    return torch.empty_like(t)


@pytest.mark.parametrize("engine", ["direct", "exchange", "pipelined"])
def test_config5_allreduce_max_float_1gib_p8(engine, monkeypatch):
    """BASELINE configs[4] at full size on one GPU: Allreduce MAX float, 1 GiB per rank, 8 ranks
    (multicore) — the direct engine, the exchange engine's plan on device copies (MPJX_SMP_COPY=1; not
    RcclTransport, whose P > 1 calls only a multi-GPU node runs) and its 64 MiB chunk pipeline. Checked bit-exactly against the oracle's MST order."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    if engine != "direct":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
        monkeypatch.setenv("MPJX_PIPE_CHUNK_MIB", "64" if engine == "pipelined" else "0")

    P, n = 8, (1 << 30) // 4
    rng = [np.random.default_rng(0x4D504A00 + 4000 + r) for r in range(P)]
    sends = [r.uniform(-1e3, 1e3, n).astype(np.float32) for r in rng]
    for r in range(P):  # edge values: NaN, +-0, +-inf, subnormals at fixed spots
        sends[r][r * 7:r * 7 + 6] = np.array([np.nan, 0.0, -0.0, np.inf, -np.inf, 1e-45], np.float32)
    exp = O.allreduce(sends, n, O.FLOAT, O.MAX)[0]
    comms = _world(P)

    def body(c):
        s = _t(sends[c.Rank()])
        c.Allreduce(s, 0, s, 0, n, MPI.FLOAT, MPI.MAX)
        return s.cpu().numpy()

    try:
        out = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    for r in range(P):
        assert np.array_equal(out[r].view(np.uint32), exp.view(np.uint32)), r


LOC = O.loc_pairs()


@pytest.mark.parametrize("P", PS)
@pytest.mark.parametrize("op,type_", LOC)
def test_maxloc_minloc_collectives(P, op, type_):
    """MAXLOC / MINLOC (src/mpi/Maxloc.java, Minloc.java) on SHORT2..DOUBLE2 through every collective,
    inputs with frequent value ties (index rule) and NaN/+-0/+-inf values for the float pairs."""
    for kind in ("allreduce", "scan"):
        got, exp = run(kind, P, op, type_, n=1500)
        _assert(kind, got, exp, op, type_)
    got, exp = run("reduce", P, op, type_, n=700, root=P - 1)
    _assert("reduce", got, exp, op, type_, only=P - 1)
    got, exp = run("reduce_scatter", P, op, type_, recvcounts=[33 + 7 * j for j in range(P)])
    _assert("reduce_scatter", got, exp, op, type_)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_ccl_allreduce_maxminloc_kat(P):
    """test/mpi/ccl/allreduce_maxminloc.java: in = (rank+i, rank); MAXLOC -> (size-1+i, size-1),
    MINLOC -> (i, 0) for INT2, LONG2, SHORT2, FLOAT2, DOUBLE2."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    comms = _world(P)
    count = 10

    def body(c):
        rank, size = c.Rank(), c.Size()
        for dt in (MPI.INT2, MPI.LONG2, MPI.SHORT2, MPI.FLOAT2, MPI.DOUBLE2):
            inp = np.zeros(2 * count, dt.np_dtype)
            inp[0::2] = rank + np.arange(count)
            inp[1::2] = rank
            for op, sol_v, sol_l in ((MPI.MAXLOC, size - 1 + np.arange(count), size - 1),
                                     (MPI.MINLOC, np.arange(count), 0)):
                out = np.zeros(2 * count, dt.np_dtype)
                out[1::2] = -1
                d_in, d_out = _t(inp), _t(out)
                c.Allreduce(d_in, 0, d_out, 0, count, dt, op)
                o = d_out.cpu().numpy()
                assert np.array_equal(o[0::2], sol_v.astype(dt.np_dtype)), (dt, op)
                assert (o[1::2] == sol_l).all(), (dt, op)
                h = out.copy()
                c.Allreduce(inp, 0, h, 0, count, dt, op)  # host-resident (Java array) path
                assert np.array_equal(h, o)

    try:
        mpi.run_multicore(comms, body)
    finally:
        _free(comms)


@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_big_endian_mpjbuf_payloads(P):
    """MPJX_FLAG_SEND/RECV_BIG_ENDIAN: reduce mpjbuf (network byte order) payloads directly, device
    and host-resident, for every element width, against the oracle on the native values."""
    import ctypes

    import torch

    from mpjexpress_amd import _lib, mpi

    L = _lib.lib()
    SBE, RBE = 0x4, 0x8
    cases = [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.BXOR, O.INT), (O.SUM, O.CHAR), (O.MIN, O.SHORT),
             (O.PROD, O.LONG), (O.LXOR, O.BOOLEAN), (O.MAXLOC, O.INT2)]
    n = 3001
    for op, t in cases:
        sends = [make_input(t, n, 55 + 3 * r, op=op) for r in range(P)]
        exp = O.allreduce(sends, n, t, op)
        be = [s.byteswap() if not s.dtype.names else s.view(s.dtype[0]).byteswap().view(s.dtype) for s in sends]
        comms = _world(P)

        def body(c):
            r = c.Rank()
            s = _t(be[r])
            d = _t(np.zeros_like(be[r]))
            torch.cuda.synchronize()
            _lib.check(L.mpjx_allreduce(c.handle, s.data_ptr(), d.data_ptr(), n, t, op, SBE | RBE, None), "ar")
            _lib.check(L.mpjx_comm_synchronize(c.handle), "sync")
            dev_be = _np(d, be[r])
            h = np.zeros_like(sends[r])
            _lib.check(L.mpjx_allreduce_host(c.handle, be[r].ctypes.data, h.ctypes.data, n, t, op, SBE), "arh")
            return dev_be, h

        try:
            out = mpi.run_multicore(comms, body)
        finally:
            _free(comms)
        for r in range(P):
            dev_native = out[r][0].byteswap() if not out[r][0].dtype.names else \
                out[r][0].view(out[r][0].dtype[0]).byteswap().view(out[r][0].dtype)
            assert same_bits(t, op, dev_native, exp[r]), (op, t, r, "device BE->BE")
            assert same_bits(t, op, out[r][1], exp[r]), (op, t, r, "host BE->native")


def _bswap(a):
    """Byte-swap every base word (pair records: each of their two words)."""
    return a.byteswap() if not a.dtype.names else a.view(a.dtype[0]).byteswap().view(a.dtype)


BE_CASES = [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.BXOR, O.INT), (O.SUM, O.CHAR), (O.PROD, O.LONG),
            (O.BAND, O.SHORT), (O.LOR, O.BOOLEAN), (O.MINLOC, O.DOUBLE2), (O.MAXLOC, O.SHORT2)]


@pytest.mark.parametrize("engine", ["direct", "exchange", "oneshot"])
@pytest.mark.parametrize("flags", [0x4, 0x8, 0xC])
@pytest.mark.parametrize("P", [1, 3, 9])
def test_big_endian_fused_collectives(P, flags, engine, monkeypatch):
    """Big-endian (mpjbuf) operands and results are swapped inside the combine kernels (§8 f4): every
    collective, every flag combination (send BE only, recv BE only, both), each multicore engine
    (direct, two exchanges, one-shot all-gather), P = 9 (compositions through native temporaries),
    old-collectives orders, ragged Reduce_scatter and a misaligned (one element per lane) buffer —
    bit-exact against the oracle on the native values."""
    import torch

    from mpjexpress_amd import _lib, mpi

    L = _lib.lib()
    SBE, RBE = bool(flags & 0x4), bool(flags & 0x8)
    monkeypatch.setenv("MPJX_SMP_COPY", "0" if engine == "direct" else "1")
    monkeypatch.setenv("MPJX_ONESHOT_KIB", "256" if engine == "oneshot" else "0")
    n = 3001
    rc = [(n // P) + (1 if r < n % P else 0) for r in range(P)]
    rc[-1] += rc[0]  # ragged
    rc[0] = 0
    for op, t in BE_CASES:
        for old in (False, True):
            oflag = O.FLAG_OLD if old else 0
            sends = [make_input(t, n, 77 + 5 * r + t, op=op) for r in range(P)]
            root = P - 1
            exp_ar = O.allreduce(sends, n, t, op, flags=oflag)
            exp_red = O.reduce(sends, n, t, op, root, flags=oflag)[root]
            exp_rs, _ = O.reduce_scatter(sends, rc, t, op, flags=oflag)
            exp_sc = O.scan(sends, n, t, op, flags=oflag)
            ins = [_bswap(s) if SBE else s for s in sends]
            comms = _world(P)

            def body(c):
                r = c.Rank()
                fl = flags | oflag
                s = _t(ins[r])
                base = _t(np.concatenate([ins[r][:1], ins[r]]))  # element 1 of it: misaligned copy
                mis = base[1:] if not ins[r].dtype.names else base[2:]
                outs = {}
                for name, src in (("ar", s), ("ar_mis", mis)):
                    d = _t(np.zeros_like(ins[r]))
                    _lib.check(L.mpjx_allreduce(c.handle, src.data_ptr(), d.data_ptr(), n, t, op, fl, None), name)
                    outs[name] = d
                d = _t(np.zeros_like(ins[r]))
                _lib.check(L.mpjx_reduce(c.handle, s.data_ptr(), d.data_ptr(), n, t, op, root, fl, None), "red")
                outs["red"] = d
                cnt = (ctypes.c_int64 * P)(*rc)
                d = _t(np.zeros(max(rc[r], 1), ins[r].dtype))
                _lib.check(L.mpjx_reduce_scatter(c.handle, s.data_ptr(), d.data_ptr(), cnt, t, op, fl, None), "rs")
                outs["rs"] = d
                d = _t(np.zeros_like(ins[r]))
                _lib.check(L.mpjx_scan(c.handle, s.data_ptr(), d.data_ptr(), n, t, op, fl, None), "scan")
                outs["scan"] = d
                _lib.check(L.mpjx_comm_synchronize(c.handle), "sync")
                return {k: _np(v, ins[r]) for k, v in outs.items()}

            try:
                out = mpi.run_multicore(comms, body)
            finally:
                _free(comms)

            def native(a):
                return _bswap(a) if RBE else a

            for r in range(P):
                tag = (op, t, r, old, engine)
                assert same_bits(t, op, native(out[r]["ar"]), exp_ar[r]), tag + ("allreduce",)
                assert same_bits(t, op, native(out[r]["ar_mis"]), exp_ar[r]), tag + ("allreduce misaligned",)
                if r == root:
                    assert same_bits(t, op, native(out[r]["red"]), exp_red), tag + ("reduce",)
                assert same_bits(t, op, native(out[r]["rs"][:rc[r]]), exp_rs[r]), tag + ("reduce_scatter",)
                assert same_bits(t, op, native(out[r]["scan"]), exp_sc[r]), tag + ("scan",)


def test_big_endian_combine_multi():
    """mpjx_combine_multi with MPJX_FLAG_SEND/RECV_BIG_ENDIAN: the big-endian combine of two
    mpjbuf payloads in one kernel (reads 2 S, writes S), FOLD / MST / SCAN orders, and P = 9
    (compositions through native temporaries)."""
    import torch

    from mpjexpress_amd import _lib

    L = _lib.lib()
    vp = ctypes.c_void_p
    for op, t in BE_CASES:
        for P, order in ((2, 0), (5, 1), (4, 2), (9, 0), (9, 1), (9, 2)):
            n = 40961
            xs = [make_input(t, n, 901 + p, op=op) for p in range(P)]
            ins = [_t(_bswap(x)) for x in xs]
            Q = P if order == 2 else 1
            outs = [_t(np.zeros_like(xs[0])) for _ in range(Q)]
            pin = (vp * P)(*[x.data_ptr() for x in ins])
            pout = (vp * Q)(*[o.data_ptr() for o in outs])
            _lib.check(L.mpjx_combine_multi(op, t, order, P, pin, pout, n, 0, 0xC, None), "combine_multi")
            torch.cuda.synchronize()
            if order == 0:  # FT_Reduce rooted at 0
                exp = [O.reduce(xs, n, t, op, 0, flags=O.FLAG_OLD)[0]]
            elif order == 1:  # MST_Reduce rooted at 0
                exp = [O.reduce(xs, n, t, op, 0)[0]]
            else:
                exp = O.scan(xs, n, t, op)
            for q in range(Q):
                got = _bswap(_np(outs[q], xs[0]))
                assert same_bits(t, op, got, exp[q]), (op, t, P, order, q)


def _mpjbuf_image(x, type_, splits=None, pad=0):
    """An mpjbuf static-buffer image of x: sections of (type code = base - 1, 3 pad bytes, big-endian
    int32 count, big-endian base words), each header at the next 8-byte boundary
    (src/mpjbuf/Buffer.java:609-704). `splits`: base-word counts of the sections (default one)."""
    base = O.PAIR_BASE.get(type_, type_)
    words = x.view(x.dtype[0]) if x.dtype.names else x
    splits = splits or [words.size]
    out = bytearray()
    k = 0
    for n in splits:
        out += bytes((8 - len(out) % 8) % 8)
        out += bytes([base - 1, 0, 0, 0]) + int(n).to_bytes(4, "big", signed=True)
        out += words[k:k + n].astype(words.dtype.newbyteorder(">")).tobytes()
        k += n
    out += bytes(pad)
    return np.frombuffer(bytes(out), np.uint8).copy()


def test_mpjbuf_combine_device_section_walk():
    """mpjx_mpjbuf_combine: acc = payload (op) acc with the mpjbuf sections walked by the kernel
    (§8 f4): one section (the 16-B streaming body, payload 16-, 8-, 4- and 1-byte aligned) and several
    (the per-element body; one splitting a MAXLOC pair), device memory, pinned host memory, every op
    family, against the oracle; malformed images (type code,
    count, overrun, > 64 sections) report their code and leave acc untouched."""
    import torch

    from mpjexpress_amd import _lib

    L = _lib.lib()
    n = 10007
    cases = [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.MIN, O.BYTE), (O.PROD, O.INT), (O.BXOR, O.LONG),
             (O.SUM, O.CHAR), (O.MAX, O.SHORT), (O.LAND, O.BOOLEAN), (O.MAXLOC, O.INT2), (O.MINLOC, O.DOUBLE2)]
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    for op, t in cases:
        acc0 = make_input(t, n, 11 + t, op=op)
        inp = make_input(t, n, 23 + t, op=op)
        exp = O.apply(op, t, acc0.copy(), inp)
        words = 2 * n if t in O.PAIR_BASE else n
        for where, splits in (("device", None), ("device", [3, words - 1003, 1000]), ("pinned", [words // 2 + 1, words - words // 2 - 1]),
                              ("misaligned", None), ("at+8", None), ("at+4", None)):
            img = _mpjbuf_image(inp, t, splits, pad=5)
            if where == "pinned":
                m = torch.from_numpy(img).pin_memory()
                mp = m.data_ptr()
            elif where == "misaligned" or where.startswith("at+"):
                k = 1 if where == "misaligned" else int(where[3:])  # +8: 16-B aligned payload; +4: 4-B
                m = torch.from_numpy(np.concatenate([np.zeros(k, np.uint8), img])).cuda()
                mp = m.data_ptr() + k
            else:
                m = torch.from_numpy(img).cuda()
                mp = m.data_ptr()
            a = _t(acc0.copy())
            st.zero_()
            _lib.check(L.mpjx_mpjbuf_combine(op, t, a.data_ptr(), mp, img.size, n, st.data_ptr(), 0, None), "mpjbuf")
            torch.cuda.synchronize()
            assert int(st.item()) == 0, (op, t, where)
            assert same_bits(t, op, _np(a, acc0), exp), (op, t, where, splits)
    # malformed images: code, acc untouched
    x = make_input(O.DOUBLE, 1000, 5)
    acc0 = make_input(O.DOUBLE, 1000, 6)
    good = _mpjbuf_image(x, O.DOUBLE)
    bad_type = good.copy()
    bad_type[0] = O.FLOAT - 1
    many = _mpjbuf_image(x, O.DOUBLE, [10] * 65 + [1000 - 650])
    for img, cnt, nbytes, code in ((bad_type, 1000, good.size, 1), (good, 999, good.size, 2),
                                   (good, 1000, good.size - 8, 3), (many, 1000, many.size, 4)):
        m = torch.from_numpy(img).cuda()
        a = _t(acc0.copy())
        st.zero_()
        _lib.check(L.mpjx_mpjbuf_combine(O.SUM, O.DOUBLE, a.data_ptr(), m.data_ptr(), nbytes, cnt, st.data_ptr(), 0,
                                         None), "mpjbuf bad")
        torch.cuda.synchronize()
        assert int(st.item()) == code, (code, int(st.item()))
        assert np.array_equal(a.cpu().numpy().view(np.uint64), acc0.view(np.uint64)), code


def test_mpjbuf_one_section_lane_realignment():
    """The one-section body realigns an 8-aligned payload across lanes (aligned 16-B loads + a lane
    shift; the last lane of a wave and of the vector load their second half themselves): vector counts
    that are a multiple of the wave, one more, one less, a partial wave, a single vector, and sub-vector
    tails, for a 2-, 4-, 8- and 16-element vector type, device and 16-B aligned payloads."""
    import torch

    from mpjexpress_amd import _lib

    L = _lib.lib()
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    for op, t in ((O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.SUM, O.SHORT), (O.BXOR, O.BYTE)):
        w = 16 // O.lib().ora_type_size(t)
        for nv, tail in ((3072, 0), (3073, 1), (3071, w - 1), (64, 0), (65, 0), (63, 0), (1, 0), (0, 1), (2047, 0)):
            n = nv * w + tail
            acc0 = make_input(t, n, 71 + n, op=op)
            inp = make_input(t, n, 73 + n, op=op)
            exp = O.apply(op, t, acc0.copy(), inp)
            img = _mpjbuf_image(inp, t, None, pad=5)
            for k in (0, 8):  # payload 8-B aligned (the realigned path) and 16-B aligned
                m = torch.from_numpy(np.concatenate([np.zeros(k, np.uint8), img])).cuda()
                a = _t(acc0.copy())
                st.zero_()
                _lib.check(L.mpjx_mpjbuf_combine(op, t, a.data_ptr(), m.data_ptr() + k, img.size, n, st.data_ptr(), 0,
                                                 None), "mpjbuf")
                torch.cuda.synchronize()
                assert int(st.item()) == 0, (op, t, nv, tail, k)
                assert same_bits(t, op, _np(a, acc0), exp), (op, t, nv, tail, k)


def test_split_create_subcommunicators():
    """Sub-communicators stay on the GPU strategy (NativeIntracomm.java:160-215 re-wraps Split/Create
    results; HipIntracomm and this mirror do too): every rank thread forms its sub-world itself
    (mpjx_comm_init_smp_rank, keyed by an id rank 0 broadcasts), worlds of different colors coexist,
    Split orders by key, nested Split and Create work, and each sub-communicator's Allreduce /
    Reduce_scatter / Scan match the oracle over its members' inputs."""
    import torch

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    P, n = 6, 5003
    sends = [make_input(O.DOUBLE, n, 4242 + r, op=O.SUM) for r in range(P)]
    comms = _world(P)

    def body(c):
        r = c.Rank()
        out = {}
        half = c.Split(r % 2, -r)  # evens and odds, each in descending parent rank
        out["half_rank"], out["half_size"] = half.Rank(), half.Size()
        s = _t(sends[r])
        d = torch.zeros_like(s)
        half.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
        out["half_ar"] = d.cpu().numpy()
        d = torch.zeros_like(s)
        half.Scan(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
        out["half_scan"] = d.cpu().numpy()
        pair = half.Split(half.Rank() // 2, half.Rank())  # nested
        d = torch.zeros_like(s)
        pair.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.MAX)
        out["pair_ar"], out["pair_size"] = d.cpu().numpy(), pair.Size()
        sub = c.Create([4, 1, 2])
        if sub is not None:
            rc = [1000, 2003, 2000]
            d = torch.zeros(rc[sub.Rank()], dtype=torch.float64, device=s.device)
            sub.Reduce_scatter(s, 0, d, 0, rc, MPI.DOUBLE, MPI.SUM)
            out["sub_rs"], out["sub_rank"] = d.cpu().numpy(), sub.Rank()
            sub.Free()
        none = c.Split(-1 if r == 0 else 7, 0)
        out["undefined"] = none is None
        if none is not None:
            none.Free()
        pair.Free()
        half.Free()
        return out

    try:
        got = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    for color in (0, 1):
        members = sorted((q for q in range(P) if q % 2 == color), key=lambda q: -q)
        xs = [sends[q] for q in members]
        ar = O.allreduce(xs, n, O.DOUBLE, O.SUM)
        sc = O.scan(xs, n, O.DOUBLE, O.SUM)
        for i, q in enumerate(members):
            assert got[q]["half_rank"] == i and got[q]["half_size"] == len(members)
            assert same_bits(O.DOUBLE, O.SUM, got[q]["half_ar"], ar[i]), ("split allreduce", q)
            assert same_bits(O.DOUBLE, O.SUM, got[q]["half_scan"], sc[i]), ("split scan", q)
        for lo in range(0, len(members), 2):
            grp = members[lo:lo + 2]
            mx = O.allreduce([sends[q] for q in grp], n, O.DOUBLE, O.MAX)
            for i, q in enumerate(grp):
                assert got[q]["pair_size"] == len(grp)
                assert same_bits(O.DOUBLE, O.MAX, got[q]["pair_ar"], mx[i]), ("nested split", q)
    grp = [4, 1, 2]
    rs, _ = O.reduce_scatter([sends[q] for q in grp], [1000, 2003, 2000], O.DOUBLE, O.SUM)
    for i, q in enumerate(grp):
        assert got[q]["sub_rank"] == i
        assert same_bits(O.DOUBLE, O.SUM, got[q]["sub_rs"], rs[i]), ("create reduce_scatter", q)
    assert [got[q]["undefined"] for q in range(P)] == [True] + [False] * (P - 1)


def test_smp_rank_init_rejects_mismatches():
    """mpjx_comm_init_smp_rank: a rank taken twice, a world-size or a devices[] disagreement are
    errors; the world forms from threads arriving in any order."""
    import ctypes
    import os

    from mpjexpress_amd import _lib

    L = _lib.lib()
    uid = os.urandom(128)
    devs = (ctypes.c_int * 2)(0, 0)
    h1, h0, hx = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    assert L.mpjx_comm_init_smp_rank(ctypes.byref(h1), 2, uid, 1, devs) == 0
    assert L.mpjx_comm_init_smp_rank(ctypes.byref(hx), 2, uid, 1, devs) != 0  # rank 1 again
    assert L.mpjx_comm_init_smp_rank(ctypes.byref(hx), 3, uid, 0, devs) != 0  # other size
    assert L.mpjx_comm_init_smp_rank(ctypes.byref(hx), 2, uid, 0, (ctypes.c_int * 2)(0, 1)) != 0  # other devices
    assert L.mpjx_comm_init_smp_rank(ctypes.byref(h0), 2, uid, 0, devs) == 0
    r0, r1 = ctypes.c_int(), ctypes.c_int()
    L.mpjx_comm_rank(h0, ctypes.byref(r0))
    L.mpjx_comm_rank(h1, ctypes.byref(r1))
    assert (r0.value, r1.value) == (0, 1)
    assert L.mpjx_comm_destroy(h0) == 0 and L.mpjx_comm_destroy(h1) == 0


def test_config4_reduce_scatter_scan_int32_band_bxor_64mib_p8():
    """BASELINE configs[3] at full size on one GPU (8 multicore ranks): Reduce_scatter + Scan of
    64 MiB int32, BAND (bits set with p = 7/8) and BXOR (uniform), recvcounts 2,097,152 each;
    bit-exact vs the oracle, plus the size-independent BXOR checksum property."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    P, n = 8, (64 << 20) // 4
    rc = [n // P] * P
    for op, opx in ((O.BAND, MPI.BAND), (O.BXOR, MPI.BXOR)):
        sends = []
        for r in range(P):
            g = np.random.default_rng(0x4D504A00 + 3000 + r)
            if op == O.BAND:  # each bit set with p = 7/8
                bits = g.random((n, 32)) < 7 / 8
                x = np.packbits(bits, axis=1, bitorder="little").view(np.int32).ravel()
            else:
                x = g.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
            sends.append(x)
        exp_rs, _ = O.reduce_scatter(sends, rc, O.INT, op)
        exp_sc = O.scan(sends, n, O.INT, op)
        comms = _world(P)

        def body(c):
            r = c.Rank()
            s = _t(sends[r])
            out = _t(np.zeros(rc[r], np.int32))
            c.Reduce_scatter(s, 0, out, 0, rc, MPI.INT, opx)
            sc = _t(np.zeros(n, np.int32))
            c.Scan(s, 0, sc, 0, n, MPI.INT, opx)
            return out.cpu().numpy(), sc.cpu().numpy()

        try:
            out = mpi.run_multicore(comms, body)
        finally:
            _free(comms)
        for r in range(P):
            assert np.array_equal(out[r][0], exp_rs[r]), (op, r)
            assert np.array_equal(out[r][1], exp_sc[r]), (op, r)
        if op == O.BXOR:  # checksum of checksums: xor of all blocks == xor over ranks of full inputs
            tot = np.bitwise_xor.reduce(np.stack(sends), axis=0)
            assert np.array_equal(np.concatenate([o[0] for o in out]), tot)


@pytest.mark.parametrize("engine", ["direct", "exchange"])
def test_config4_big_endian_full_size(engine, monkeypatch):
    """configs[3]'s shape with mpjbuf (big-endian) payloads in and results out, at full size: 8
    multicore ranks x 64 MiB int32, Reduce_scatter BAND and Scan BXOR with MPJX_FLAG_SEND/RECV_
    BIG_ENDIAN — the register byte swap over 16.7 M elements per rank — bit-exact against the
    oracle on the native values, on the direct and the exchange engine."""
    import torch

    from mpjexpress_amd import _lib
    from mpjexpress_amd.mpi import run_multicore

    monkeypatch.setenv("MPJX_SMP_COPY", "0" if engine == "direct" else "1")
    L = _lib.lib()
    P, n = 8, (64 << 20) // 4
    rc = [n // P] * P
    g = [np.random.default_rng(0x4D504A00 + 3100 + r) for r in range(P)]
    sends = [x.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32) for x in g]
    exp_rs, _ = O.reduce_scatter(sends, rc, O.INT, O.BAND)
    exp_sc = O.scan(sends, n, O.INT, O.BXOR)
    comms = _world(P)

    def body(c):
        r = c.Rank()
        s = _t(sends[r].byteswap())
        out = torch.zeros(rc[r], dtype=torch.int32, device=s.device)
        sc = torch.zeros(n, dtype=torch.int32, device=s.device)
        cnt = (ctypes.c_int64 * P)(*rc)
        _lib.check(L.mpjx_reduce_scatter(c.handle, s.data_ptr(), out.data_ptr(), cnt, O.INT, O.BAND, 0xC, None), "rs")
        _lib.check(L.mpjx_scan(c.handle, s.data_ptr(), sc.data_ptr(), n, O.INT, O.BXOR, 0xC, None), "scan")
        _lib.check(L.mpjx_comm_synchronize(c.handle), "sync")
        return out.cpu().numpy().byteswap(), sc.cpu().numpy().byteswap()

    try:
        out = run_multicore(comms, body)
    finally:
        _free(comms)
    for r in range(P):
        assert np.array_equal(out[r][0], exp_rs[r]), ("reduce_scatter BAND BE", r)
        assert np.array_equal(out[r][1], exp_sc[r]), ("scan BXOR BE", r)


@pytest.mark.parametrize("P", [1, 2, 3, 5, 8])
def test_gather_scatter_bcast(P):
    """Gather / Scatter / Bcast device paths (src/mpi/PureIntracomm.java:592-1171) at every root:
    pure data movement, checked against the reference semantics (concatenation / blocks)."""
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    n = 1031
    xs = [make_input(O.LONG, n, 600 + r) for r in range(P)]
    for root in range(P):
        comms = _world(P)

        def body(c):
            r = c.Rank()
            s = _t(xs[r])
            g = _t(np.zeros(n * P, np.int64))
            c.Gather(s, 0, n, g, 0, n, MPI.LONG, root)
            allv = _t(np.concatenate(xs)) if r == root else _t(np.zeros(n * P, np.int64))
            sc = _t(np.zeros(n, np.int64))
            c.Scatter(allv, 0, n, sc, 0, n, MPI.LONG, root)
            b = _t(xs[r].copy())
            c.Bcast(b, 0, n, MPI.LONG, root)
            return g.cpu().numpy(), sc.cpu().numpy(), b.cpu().numpy()

        try:
            out = mpi.run_multicore(comms, body)
        finally:
            _free(comms)
        assert np.array_equal(out[root][0], np.concatenate(xs)), ("gather", root)
        for r in range(P):
            assert np.array_equal(out[r][1], xs[r]), ("scatter", root, r)
            assert np.array_equal(out[r][2], xs[root]), ("bcast", root, r)


def test_two_multicore_worlds_concurrently():
    """Two independent multicore communicators (3 ranks each) reducing at the same time from six
    threads: no state is shared between communicators (each has its own rendezvous, events and
    scratch), results bit-exact for both."""
    import threading

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    P, n = 3, 70001
    worlds = [_world(P), _world(P)]
    sends = [[make_input(O.DOUBLE, n, 4000 + 10 * w + r, specials=False) for r in range(P)] for w in range(2)]
    exps = [O.allreduce(sends[w], n, O.DOUBLE, O.SUM) for w in range(2)]
    outs = [[None] * P for _ in range(2)]
    errs = []

    def body(w, r):
        try:
            import torch

            torch.cuda.set_device(0)
            c = worlds[w][r]
            s = _t(sends[w][r])
            d = _t(np.zeros(n))
            for _ in range(20):
                c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
            outs[w][r] = d.cpu().numpy()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=body, args=(w, r)) for w in range(2) for r in range(P)]
    try:
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        for w in worlds:
            _free(w)
    assert not errs, errs[0]
    for w in range(2):
        for r in range(P):
            assert np.array_equal(outs[w][r].view(np.uint64), exps[w][r].view(np.uint64)), (w, r)


@pytest.mark.parametrize("how", ["host_array", "bad_root"])
@pytest.mark.parametrize("engine", ["direct", "exchange"])
def test_multicore_rank_with_bad_arguments_fails_every_rank(engine, how, monkeypatch):
    """One multicore rank hands a pageable host array to Allreduce (a rejected buffer), or passes a root
    out of range to Reduce (a plain argument error, before any rendezvous): it gets MPJX_ERR_ARG before any
    kernel, and the other ranks' matching calls fail instead of waiting for it forever — the world is
    marked failed (`ended` -> Transport::call_failed), so erroneous MPI programs cannot hang the JVM's
    rank threads — and every later call on every rank fails too."""
    import ctypes

    from mpjexpress_amd import _lib, mpi

    if engine == "exchange":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    P, n = 3, 4096
    comms = _world(P)
    host = np.zeros(n)
    rcs = [None] * P
    later = [None] * P
    L = _lib.lib()

    def body(c):
        r = c.Rank()
        d = _t(np.ones(n))
        o = _t(np.zeros(n))
        import torch

        torch.cuda.synchronize()
        sp, op_ = ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(o.data_ptr())
        if how == "host_array":
            send = ctypes.c_void_p(host.ctypes.data) if r == 1 else sp
            rcs[r] = L.mpjx_allreduce(c.handle, send, op_, n, 8, 3, 0, None)
        else:
            rcs[r] = L.mpjx_reduce(c.handle, sp, op_, n, 8, 3, P if r == 1 else 0, 0, None)
        L.mpjx_comm_synchronize(c.handle)
        later[r] = L.mpjx_allreduce(c.handle, sp, op_, n, 8, 3, 0x10, None)

    try:
        mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    assert rcs[1] == -1, rcs
    assert all(rc is not None and rc < 0 for rc in rcs), rcs
    assert all(rc is not None and rc < 0 for rc in later), later


def test_calls_on_different_streams_are_ordered():
    """Consecutive calls on one communicator are ordered even when they come on different streams
    (include/mpjx.h; the ordering event is recorded on the previous call's stream only when the
    stream changes): a chain send -> t1 (stream A) -> t2 (stream B) -> out (the communicator's own
    stream), 64 MiB per step so a missing wait would let a later copy read stale bytes."""
    import torch

    from mpjexpress_amd import _lib

    L = _lib.lib()
    c = _world(1)[0]
    try:
        n = 8 << 20
        send = torch.arange(n, dtype=torch.float64, device="cuda")
        for rep in range(3):
            t1, t2, out = (torch.full_like(send, -1.0) for _ in range(3))
            a, b = torch.cuda.Stream(), torch.cuda.Stream()
            torch.cuda.synchronize()
            _lib.check(L.mpjx_allreduce(c.handle, send.data_ptr(), t1.data_ptr(), n, 8, 3, 0, a.cuda_stream), "a")
            _lib.check(L.mpjx_allreduce(c.handle, t1.data_ptr(), t2.data_ptr(), n, 8, 3, 0, b.cuda_stream), "b")
            _lib.check(L.mpjx_allreduce(c.handle, t2.data_ptr(), out.data_ptr(), n, 8, 3, 0, None), "own")
            _lib.check(L.mpjx_comm_synchronize(c.handle), "sync")
            assert torch.equal(out, send), rep
    finally:
        c.Free()


# ---- JGF SparseMatmult: the reference-held double result on the Allreduce(DOUBLE, SUM) path ----

JGF_CASES = [(P, flags, where, "direct") for P in (1, 2, 3, 4, 8) for flags in (0, O.FLAG_OLD)
             for where in ("device", "host")] + [(8, 0, "device", "exchange"), (8, O.FLAG_OLD, "device", "exchange"),
                                                 (3, 0, "device", "exchange")]


@pytest.mark.parametrize("P,flags,where,engine", JGF_CASES,
                         ids=[f"P{p}-{'old' if f else 'mst'}-{w}-{e}" for p, f, w, e in JGF_CASES])
def test_jgf_sparsematmult_refval(P, flags, where, engine, monkeypatch):
    """test/jgf_mpj_benchmarks/section2/sparsematmult (size A): every rank runs SparseMatmult.java's
    loop — 200 reps of p_y[row[i]] += x[col[i]] * val[i] on its share (host, the oracle's restatement
    of the application) followed by Allreduce(p_y, 0, y, 0, M, DOUBLE, SUM) through libmpjx. Rank 0's
    ytotal must equal the oracle's bit for bit (same combine order) and lie within the reference's
    1e-12 of refval = 75.02484945753453 (JGFSparseMatmultBench.java:148-150); at P = 1 it IS refval."""
    import torch

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    if engine == "exchange":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    J = O.JgfSparse("A")
    M = J.M
    comms = _world(P)

    def body(c):
        r = c.Rank()
        p_y = np.zeros(M, np.float64)
        if where == "device":
            ps = torch.zeros(M, dtype=torch.float64, device="cuda")
            y = torch.zeros(M, dtype=torch.float64, device="cuda")
        else:
            y = np.zeros(M, np.float64)
        for _ in range(O.JGF_ITERS):
            J.rep(p_y, r, P)
            if where == "device":
                ps.copy_(torch.from_numpy(p_y))
                c.Allreduce(ps, 0, y, 0, M, MPI.DOUBLE, MPI.SUM)
            else:
                c.Allreduce(p_y, 0, y, 0, M, MPI.DOUBLE, MPI.SUM)
        return y.cpu().numpy() if where == "device" else y

    try:
        with old_collectives(bool(flags & O.FLAG_OLD)):
            got = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    exp_total, exp_y = O.jgf_sparse_matmult(P, flags=flags, return_y=True)
    for r in range(P):
        assert np.array_equal(got[r].view(np.uint64), exp_y[r].view(np.uint64)), r
    ytotal = J.ytotal(got[0])
    assert ytotal == exp_total
    assert abs(ytotal - O.JGF_REFVAL["A"]) <= 1e-12, ytotal
    if P == 1:
        assert ytotal == O.JGF_REFVAL["A"]


@pytest.mark.parametrize("flags", [0, O.FLAG_OLD])
def test_topo_map_reduce_kat(flags):
    """test/mpi/topo/map.java:63-79 on 8 ranks: sbuf[new_rank] = 1 (Cartcomm.Map returns the rank,
    src/mpi/Cartcomm.java:515), Reduce(INT, SUM, root 0), rbuf[i] == 1 for every i."""
    import torch

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    size = 8
    comms = _world(size)

    def body(c):
        sbuf = torch.zeros(size, dtype=torch.int32, device="cuda")
        sbuf[c.Rank()] = 1
        rbuf = torch.zeros(size, dtype=torch.int32, device="cuda")
        c.Reduce(sbuf, 0, rbuf, 0, size, MPI.INT, MPI.SUM, 0)
        return rbuf.cpu().tolist()

    try:
        with old_collectives(bool(flags & O.FLAG_OLD)):
            got = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    assert got[0] == [1] * size


FAITHFUL_CASES = [(O.SUM, O.DOUBLE), (O.PROD, O.INT), (O.MAX, O.FLOAT), (O.BAND, O.SHORT), (O.BXOR, O.LONG),
                  (O.MIN, O.CHAR), (O.LAND, O.BOOLEAN), (O.SUM, O.BYTE)]


@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("engine", ["direct", "exchange"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 8, 9])
def test_faithful_buffers_every_rank(P, engine, where, monkeypatch):
    """MPJX_FLAG_FAITHFUL leaves every buffer as the reference does, compared with the oracle's faithful
    mode element for element on EVERY rank (the per-flag table of include/mpjx.h MPJX_FLAG_FAITHFUL and
    INTEGRATION.md §1 "Buffers each call writes"):
    - mpjx_reduce, FAITHFUL: EVERY rank's recvbuf = its MST sub-tree partial, the reduction of the
      largest sub-tree it roots (PureIntracomm.java:1937-1939, 1966-1986); the root's is the result;
    - mpjx_reduce, FAITHFUL + OLD_COLLECTIVES: every non-root's recvbuf = a copy of its own sendbuf
      (:2038,2052);
    - mpjx_reduce_scatter, FAITHFUL, P >= 2, non-pair types: the caller's SENDBUF is overwritten
      (:2427-2428) — own block = the rank's result, every other element x = x (op) 0 folded P-1 times;
      with OLD_COLLECTIVES the sendbuf is left alone."""
    import torch

    from mpjexpress_amd import mpi

    if engine == "exchange":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    n, rc = 1000, [37 * (r % 3) + 40 for r in range(P)]  # ragged blocks, not 16-B multiples
    total = sum(rc)
    for ci, (op, type_) in enumerate(FAITHFUL_CASES):
        dt, opx = mpi.datatype(type_), mpi.OPS[op - 1]
        for flags in (O.FLAG_FAITHFUL, O.FLAG_FAITHFUL | O.FLAG_OLD):
            root = (ci + P // 2) % P
            sends = [make_input(type_, max(n, total), 101 * r + 7 * ci + flags, op=op) for r in range(P)]
            comms = _world(P, faithful=True)

            def body(c):
                r = c.Rank()
                sentinel = np.full(n, 0x5A, np.uint8).view(np.uint8)
                if where == "device":
                    s = _t(sends[r][:n].copy())
                    rv = torch.from_numpy(np.frombuffer(np.resize(sentinel, n * sends[r].itemsize).tobytes(),
                                                        sends[r].dtype).copy()).cuda()
                    c.Reduce(s, 0, rv, 0, n, dt, opx, root)
                    red = rv.cpu().numpy()
                    s2 = _t(sends[r][:total].copy())
                    out = _t(np.zeros(rc[r], sends[r].dtype))
                    c.Reduce_scatter(s2, 0, out, 0, rc, dt, opx)
                    return red, out.cpu().numpy(), s2.cpu().numpy()
                s = sends[r][:n].copy()
                rv = np.frombuffer(np.resize(sentinel, n * sends[r].itemsize).tobytes(), sends[r].dtype).copy()
                c.Reduce(s, 0, rv, 0, n, dt, opx, root)
                s2 = sends[r][:total].copy()
                out = np.zeros(rc[r], sends[r].dtype)
                c.Reduce_scatter(s2, 0, out, 0, rc, dt, opx)
                return rv, out, s2

            try:
                with old_collectives(bool(flags & O.FLAG_OLD)):
                    got = mpi.run_multicore(comms, body)
            finally:
                _free(comms)
            exp_red = O.reduce([x[:n] for x in sends], n, type_, op, root, flags=flags)
            old = bool(flags & O.FLAG_OLD)
            rs_counts = rc if not old else [rc[0]] * P  # FT_Scatter strides by recvcounts[0] (quirk)
            exp_rs, exp_send = O.reduce_scatter([x[:sum(rs_counts)] for x in sends], rs_counts, type_, op, flags=flags)
            ctx = f"{O.OP_NAMES[op]} {O.TYPE_NAMES[type_]} flags={flags} root={root}"
            for r in range(P):
                assert same_bits(type_, op, got[r][0], exp_red[r]), f"reduce recvbuf rank {r} {ctx}"
                if not old:
                    assert same_bits(type_, op, got[r][1], exp_rs[r]), f"reduce_scatter recv rank {r} {ctx}"
                    assert same_bits(type_, op, got[r][2], exp_send[r]), f"reduce_scatter sendbuf rank {r} {ctx}"
                else:  # FT_Reduce_scatter never writes sendbuf
                    assert same_bits(type_, op, got[r][2], sends[r][:total]), f"FT sendbuf rank {r} {ctx}"


@pytest.mark.parametrize("skew", [0, 4096])
@pytest.mark.parametrize("engine", ["direct", "exchange"])
@pytest.mark.parametrize("P", [3, 4, 8])
def test_faithful_reduce_in_place(P, engine, skew, monkeypatch):
    """Faithful MST Reduce with sendbuf == recvbuf on every rank: on the exchange engine with
    uneven blocks (or skewed input slots) rank r's own operand is read in place from its send, which
    is also where its sub-tree partial is stored — the partial must be computed after every other
    partial has read it. Every root, every rank's buffer against the oracle's faithful mode."""
    import torch

    from mpjexpress_amd import mpi

    if engine == "exchange":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    if skew:
        monkeypatch.setenv("MPJX_SLOT_SKEW", str(skew))
    n = 1000  # 1000 doubles over P ranks: blocks of 256-B multiples, the last one short
    for root in range(P):
        sends = [make_input(O.DOUBLE, n, 17 * r + root, op=O.SUM) for r in range(P)]
        comms = _world(P, faithful=True)

        def body(c):
            b = _t(sends[c.Rank()].copy())
            c.Reduce(b, 0, b, 0, n, mpi.MPI.DOUBLE, mpi.MPI.SUM, root)
            return b.cpu().numpy()

        try:
            got = mpi.run_multicore(comms, body)
        finally:
            _free(comms)
        exp = O.reduce(sends, n, O.DOUBLE, O.SUM, root, flags=O.FLAG_FAITHFUL)
        for r in range(P):
            assert same_bits(O.DOUBLE, O.SUM, got[r], exp[r]), f"rank {r} root {root}"
    del torch


def test_caller_stream_destroyed_between_calls():
    """A caller-supplied stream may be destroyed once the call returned and its work is done: the next
    call (on another stream) must not record the ordering event on the destroyed one. Each
    call runs on a fresh hipStreamCreate'd stream that is destroyed right after it; results stay exact."""
    import ctypes

    import torch

    from mpjexpress_amd import _lib

    hip = ctypes.CDLL("libamdhip64.so")
    L = _lib.lib()
    for P in (1, 2):
        comms = _world(P)
        try:
            n = 1 << 20
            send = torch.arange(n, dtype=torch.float64, device="cuda")
            outs = [torch.full_like(send, -1.0) for _ in range(P)]
            torch.cuda.synchronize()

            def body(c):
                r = c.Rank()
                for rep in range(4):
                    st = ctypes.c_void_p()
                    assert hip.hipStreamCreate(ctypes.byref(st)) == 0
                    _lib.check(L.mpjx_allreduce(c.handle, send.data_ptr(), outs[r].data_ptr(), n, 8, 3, 0, st), "ar")
                    assert hip.hipStreamSynchronize(st) == 0
                    assert hip.hipStreamDestroy(st) == 0
                _lib.check(L.mpjx_allreduce(c.handle, send.data_ptr(), outs[r].data_ptr(), n, 8, 3, 0, None), "own")
                _lib.check(L.mpjx_comm_synchronize(c.handle), "sync")

            from mpjexpress_amd import mpi

            mpi.run_multicore(comms, body)
            for r in range(P):
                assert torch.equal(outs[r], send * P), (P, r)
        finally:
            _free(comms)


@pytest.mark.parametrize("engine", ["direct", "exchange", "pipelined"])
def test_phase_timing(engine, monkeypatch):
    """mpjx_comm_phase_timing / mpjx_comm_last_phases (bench.py's N > 1 "phases"): an instrumented
    Allreduce reports its engine and non-negative phase times; results are unchanged by the events."""
    import ctypes

    import torch

    from mpjexpress_amd import _lib, mpi

    if engine != "direct":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    if engine == "pipelined":
        monkeypatch.setenv("MPJX_PIPE_CHUNK_MIB", "1")
    L = _lib.lib()
    P, n = 4, (4 << 20) // 8
    sends = [make_input(O.DOUBLE, n, 900 + r, specials=False) for r in range(P)]
    exp = O.allreduce(sends, n, O.DOUBLE, O.SUM)
    comms = _world(P)

    def body(c):
        s = _t(sends[c.Rank()])
        d = torch.empty_like(s)
        _lib.check(L.mpjx_comm_phase_timing(c.handle, 1), "on")
        _lib.check(L.mpjx_allreduce(c.handle, s.data_ptr(), d.data_ptr(), n, 8, 3, 0, None), "ar")
        ms, kind = (ctypes.c_float * 3)(), ctypes.c_int()
        _lib.check(L.mpjx_comm_last_phases(c.handle, ms, ctypes.byref(kind)), "phases")
        _lib.check(L.mpjx_comm_phase_timing(c.handle, 0), "off")
        _lib.check(L.mpjx_comm_synchronize(c.handle), "sync")
        return d.cpu().numpy(), kind.value, list(ms)

    try:
        got = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    want = {"direct": 2, "exchange": 1, "pipelined": 3}[engine]
    for r in range(P):
        out, kind, ms = got[r]
        assert np.array_equal(out.view(np.uint64), exp[r].view(np.uint64)), r
        assert kind == want, (r, kind)
        assert ms[0] >= 0 and (kind == 3 or (ms[1] >= 0 and ms[2] >= 0)), ms


@pytest.mark.parametrize("engine", ["direct", "exchange"])
def test_phase_timing_reduce_scatter_scan_oneshot(engine, monkeypatch):
    """Phase marks on Reduce_scatter and Scan (bench.py's configs[3] "phases") and on
    the one-shot path (engine 5); an instrumented call on a path without marks (Reduce) makes the next
    mpjx_comm_last_phases fail instead of returning the previous call's phases."""
    import ctypes

    import torch

    from mpjexpress_amd import _lib, mpi

    if engine == "exchange":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    L = _lib.lib()
    P, n = 4, (1 << 20) // 4
    rc = (ctypes.c_int64 * P)(*([n // P] * P))
    sends = [np.random.default_rng(70 + r).integers(-2**31, 2**31 - 1, n, dtype=np.int32) for r in range(P)]
    comms = _world(P)

    def phases(c):
        ms, kind = (ctypes.c_float * 3)(), ctypes.c_int()
        st = L.mpjx_comm_last_phases(c.handle, ms, ctypes.byref(kind))
        return st, kind.value, list(ms)

    def body(c):
        s = _t(sends[c.Rank()])
        d = torch.empty(n // P, dtype=torch.int32, device="cuda")
        z = torch.empty_like(s)
        _lib.check(L.mpjx_comm_phase_timing(c.handle, 1), "on")
        out = []
        _lib.check(L.mpjx_reduce_scatter(c.handle, s.data_ptr(), d.data_ptr(), rc, 5, 6, 0, None), "rs")
        out.append(phases(c))
        _lib.check(L.mpjx_scan(c.handle, s.data_ptr(), z.data_ptr(), n, 5, 10, 0, None), "scan")
        out.append(phases(c))
        _lib.check(L.mpjx_allreduce(c.handle, s.data_ptr(), z.data_ptr(), 1000, 5, 6, 0, None), "oneshot")
        out.append(phases(c))
        _lib.check(L.mpjx_reduce(c.handle, s.data_ptr(), z.data_ptr(), 1000, 5, 6, 0, 0, None), "reduce")
        out.append(phases(c))
        _lib.check(L.mpjx_comm_phase_timing(c.handle, 0), "off")
        _lib.check(L.mpjx_comm_synchronize(c.handle), "sync")
        return out, d.cpu().numpy()

    try:
        got = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    want = 2 if engine == "direct" else 1
    for r in range(P):
        (rs, sc, one, red), d = got[r]
        exp = np.bitwise_and.reduce(np.stack([x[r * (n // P):(r + 1) * (n // P)] for x in sends]), axis=0)
        assert np.array_equal(d, exp), r
        for st, kind, ms in (rs, sc):
            assert st == 0 and kind == want and min(ms) >= 0, (r, st, kind, ms)
        if engine == "exchange":  # the direct engine has no one-shot path
            assert one[0] == 0 and one[1] == 5 and min(one[2]) >= 0, one
        assert red[0] != 0 and red[1] == 0, red  # no stale phases


MD_CASES = [(P, flags, where) for P in (1, 2, 3, 4, 8) for flags in (0, O.FLAG_OLD) for where in ("device", "host")]


@pytest.mark.parametrize("P,flags,where", MD_CASES,
                         ids=[f"P{p}-{'old' if f else 'mst'}-{w}" for p, f, w in MD_CASES])
def test_jgf_moldyn_refval(P, flags, where):
    """test/jgf_mpj_benchmarks/section3/moldyn (size A): every rank runs md.runiters() — its cyclic share
    of the forces on the host (the oracle's restatement of the application), then the reference's six
    IN-PLACE Allreduce calls per move through libmpjx: x/y/z forces (DOUBLE, 2048), epot, vir (DOUBLE,
    1) and the interaction count (INT, 1, never reset: it wraps). After 50 moves rank 0's kinetic energy
    must equal the oracle's bit for bit (same combine orders) — at P = 1 that is refval =
    1731.4306625334357 itself (JGFMolDynBench.java:72) — and every rank's interaction count the oracle's."""
    import torch

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    comms = _world(P)

    def body(c):
        r = c.Rank()
        md = O.MolDyn("A")
        n = md.n
        for _ in range(md.moves):
            xf, yf, zf, ev, inter = md.step_forces(r, P)
            ep, vi = ev[:1].copy(), ev[1:].copy()
            bufs = [(xf, MPI.DOUBLE, n), (yf, MPI.DOUBLE, n), (zf, MPI.DOUBLE, n), (ep, MPI.DOUBLE, 1),
                    (vi, MPI.DOUBLE, 1), (inter, MPI.INT, 1)]
            for a, dt, cnt in bufs:  # md.java:248-264: Allreduce(buf, 0, buf, 0, ...) — in place
                if where == "device":
                    t = torch.from_numpy(a).cuda()
                    c.Allreduce(t, 0, t, 0, cnt, dt, MPI.SUM)
                    a[:] = t.cpu().numpy()
                else:
                    c.Allreduce(a, 0, a, 0, cnt, dt, MPI.SUM)
            md.step_finish(xf, yf, zf, np.array([ep[0], vi[0]]), inter)
        return md.ek, md.interactions

    try:
        with old_collectives(bool(flags & O.FLAG_OLD)):
            got = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    exp_ek, exp_inter = O.jgf_moldyn(P, flags=flags)
    assert got[0][0] == exp_ek, (got[0][0], exp_ek)
    assert [g[1] for g in got] == exp_inter
    if P == 1:
        assert got[0][0] == O.MD_REFVAL["A"]


RT_CASES = [(P, flags, where, eng) for P in (1, 2, 3, 4, 8) for flags in (0, O.FLAG_OLD, O.FLAG_FAITHFUL)
            for where in ("device", "host") for eng in ("direct", "exchange")]


@pytest.mark.parametrize("P,flags,where,engine", RT_CASES,
                         ids=[f"P{p}-{ {0: 'mst', O.FLAG_OLD: 'old', O.FLAG_FAITHFUL: 'faithful'}[f]}-{w}-{e}"
                              for p, f, w, e in RT_CASES])
def test_jgf_raytracer_reduce_refval(P, flags, where, engine, monkeypatch):
    """test/jgf_mpj_benchmarks/section3/raytracer (size A), the reference's only Reduce on DOUBLE with an
    exact reference-held result: every rank's partial pixel checksum (the oracle's restatement of the
    renderer, rows y = rank, rank + P, ...) goes through libmpjx's IN-PLACE Reduce(tmp, 0, tmp, 0, 1,
    DOUBLE, SUM, 0) (RayTracer.java:275-279); rank 0's (long) tmp[0] must be refval = 2676692
    (JGFRayTracerBench.java:87) at every P, on device and host buffers, both engines, MST / FT / faithful
    orders. Under FAITHFUL every rank's buffer must also hold its MST sub-tree partial, as the oracle's."""
    import torch

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    if engine == "exchange":
        monkeypatch.setenv("MPJX_SMP_COPY", "1")
    parts = O.jgf_raytracer_partials(P, "A")
    comms = _world(P, faithful=bool(flags & O.FLAG_FAITHFUL))

    def body(c):
        tmp = parts[c.Rank()].copy()
        if where == "device":
            t = torch.from_numpy(tmp).cuda()
            c.Reduce(t, 0, t, 0, 1, MPI.DOUBLE, MPI.SUM, 0)
            tmp[:] = t.cpu().numpy()
        else:
            c.Reduce(tmp, 0, tmp, 0, 1, MPI.DOUBLE, MPI.SUM, 0)
        return tmp

    try:
        with old_collectives(bool(flags & O.FLAG_OLD)):
            got = mpi.run_multicore(comms, body)
    finally:
        _free(comms)
    assert int(got[0][0]) == O.RT_REFVAL["A"], got[0]
    if flags & O.FLAG_FAITHFUL:
        exp = O.reduce(parts, 1, O.DOUBLE, O.SUM, 0, flags=flags)
        for r in range(P):
            assert got[r][0] == exp[r][0], (r, got[r], exp[r])


@pytest.mark.parametrize("P", [3, 8])
def test_slot_skew_exchange_engine(P, monkeypatch):
    """MPJX_SLOT_SKEW: the exchange engine's input slots 4 KiB apart beyond the block (output slots are
    always skewed): every collective still bit-exact vs the oracle, equal and ragged blocks."""
    monkeypatch.setenv("MPJX_SMP_COPY", "1")
    monkeypatch.setenv("MPJX_SLOT_SKEW", "4096")
    for op, type_ in [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.BXOR, O.INT)]:
        for n in (P * 4096, 100003):
            for kind in ("allreduce", "scan"):
                got, exp = run(kind, P, op, type_, n=n)
                _assert(kind, got, exp, op, type_, ctx=f"skew {kind} n={n}")
            got, exp = run("reduce", P, op, type_, n=n, root=P - 1)
            _assert("reduce", got, exp, op, type_, only=P - 1, ctx=f"skew reduce n={n}")
            for flags in (0, O.FLAG_OLD):
                got, exp = run("allreduce", P, op, type_, n=n, flags=flags)
                _assert("allreduce", got, exp, op, type_, ctx=f"skew flags={flags}")
        got, exp = run("reduce_scatter", P, op, type_, recvcounts=[1000 + 37 * r for r in range(P)])
        _assert("reduce_scatter", got, exp, op, type_, ctx="skew reduce_scatter")


def test_counts_beyond_int32_range():
    """Counts past 2^31 elements (the C ABI's counts are int64; Java's are int, so this is beyond any
    single reference call but inside one mpjbuf-free device call): a BYTE SUM combine and a 2-rank
    Allreduce over 2^31 + 4099 elements, checked on the device against torch's int8 wrap-around add
    (exact and order-free), so every 64-bit index path of the kernels (vector body, sub-vector tail,
    block split) is exercised."""
    import torch

    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    n = (1 << 31) + 4099
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.randint(-128, 128, (n,), dtype=torch.int8, device="cuda", generator=g)
    b = torch.randint(-128, 128, (n,), dtype=torch.int8, device="cuda", generator=g)
    exp = a + b
    torch.cuda.synchronize()
    mpi.combine(MPI.SUM, MPI.BYTE, a, b)
    torch.cuda.synchronize()
    assert torch.equal(a, exp)
    del exp
    a.sub_(b)  # back to the first operand
    exp = a + b
    outs = [torch.empty_like(a), torch.empty_like(a)]
    torch.cuda.synchronize()
    comms = _world(2)
    try:
        mpi.run_multicore(comms, lambda c: c.Allreduce(a if c.Rank() == 0 else b, 0, outs[c.Rank()], 0, n,
                                                       MPI.BYTE, MPI.SUM))
    finally:
        _free(comms)
    assert torch.equal(outs[0], exp) and torch.equal(outs[1], exp)


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_microbenchmark_max_pattern_gpu(P):
    """test/microbenchmarkmpiJava/{allreduce,reduce,reducescatter,scan}.java's input, A[i] = 1/(i+1) on
    every rank, with MPI.MAX through libmpjx: every result is A (or its block), MPI and faithful modes."""
    n = 4096 * P
    A = 1.0 / (np.arange(n) + 1.0)
    for flags in (0, O.FLAG_OLD, O.FLAG_FAITHFUL):
        inputs = [A.copy() for _ in range(P)]
        for kind in ("allreduce", "scan"):
            got, _ = run(kind, P, O.MAX, O.DOUBLE, n=n, flags=flags, inputs=[a.copy() for a in inputs])
            assert all(np.array_equal(g, A) for g in got), (kind, flags)
        got, _ = run("reduce", P, O.MAX, O.DOUBLE, n=n, root=0, flags=flags, inputs=[a.copy() for a in inputs])
        assert np.array_equal(got[0], A), ("reduce", flags)
        got, _ = run("reduce_scatter", P, O.MAX, O.DOUBLE, recvcounts=[4096] * P, flags=flags,
                     inputs=[a.copy() for a in inputs])
        assert all(np.array_equal(got[r], A[4096 * r:4096 * (r + 1)]) for r in range(P)), ("rs", flags)


@pytest.mark.parametrize("mode", ["all", "none", "leader_only", "others_only"])
def test_blocking_flag_multicore(mode):
    """MPJX_FLAG_BLOCKING in multicore mode (4 rank threads, one GPU, rank 0 launching for all): a
    blocking call returns with its results complete, the launching rank drains its stream before the
    rendezvous and the others skip their device-side waits on it. Ranks may disagree on the flag
    (`leader_only`, `others_only`): a rank waits on the device for every launcher that did not drain.
    Allreduce / Reduce / Reduce_scatter / Scan, 40 calls each on fresh data, every element against the
    oracle; a non-blocking rank synchronises before it checks."""
    import torch

    from mpjexpress_amd import _lib, mpi

    L = _lib.lib()
    P, n = 4, 3 * 1024 + 16
    B = 0x10
    comms = mpi.smp_world(P, [0] * P)

    def blocking(r):
        return {"all": True, "none": False, "leader_only": r == 0, "others_only": r != 0}[mode]

    rounds = []
    for it in range(10):
        sends = [make_input(O.DOUBLE, n, 4000 + 97 * it + r, specials=False) for r in range(P)]
        rounds.append(sends)

    def body(c):
        r = c.Rank()
        h = c.handle
        f = B if blocking(r) else 0
        got = []
        for sends in rounds:
            x = torch.from_numpy(sends[r]).cuda()
            y = torch.zeros_like(x)
            z = torch.zeros(n // P, dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            rc = (ctypes.c_int64 * P)(*([n // P] * P))
            out = []
            for call in ("ar", "rd", "rs", "sc"):
                if call == "ar":
                    st = L.mpjx_allreduce(h, x.data_ptr(), y.data_ptr(), n, O.DOUBLE, O.SUM, f, None)
                elif call == "rd":
                    st = L.mpjx_reduce(h, x.data_ptr(), y.data_ptr(), n, O.DOUBLE, O.SUM, 0, f, None)
                elif call == "rs":
                    st = L.mpjx_reduce_scatter(h, x.data_ptr(), z.data_ptr(), rc, O.DOUBLE, O.SUM, f, None)
                else:
                    st = L.mpjx_scan(h, x.data_ptr(), y.data_ptr(), n, O.DOUBLE, O.SUM, f, None)
                _lib.check(st, call)
                if not f:
                    _lib.check(L.mpjx_comm_synchronize(h), "sync")
                res = z if call == "rs" else y
                out.append(res.cpu().numpy().copy() if (call != "rd" or r == 0) else None)
            got.append(out)
        return got

    try:
        res = mpi.run_multicore(comms, body)
    finally:
        for c in comms:
            c.Free()
    for it, sends in enumerate(rounds):
        ar = O.allreduce(sends, n, O.DOUBLE, O.SUM)
        rd = O.reduce(sends, n, O.DOUBLE, O.SUM, 0)[0]
        sc = O.scan(sends, n, O.DOUBLE, O.SUM)
        rs = O.reduce_scatter(sends, [n // P] * P, O.DOUBLE, O.SUM)[0]
        for r in range(P):
            a_, d_, s_, c_ = res[r][it]
            assert same_bits(O.DOUBLE, O.SUM, a_, ar[r]), (mode, it, r, "allreduce")
            if r == 0:
                assert same_bits(O.DOUBLE, O.SUM, d_, rd), (mode, it, "reduce")
            assert same_bits(O.DOUBLE, O.SUM, s_, rs[r]), (mode, it, r, "reduce_scatter")
            assert same_bits(O.DOUBLE, O.SUM, c_, sc[r]), (mode, it, r, "scan")
