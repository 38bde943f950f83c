"""GPU parity: the element-wise combine (one typed Op.perform, src/mpi/SumDouble.java:49-55) for all
46 (op, type) pairs of the reference, through the C ABI (mpjx_combine), bit-exact vs the oracle."""
import numpy as np
import pytest

import oracle as O
from util import flat, make_input, same_bits

pytestmark = pytest.mark.gpu

SIZES = [1, 7, 16, 33, 1000, 4097, 65536 + 5]


def _torch():
    import torch

    return torch


def _dev(a, misalign=0):
    """Copy numpy -> device tensor; misalign > 0 places it at an element offset (unaligned pointer)."""
    torch = _torch()
    t = torch.from_numpy(np.concatenate([np.zeros(misalign, a.dtype), a])).cuda()
    return t[misalign:]


@pytest.mark.parametrize("op,type_", [(o, t) for o in range(1, 11) for t in range(1, 9)
                                       if (o, t) in set(O.valid_pairs())])
def test_combine_all_pairs(op, type_):
    from mpjexpress_amd import mpi

    dt = mpi.DATATYPES[type_ - 1]
    opx = mpi.OPS[op - 1]
    for n in SIZES:
        for mis in (0, 1):
            acc = make_input(type_, n, 1000 + n, op=op)
            inp = make_input(type_, n, 2000 + n, op=op)
            exp = O.apply(op, type_, acc.copy(), inp)
            ta, tb = _dev(acc, mis), _dev(inp, mis)
            mpi.combine(opx, dt, ta, tb)
            _torch().cuda.synchronize()
            got = ta.cpu().numpy()
            assert same_bits(type_, op, got, exp), (O.OP_NAMES[op], O.TYPE_NAMES[type_], n, mis)
            assert np.array_equal(tb.cpu().numpy().view(np.uint8), inp.view(np.uint8))


def test_combine_java_max_min_semantics():
    """MAX/MIN as `if (in > acc) acc = in`: a NaN in never replaces, a NaN acc stays, +0/-0 ties
    keep the accumulator (src/mpi/MaxDouble.java:51-53, MinDouble.java:53-55) — not fmax/fmin."""
    from mpjexpress_amd import mpi

    nan = np.nan
    acc = np.array([1.0, nan, 0.0, -0.0, 2.0, -np.inf, 5e-324] * 4, dtype=np.float64)
    inp = np.array([nan, 3.0, -0.0, 0.0, 2.0, np.inf, -5e-324] * 4, dtype=np.float64)
    for opx, op in ((mpi.MPI.MAX, O.MAX), (mpi.MPI.MIN, O.MIN)):
        ta, tb = _dev(acc), _dev(inp)
        mpi.combine(opx, mpi.MPI.DOUBLE, ta, tb)
        got = ta.cpu().numpy()
        exp = O.apply(op, O.DOUBLE, acc.copy(), inp)
        assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))
        # explicit expectations (tie keeps acc sign; NaN acc stays NaN; NaN in ignored)
        assert got[0] == 1.0 and np.isnan(got[1])
        assert np.signbit(got[2]) == np.signbit(acc[2]) and np.signbit(got[3]) == np.signbit(acc[3])


def test_combine_char_is_unsigned_and_wraps():
    from mpjexpress_amd import mpi

    acc = np.array([0xFFFF, 1, 0x8000, 300] * 8, dtype=np.uint16)
    inp = np.array([2, 0xFFFF, 0x7FFF, 300] * 8, dtype=np.uint16)
    for opx, op in ((mpi.MPI.SUM, O.SUM), (mpi.MPI.PROD, O.PROD), (mpi.MPI.MAX, O.MAX), (mpi.MPI.MIN, O.MIN)):
        ta, tb = _dev(acc), _dev(inp)
        mpi.combine(opx, mpi.MPI.CHAR, ta, tb)
        assert np.array_equal(ta.cpu().numpy(), O.apply(op, O.CHAR, acc.copy(), inp))


def test_combine_invalid_pairs_raise():
    """SUM on BOOLEAN throws (src/mpi/SumWorker.java:60); BAND on DOUBLE (BandWorker.java:60)."""
    from mpjexpress_amd import mpi

    t = _dev(np.zeros(8, np.uint8))
    with pytest.raises(mpi.MPIException, match="BOOLEAN"):
        mpi.combine(mpi.MPI.SUM, mpi.MPI.BOOLEAN, t, t)
    d = _dev(np.zeros(8, np.float64))
    with pytest.raises(mpi.MPIException, match="DOUBLE"):
        mpi.combine(mpi.MPI.BAND, mpi.MPI.DOUBLE, d, d)


def test_host_pointers_rejected_before_any_kernel():
    """A pageable host array handed to a device entry point is an argument error, never a kernel
    launch (a kernel dereferencing it would fault the GPU): combine, combine_multi and a 1-rank
    Allreduce through the C ABI all return MPJX_ERR_ARG."""
    import ctypes

    from mpjexpress_amd import _lib, mpi

    L = _lib.lib()
    host = np.zeros(1024)
    d = _dev(np.zeros(1024))
    hp, dp = ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(d.data_ptr())
    assert L.mpjx_combine(3, 8, dp, hp, 1024, None) == -1
    assert b"not GPU-accessible" in L.mpjx_last_error()
    assert L.mpjx_combine(3, 8, hp, dp, 1024, None) == -1
    ins = (ctypes.c_void_p * 2)(dp, hp)
    outs = (ctypes.c_void_p * 1)(dp)
    assert L.mpjx_combine_multi(3, 8, 0, 2, ins, outs, 1024, 0, 0, None) == -1
    (c,) = mpi.smp_world(1)
    try:
        assert L.mpjx_allreduce(c.handle, hp, dp, 1024, 8, 3, 0, None) == -1
        assert L.mpjx_allreduce(c.handle, dp, dp, 1024, 8, 3, 0, None) == 0
    finally:
        c.Free()


def test_combine_c2_full_size_double_sum():
    """Config C2 at its full size: 2 x 256 MiB double, inout = in + inout, bit-exact."""
    n = 33554432
    acc = make_input(O.DOUBLE, n, 0x4D504A00 + 2000, specials=False)
    inp = make_input(O.DOUBLE, n, 0x4D504A00 + 2001, specials=False)
    from mpjexpress_amd import mpi

    ta, tb = _dev(acc), _dev(inp)
    mpi.combine(mpi.MPI.SUM, mpi.MPI.DOUBLE, ta, tb)
    got = ta.cpu().numpy()
    O.apply(O.SUM, O.DOUBLE, acc, inp)
    assert np.array_equal(got.view(np.uint64), acc.view(np.uint64))


@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8, 9, 13])
def test_combine_multi_orders(P):
    """mpjx_combine_multi: MST at every root, FOLD and SCAN, against the oracle's collectives run on
    the same P slices (the MST root-r Reduce, the Scan, and FT_Reduce rooted at 0)."""
    import ctypes

    import torch

    from mpjexpress_amd import _lib

    L = _lib.lib()
    n = 2051
    for op, t in [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.PROD, O.INT), (O.LXOR, O.BOOLEAN)]:
        xs = [make_input(t, n, 97 * p + P, op=op) for p in range(P)]
        dev = [_dev(x) for x in xs]
        pin = (ctypes.c_void_p * P)(*[d.data_ptr() for d in dev])
        for root in range(P):
            out = torch.empty_like(dev[0])
            pout = (ctypes.c_void_p * 1)(out.data_ptr())
            _lib.check(L.mpjx_combine_multi(op, t, 1, P, pin, pout, n, root, 0, None), "mst")
            torch.cuda.synchronize()
            exp = O.reduce(xs, n, t, op, root)[root]
            assert same_bits(t, op, out.cpu().numpy(), exp), ("mst", P, root, op, t)
        out = torch.empty_like(dev[0])
        pout = (ctypes.c_void_p * 1)(out.data_ptr())
        _lib.check(L.mpjx_combine_multi(op, t, 0, P, pin, pout, n, 0, 0, None), "fold")
        torch.cuda.synchronize()
        exp = O.reduce(xs, n, t, op, 0, flags=O.FLAG_OLD)[0]
        assert same_bits(t, op, out.cpu().numpy(), exp), ("fold", P, op, t)
        outs = [torch.empty_like(dev[0]) for _ in range(P)]
        pout = (ctypes.c_void_p * P)(*[o.data_ptr() for o in outs])
        _lib.check(L.mpjx_combine_multi(op, t, 2, P, pin, pout, n, 0, 0, None), "scan")
        torch.cuda.synchronize()
        exp = O.scan(xs, n, t, op)
        for r in range(P):
            assert same_bits(t, op, outs[r].cpu().numpy(), exp[r]), ("scan", P, r, op, t)


@pytest.mark.parametrize("op,type_", O.loc_pairs())
def test_combine_maxloc_minloc(op, type_):
    """One MAXLOC / MINLOC combine on pair buffers, aligned and offset by one base element."""
    from mpjexpress_amd import mpi

    dt = mpi.datatype(type_)
    for n in (1, 5, 64, 1001, 40000):
        for mis in (0, 1):
            acc = make_input(type_, n, 31 + n)
            inp = make_input(type_, n, 77 + n)
            exp = O.apply(op, type_, acc.copy(), inp)
            ta, tb = _dev(flat(acc, type_), mis), _dev(flat(inp, type_), mis)
            mpi.combine(mpi.OPS[op - 1], dt, ta, tb)
            _torch().cuda.synchronize()
            got = ta.cpu().numpy().view(acc.dtype)
            assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), (op, type_, n, mis)


@pytest.mark.parametrize("form", ["streaming", "short"])
def test_streaming_form_every_instantiation(form):
    """The streaming forms (mpjx_kernels.hpp launch_pw) run only for launches that stream >= 64 MiB: the
    1024/512-lane non-temporal tiles from 256 MiB up, and below that the short-launch forms (deep 256-lane
    tiles for K_SCAN, a persistent one-block-per-CU grid for the others). A child process with
    MPJX_NT_MIN_MIB=0 (and MPJX_SHORT_MAX_MIB=0 for the long form) sends every vector launch through
    one of them at oracle-checkable sizes: every pair's fold, FOLD/MST/SCAN at P = 2..8 (incl. the
    512-lane narrow-type instantiations, the shallower byte / 16-bit / pair tiles and MAXLOC/MINLOC),
    native and big-endian."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MPJX_NT_MIN_MIB="0")
    if form == "streaming":
        env["MPJX_SHORT_MAX_MIB"] = "0"
    else:
        env.pop("MPJX_SHORT_MAX_MIB", None)
    p = subprocess.run([sys.executable, os.path.join(here, "stream_worker.py")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    assert "streaming form: 0 mismatches" in p.stdout


@pytest.mark.parametrize("op,type_", [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.BXOR, O.INT), (O.MAXLOC, O.DOUBLE2)])
@pytest.mark.parametrize("swap", [0, 0xC])
@pytest.mark.parametrize("kind", [1, 2])
def test_p8_colliding_streams(op, type_, swap, kind):
    """K_MST / K_SCAN P=8 at streaming size with the 8 inputs in ONE allocation at a 16 MiB stride (the
    RCCL exchange engine's contiguous slots): the launcher sees the streams congruent mod 16 MiB and
    runs the staggered load group (mpjx_kernels.hpp streams_collide / CollideGroup) — native and
    big-endian bodies, MST roots 0 and 5, bit-exact vs the oracle's MST_Reduce / Scan
    (PureIntracomm.java:1943-1992, 2526-2544)."""
    import ctypes

    import torch

    from mpjexpress_amd import _lib

    if swap and type_ in O.PAIR_BASE:
        pytest.skip("big-endian pairs are covered by test_big_endian_combine_multi")
    L = _lib.lib()
    P, stride = 8, 16 << 20
    esz = np.dtype(O.NP_DTYPE[type_]).itemsize
    n = stride // esz  # 16 MiB per slice: 9 x 16 MiB streamed, the streaming (non-temporal) form
    xs = [make_input(type_, n, 4242 + p, op=op) for p in range(P)]
    buf = torch.empty(P * stride, dtype=torch.uint8, device="cuda")
    for p, x in enumerate(xs):
        b = flat(x, type_)
        if swap:
            b = b.byteswap()
        buf[p * stride:(p + 1) * stride] = torch.from_numpy(np.ascontiguousarray(b).view(np.uint8))
    Q = P if kind == 2 else 1
    out = torch.empty(Q * (stride + 4096), dtype=torch.uint8, device="cuda")  # output slots skewed, as the engines
    pin = (ctypes.c_void_p * P)(*[buf.data_ptr() + p * stride for p in range(P)])
    pout = (ctypes.c_void_p * Q)(*[out.data_ptr() + q * (stride + 4096) for q in range(Q)])
    for root in ((0, 5) if kind == 1 else (0,)):
        _lib.check(L.mpjx_combine_multi(op, type_, kind, P, pin, pout, n, root, swap, None), "combine_multi")
        torch.cuda.synchronize()
        exp = [O.reduce(xs, n, type_, op, root)[root]] if kind == 1 else O.scan(xs, n, type_, op)
        host = out.cpu().numpy()
        for q in range(Q):
            raw = host[q * (stride + 4096):q * (stride + 4096) + stride]
            if xs[0].dtype.names:
                assert np.array_equal(raw, exp[q].view(np.uint8)), (op, type_, kind, root, q)
                continue
            got = raw.view(xs[0].dtype)
            if swap:
                got = flat(got, type_).byteswap().view(xs[0].dtype)
            assert same_bits(type_, op, got, exp[q]), (op, type_, swap, kind, root, q)
