"""Drives the JNI shim (integration/jni/mpi_HipIntracomm.c) through the functional JNIEnv stand-in
(tests/jni/fakejvm.c), as a JVM's HipIntracomm would call it — VERDICT r4 "do this" #3. Run as its own
process by tests/test_gpu_jni.py (and by the CPU checks in tests/test_jni_fake.py with --cpu): no torch,
so libmpjx binds /opt/rocm's HIP runtime and RCCL, the pairing a JVM gets.

Scenarios (each result bit for bit against the oracle on offset-0 copies of the same windows):
  single  one JVM per GPU: a 1-rank RCCL world (nativeUniqueId + nativeInitRank; MPJX_P1_EXCHANGE=1 sends
          the calls through the exchange path) and a 1-rank IPC world (nativeInitIpc), nativeDeviceCount;
          arrays pinned with GetPrimitiveArrayCritical, which the
          stand-in serves as COPIES: only the write-back modes the shim chooses decide what reaches the
          Java arrays (recv: mode 0, send: JNI_ABORT);
  multicore  smpdev: P = 4 rank threads of this process, each forming its communicator with
          nativeInitSmp; Allreduce / Reduce / Reduce_scatter / Scan with rank-local nonzero offsets,
          direct buffers with the big-endian flags, MAXLOC on DOUBLE2 with a pair offset; then an
          invalid (op, type) pair on every rank, and a too-short array on ONE rank (that rank gets the
          shim's bounds message, the others an MPIException instead of a hang).
Every call also checks: no JNI rule broken (fakejvm's violation log), no critical region left held,
elements outside the call's window untouched.
Prints one JSON object: {"cases": {name: "ok" | error text}, "violations": [...]}.
"""
import ctypes
import faulthandler
import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (the checker)

SO = os.environ.get("MPJX_JNI_DRIVER_SO") or os.path.join(ROOT, "tests", "jni", "libmpjx_jni_fake.so")
FLAG_SEND_BE, FLAG_RECV_BE = 0x4, 0x8
ESZ = {O.BYTE: 1, O.CHAR: 2, O.SHORT: 2, O.BOOLEAN: 1, O.INT: 4, O.LONG: 8, O.FLOAT: 4, O.DOUBLE: 8}

L = ctypes.CDLL(SO)
VP, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
L.fj_env.restype = VP
L.fj_array.restype = VP
L.fj_array.argtypes = [ctypes.c_int, ctypes.c_longlong]
L.fj_direct.restype = VP
L.fj_direct.argtypes = [VP, ctypes.c_longlong]
L.fj_object.restype = VP
L.fj_data.restype = VP
L.fj_data.argtypes = [VP]
L.fj_free.argtypes = [VP]
L.fj_exception.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
L.fj_violations.argtypes = [ctypes.c_char_p, ctypes.c_int]
L.fj_release_modes.argtypes = [VP, ctypes.POINTER(ctypes.c_int)]
L.mpjx_jni_staging_live.restype = ctypes.c_long
L.mpjx_comm_destroy.argtypes = [VP]
J = "Java_mpi_HipIntracomm_"
for name, res, args in (
        ("nativeDeviceCount", I32, [VP, VP]),
        ("nativeUniqueId", None, [VP, VP, VP]),
        ("nativeInitRank", I64, [VP, VP, I32, I32, I32, VP]),
        ("nativeInitSmp", I64, [VP, VP, VP, I32, I32, VP]),
        ("nativeInitIpc", I64, [VP, VP, I32, I32, I32, VP]),
        ("nativeFree", None, [VP, VP, I64]),
        ("nativeReduce", None, [VP, VP, I64, VP, I32, VP, I32, I32, I32, I32, I32, I32]),
        ("nativeAllreduce", None, [VP, VP, I64, VP, I32, VP, I32, I32, I32, I32, I32]),
        ("nativeReduceScatter", None, [VP, VP, I64, VP, I32, VP, I32, VP, I32, I32, I32]),
        ("nativeScan", None, [VP, VP, I64, VP, I32, VP, I32, I32, I32, I32, I32])):
    f = getattr(L, J + name)
    f.restype, f.argtypes = res, args
ENV = L.fj_env()
SELF = L.fj_object()
VERBOSE = os.environ.get("MPJX_JNI_DRIVER_VERBOSE") == "1"
faulthandler.enable()  # a native crash prints every thread's Python stack (which native call it was)
if os.environ.get("MPJX_JNI_DRIVER_WATCHDOG_S"):  # a hang prints every thread's stacks, then ends the run
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import watchdog

    watchdog.arm(os.environ["MPJX_JNI_DRIVER_WATCHDOG_S"])


def native(name, *args):
    """One native method call; returns (result, pending exception (class, message) or None)."""
    if VERBOSE:
        print(f"jni_driver: {threading.current_thread().name} {name}", file=sys.stderr, flush=True)
    f = getattr(L, J + name)
    assert f.argtypes is not None, f"{name}: no ctypes signature declared (pointers would be truncated)"
    r = f(ENV, SELF, *args)
    cls, msg = ctypes.create_string_buffer(128), ctypes.create_string_buffer(1024)
    exc = (cls.value.decode(), msg.value.decode()) if L.fj_exception(cls, 128, msg, 1024) else None
    if L.fj_crit_held():
        raise AssertionError(f"{name}: {L.fj_crit_held()} critical region(s) still held on return")
    return r, exc


def jarray(np_arr):
    """A Java array holding a copy of np_arr; (object, numpy view of its elements)."""
    a = np.ascontiguousarray(np_arr)
    o = L.fj_array(a.itemsize, a.size)
    v = np.frombuffer((ctypes.c_uint8 * max(1, a.size * a.itemsize)).from_address(L.fj_data(o)), dtype=a.dtype,
                      count=a.size)
    v[:] = a
    return o, v


def release_modes(o):
    m = (ctypes.c_int * 3)()
    L.fj_release_modes(o, m)
    return list(m)


def violations():
    buf = ctypes.create_string_buffer(4096)
    n = L.fj_violations(buf, 4096)
    return n, buf.value.decode()


def same(got, exp):
    g, e = np.asarray(got), np.asarray(exp)
    if g.dtype.kind == "f":  # NaN payloads compare equal (tests/util.py:same_bits)
        gn, en = np.isnan(g), np.isnan(e)
        return bool(np.array_equal(gn, en) and np.array_equal(g[~gn].view(np.uint8), e[~en].view(np.uint8)))
    return bool(np.array_equal(g.view(np.uint8), e.view(np.uint8)))


def sentinel(dtype, n):
    return np.full(n, 77, dtype=dtype)


def rng_vals(t, n, seed):
    r = np.random.default_rng(seed)
    dt = np.dtype(O.NP_DTYPE[t])
    if dt.kind == "f":
        return r.uniform(-1, 1, n).astype(dt)
    info = np.iinfo(dt)
    return r.integers(info.min, info.max, n, endpoint=True, dtype=dt)


# ---------------------------------------------------------------------------------------------------
def single(cases):
    """One rank per JVM: the critical-region path, with the stand-in handing out copies."""
    L.fj_copy_mode(1)
    uo, _ = jarray(np.zeros(128, np.int8))
    _, exc = native("nativeUniqueId", uo)
    assert exc is None, exc
    comm, exc = native("nativeInitRank", 0, 1, 0, uo)
    assert exc is None and comm, exc
    n, soff, roff = 10007, 3, 5
    x = rng_vals(O.DOUBLE, n, 1)
    so, sv = jarray(np.concatenate([sentinel(np.float64, soff), x, sentinel(np.float64, 4)]))
    ro, rv = jarray(sentinel(np.float64, roff + n + 6))
    send_before = sv.copy()
    _, exc = native("nativeAllreduce", comm, so, soff, ro, roff, n, O.DOUBLE, O.SUM, 0)
    ok = exc is None and same(rv[roff:roff + n], O.allreduce([x], n, O.DOUBLE, O.SUM)[0])
    ok = ok and same(rv[:roff], sentinel(np.float64, roff)) and same(rv[roff + n:], sentinel(np.float64, 6))
    ok = ok and same(sv, send_before)
    # recv released with mode 0 (copied back), send with JNI_ABORT (the call does not write it)
    modes = (release_modes(so), release_modes(ro))
    cases["single_allreduce_offsets_writeback"] = "ok" if ok and modes == ([0, 0, 1], [1, 0, 0]) else \
        f"exc={exc} modes={modes}"
    # larger than the host pipeline's 16 MiB chunk (40 MiB + 3 elements, pinned through the critical
    # region, pageable as far as the HIP runtime knows): the chunked H2D / collective / D2H path and its
    # drain thread under the shim, with offsets
    nb = (40 << 20) // 8 + 3
    xb = rng_vals(O.DOUBLE, nb, 2)
    bso, bsv = jarray(np.concatenate([sentinel(np.float64, 7), xb]))
    bro, brv = jarray(sentinel(np.float64, nb + 11))
    _, exc = native("nativeAllreduce", comm, bso, 7, bro, 2, nb, O.DOUBLE, O.SUM, 0)
    ok = exc is None and same(brv[2:2 + nb], xb) and same(brv[:2], sentinel(np.float64, 2)) and \
        same(brv[2 + nb:], sentinel(np.float64, 9))
    cases["single_allreduce_40MiB_chunked"] = "ok" if ok else f"exc={exc}"
    # Reduce root 0, Scan, Reduce_scatter: the other entry points' buffer handling
    for name, fn in (("reduce", lambda: native("nativeReduce", comm, so, soff, ro, roff, n, O.DOUBLE, O.MAX, 0, 0)),
                     ("scan", lambda: native("nativeScan", comm, so, soff, ro, roff, n, O.DOUBLE, O.PROD, 0))):
        rv[:] = 77
        _, exc = fn()
        cases[f"single_{name}"] = "ok" if exc is None and same(rv[roff:roff + n], x) and \
            same(rv[:roff], sentinel(np.float64, roff)) else f"exc={exc}"
    rc_o, _ = jarray(np.array([n], np.int32))
    rv[:] = 77
    _, exc = native("nativeReduceScatter", comm, so, soff, ro, roff, rc_o, O.DOUBLE, O.SUM, 0)
    cases["single_reduce_scatter"] = "ok" if exc is None and same(rv[roff:roff + n], x) else f"exc={exc}"
    # direct buffers (mpjbuf payloads) with the byte-order flags: big-endian in, native out
    xb = x.astype(">f8")
    dsend = np.frombuffer(xb.tobytes(), dtype=np.uint8).copy()
    drecv = np.zeros(8 * n, np.uint8)
    ds, dr = L.fj_direct(dsend.ctypes.data, dsend.size), L.fj_direct(drecv.ctypes.data, drecv.size)
    _, exc = native("nativeAllreduce", comm, ds, 0, dr, 0, n, O.DOUBLE, O.SUM, FLAG_SEND_BE)
    cases["single_direct_big_endian_in"] = "ok" if exc is None and same(drecv.view(np.float64), x) else f"exc={exc}"
    _, exc = native("nativeAllreduce", comm, ds, 0, dr, 0, n, O.DOUBLE, O.SUM, FLAG_SEND_BE | FLAG_RECV_BE)
    cases["single_direct_big_endian_in_out"] = "ok" if exc is None and same(drecv, dsend) else f"exc={exc}"
    small = L.fj_direct(drecv.ctypes.data, 8 * n - 1)
    _, exc = native("nativeAllreduce", comm, ds, 0, small, 0, n, O.DOUBLE, O.SUM, 0)
    cases["single_direct_too_small"] = "ok" if exc and exc[0] == "mpi/MPIException" and "too small" in exc[1] \
        else f"exc={exc}"
    # an (op, type) pair the reference has no worker for: mpi.MPIException with libmpjx's own text
    rv[:] = 77
    _, exc = native("nativeAllreduce", comm, so, soff, ro, roff, n, O.DOUBLE, O.BAND, 0)
    cases["single_invalid_pair"] = "ok" if exc and exc[0] == "mpi/MPIException" and "Allreduce" in exc[1] and \
        same(rv, sentinel(np.float64, rv.size)) else f"exc={exc}"
    _, exc = native("nativeFree", comm)
    cases["single_free"] = "ok" if exc is None else f"exc={exc}"
    ndev, exc = native("nativeDeviceCount")
    cases["single_device_count"] = "ok" if exc is None and ndev >= 1 else f"exc={exc} n={ndev}"
    # one JVM per GPU without RCCL: the HIP-IPC world (-Dmpjx.engine=ipc), any 128 bytes as its id
    io, _ = jarray(np.random.default_rng(9).integers(-128, 127, 128, dtype=np.int8))
    ic, exc = native("nativeInitIpc", 0, 1, 0, io)
    if exc is None and ic:
        rv[:] = 77
        _, exc = native("nativeAllreduce", ic, so, soff, ro, roff, n, O.DOUBLE, O.MIN, 0)
        ok = exc is None and same(rv[roff:roff + n], x) and same(rv[:roff], sentinel(np.float64, roff))
        _, exc2 = native("nativeFree", ic)
        cases["single_ipc_world"] = "ok" if ok and exc2 is None else f"exc={exc} free={exc2}"
    else:
        cases["single_ipc_world"] = f"init: exc={exc}"
    L.fj_copy_mode(0)


def multicore(cases, P=4):
    """smpdev: P rank threads, each forming its communicator through the shim (nativeInitSmp)."""
    idv = np.random.default_rng(7).integers(-128, 127, 128, dtype=np.int8)
    res = {}

    def run(body):
        errs = [None] * P
        out = [None] * P

        def th(r):
            try:
                out[r] = body(r)
            except BaseException as e:  # noqa: BLE001
                errs[r] = repr(e)
        ts = [threading.Thread(target=th, args=(r,)) for r in range(P)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=300)
        if any(t.is_alive() for t in ts):
            raise AssertionError("a rank thread hung")
        for e in errs:
            if e:
                raise AssertionError(e)
        return out

    def init(idbytes):
        def body(r):
            io, _ = jarray(idbytes)
            do, _ = jarray(np.zeros(P, np.int32))
            c, exc = native("nativeInitSmp", io, r, P, do)
            assert exc is None and c, exc
            return c
        return run(body)

    comms = init(idv)

    def collective(name, t, op, count_of, soff_of, roff_of, call, expected, recv_len=None, direct=None):
        """Each rank r passes its own offsets; expected(windows) -> per-rank expected windows."""
        xs = [rng_vals(t, count_of(r, "send"), 100 * r + 11) for r in range(P)]
        dt = np.dtype(O.NP_DTYPE[t])
        objs, views = [], []
        for r in range(P):
            so, sv = jarray(np.concatenate([sentinel(dt, soff_of(r)), xs[r], sentinel(dt, 3)]))
            rl = recv_len(r) if recv_len else count_of(r, "recv")
            ro, rv = jarray(sentinel(dt, roff_of(r) + rl + 5))
            objs.append((so, ro))
            views.append((sv, rv, sv.copy()))

        def body(r):
            _, exc = call(r, comms[r], objs[r][0], soff_of(r), objs[r][1], roff_of(r))
            return exc
        excs = run(body)
        exp = expected(xs)
        bad = []
        for r in range(P):
            sv, rv, s0 = views[r]
            rl = recv_len(r) if recv_len else count_of(r, "recv")
            if excs[r] is not None:
                bad.append(f"rank {r}: {excs[r]}")
            elif exp[r] is not None and not same(rv[roff_of(r):roff_of(r) + rl], exp[r]):
                bad.append(f"rank {r}: result differs")
            elif not same(rv[:roff_of(r)], sentinel(dt, roff_of(r))) or not same(rv[roff_of(r) + rl:], sentinel(dt, 5)):
                bad.append(f"rank {r}: wrote outside its window")
            elif not same(sv, s0):
                bad.append(f"rank {r}: sendbuf changed")
        res[name] = "ok" if not bad else "; ".join(bad)

    n = 10007
    collective("mc_allreduce_double_sum_offsets", O.DOUBLE, O.SUM, lambda r, k: n, lambda r: r + 1, lambda r: 2 * r,
               lambda r, c, s, so, rr, ro: native("nativeAllreduce", c, s, so, rr, ro, n, O.DOUBLE, O.SUM, 0),
               lambda xs: O.allreduce(xs, n, O.DOUBLE, O.SUM))
    collective("mc_reduce_int_sum_root2", O.INT, O.SUM, lambda r, k: n, lambda r: 3 * r, lambda r: r,
               lambda r, c, s, so, rr, ro: native("nativeReduce", c, s, so, rr, ro, n, O.INT, O.SUM, 2, 0),
               lambda xs: [O.reduce(xs, n, O.INT, O.SUM, 2)[2] if r == 2 else None for r in range(P)])
    rcs = [3, 1000, 0, 517]
    tot = sum(rcs)

    def rs_call(r, c, s, so, rr, ro):
        rco, _ = jarray(np.array(rcs, np.int32))
        return native("nativeReduceScatter", c, s, so, rr, ro, rco, O.FLOAT, O.SUM, 0)
    collective("mc_reduce_scatter_float_ragged", O.FLOAT, O.SUM, lambda r, k: tot if k == "send" else rcs[r],
               lambda r: r, lambda r: 1, rs_call, lambda xs: O.reduce_scatter(xs, rcs, O.FLOAT, O.SUM)[0])
    collective("mc_scan_double_sum", O.DOUBLE, O.SUM, lambda r, k: n, lambda r: 0, lambda r: r + 2,
               lambda r, c, s, so, rr, ro: native("nativeScan", c, s, so, rr, ro, n, O.DOUBLE, O.SUM, 0),
               lambda xs: O.scan(xs, n, O.DOUBLE, O.SUM))
    # MAXLOC on DOUBLE2: offsets and counts in base elements / pairs (the array is a double[])
    npair = 999

    def pairs(r):
        v = rng_vals(O.DOUBLE, 2 * npair, 500 + r)
        v[1::2] = r  # index = rank
        v[0::2] = np.round(v[0::2] * 4) / 4  # ties across ranks
        return v
    pv = [pairs(r) for r in range(P)]
    pobjs = []
    for r in range(P):
        so, sv = jarray(np.concatenate([sentinel(np.float64, 2 * r), pv[r]]))
        ro, rv = jarray(sentinel(np.float64, 2 + 2 * npair))
        pobjs.append((so, ro, rv))
    excs = run(lambda r: native("nativeAllreduce", comms[r], pobjs[r][0], 2 * r, pobjs[r][1], 2, npair,
                                O.DOUBLE2, O.MAXLOC, 0)[1])
    exp = O.allreduce([p.view(O.NP_DTYPE[O.DOUBLE2]) for p in pv], npair, O.DOUBLE2, O.MAXLOC)
    ok = all(e is None for e in excs) and all(same(pobjs[r][2][2:], np.asarray(exp[r]).view(np.float64))
                                               for r in range(P))
    res["mc_allreduce_double2_maxloc_pair_offsets"] = "ok" if ok else f"excs={excs}"
    # direct buffers, big-endian payloads in and out (mpjbuf sections as niodev delivers them)
    xs = [rng_vals(O.FLOAT, n, 900 + r) for r in range(P)]
    dsend = [np.frombuffer(x.astype(">f4").tobytes(), np.uint8).copy() for x in xs]
    drecv = [np.zeros(4 * n, np.uint8) for _ in range(P)]
    dobj = [(L.fj_direct(dsend[r].ctypes.data, dsend[r].size), L.fj_direct(drecv[r].ctypes.data, drecv[r].size))
            for r in range(P)]
    excs = run(lambda r: native("nativeAllreduce", comms[r], dobj[r][0], 0, dobj[r][1], 0, n, O.FLOAT, O.MAX,
                                FLAG_SEND_BE | FLAG_RECV_BE)[1])
    exp = O.allreduce(xs, n, O.FLOAT, O.MAX)
    ok = all(e is None for e in excs) and all(same(drecv[r].view(">f4").astype(np.float32), exp[r]) for r in range(P))
    res["mc_allreduce_direct_big_endian"] = "ok" if ok else f"excs={excs}"
    # an invalid (op, type) pair on every rank: each rank's own MPIException, nobody waits
    ao, _ = jarray(np.zeros(16, np.float64))
    bo, _ = jarray(np.zeros(16, np.float64))
    excs = run(lambda r: native("nativeAllreduce", comms[r], ao, 0, bo, 0, 16, O.DOUBLE, O.BXOR, 0)[1])
    res["mc_invalid_pair_every_rank"] = "ok" if all(e and e[0] == "mpi/MPIException" for e in excs) else f"excs={excs}"
    for c in comms:
        native("nativeFree", c)
    # a fresh world: rank 1's sendbuf is too short for the call. Rank 1 raises the shim's bounds message;
    # libmpjx, handed NULL by the shim, fails the world, so ranks 0, 2, 3 raise too instead of hanging.
    comms = init(np.roll(idv, 1))
    objs = []
    for r in range(P):
        so, _ = jarray(np.ones(n - 1 if r == 1 else n, np.float64))
        ro, _ = jarray(np.zeros(n, np.float64))
        objs.append((so, ro))
    excs = run(lambda r: native("nativeAllreduce", comms[r], objs[r][0], 0, objs[r][1], 0, n, O.DOUBLE, O.SUM, 0)[1])
    ok = excs[1] is not None and "too short" in excs[1][1] and all(e is not None and e[0] == "mpi/MPIException"
                                                                  for e in excs)
    res["mc_bounds_one_rank_releases_the_others"] = "ok" if ok else f"excs={excs}"
    for c in comms:
        native("nativeFree", c)
    long_lived(res, idv)
    cases.update(res)


def long_lived(res, idv, P=4, calls=8):
    """P rank threads that live across many calls (a JVM's rank threads), each call with NEW
    data in the thread's reused page-locked staging (host-direct form at the smaller sizes, the chunk
    pipeline through the same staging above 16 MiB), sizes growing and shrinking, Allreduce and Scan
    alternating — every result against the oracle. Then the staging's life: freed with each thread when it
    exits (pthread key destructor), so the count of live regions is back to zero."""
    sizes = [1001, (1 << 20) // 8, 77, (3 << 20) // 8 + 5, 5003, (20 << 20) // 8 + 9, 64, (1 << 20) // 8]
    kinds = [("nativeAllreduce", O.DOUBLE, O.SUM), ("nativeScan", O.DOUBLE, O.MAX), ("nativeAllreduce", O.INT, O.BXOR),
             ("nativeScan", O.LONG, O.SUM)]
    plan = []
    for i in range(calls):
        name, t, op = kinds[i % len(kinds)]
        n = sizes[i % len(sizes)]
        xs = [rng_vals(t, n, 3000 + 31 * i + r) for r in range(P)]
        plan.append((name, t, op, n, xs))
    got = [[None] * calls for _ in range(P)]
    errs = [None] * P
    live_during = [0]
    bar = threading.Barrier(P)

    def body(r):
        try:
            io, _ = jarray(np.roll(idv, 5))
            do, _ = jarray(np.zeros(P, np.int32))
            c, exc = native("nativeInitSmp", io, r, P, do)
            assert exc is None and c, exc
            for i, (name, t, op, n, xs) in enumerate(plan):
                so, _ = jarray(xs[r])
                ro, rv = jarray(sentinel(xs[r].dtype, n))
                _, exc = native(name, c, so, 0, ro, 0, n, t, op, 0)
                assert exc is None, (i, exc)
                got[r][i] = rv.copy()
                L.fj_free(so)
                L.fj_free(ro)
            bar.wait()
            live_during[0] = max(live_during[0], L.mpjx_jni_staging_live())
            bar.wait()
            if r == 0:  # one rank's staging goes with nativeFree, the others' when their threads exit
                native("nativeFree", c)
            else:  # the communicator alone (libmpjx directly): the thread's staging stays until it exits
                assert L.mpjx_comm_destroy(VP(c)) == 0
            bar.wait()
        except BaseException as e:  # noqa: BLE001
            errs[r] = repr(e)
            bar.abort()
    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    bad = [e for e in errs if e]
    for i, (name, t, op, n, xs) in enumerate(plan):
        exp = (O.allreduce if name == "nativeAllreduce" else O.scan)(xs, n, t, op)
        for r in range(P):
            if got[r][i] is None or not same(got[r][i], exp[r]):
                bad.append(f"call {i} ({name} {O.TYPE_NAMES[t]} n={n}) rank {r} differs")
    res["mc_long_lived_threads_reuse_staging"] = "ok" if not bad else "; ".join(bad[:6])
    live = L.mpjx_jni_staging_live()
    res["mc_staging_freed_with_threads"] = "ok" if live == 0 and live_during[0] > 0 else \
        f"live regions after the threads exited: {live} (during: {live_during[0]})"


def rccl_ranks(cases, P=3):
    """One JVM per GPU at P > 1 — the RCCL engine — played by P rank threads through the RCCL stand-in
    (MPJX_JNI_DRIVER_SO = tests/jni/libmpjx_jni_fake_standin.so: the shim and JNIEnv over the same libmpjx
    objects linked against tests/rccl/rccl_standin.hip). Rank 0's nativeUniqueId, every rank's
    nativeInitRank with it; arrays pinned through critical regions (served as copies) as in a one-rank JVM;
    Allreduce with rank-local offsets, a 20 MiB Allreduce through the chunked host pipeline, Reduce at the
    last rank, Scan, a ragged Reduce_scatter (one empty block); an invalid pair on every rank, then a valid
    call on the aborted communicators."""
    L.fj_copy_mode(1)
    uo, uv = jarray(np.zeros(128, np.int8))
    _, exc = native("nativeUniqueId", uo)
    assert exc is None, exc
    idv = uv.copy()
    res = {}

    def run(body):
        errs, out = [None] * P, [None] * P

        def th(r):
            try:
                out[r] = body(r)
            except BaseException as e:  # noqa: BLE001
                errs[r] = repr(e)
        ts = [threading.Thread(target=th, args=(r,)) for r in range(P)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=300)
        if any(t.is_alive() for t in ts):
            raise AssertionError("a rank thread hung")
        bad = [e for e in errs if e]
        if bad:
            raise AssertionError("; ".join(bad))
        return out

    def init(r):
        io, _ = jarray(idv)
        c, exc = native("nativeInitRank", r, P, 0, io)
        assert exc is None and c, exc
        return c
    comms = run(init)

    def case(name, t, op, n, call, expected, soff=lambda r: 0, roff=lambda r: 0, recv_len=None):
        xs = [rng_vals(t, n, 6000 + 13 * r + n) for r in range(P)]
        dt = np.dtype(O.NP_DTYPE[t])
        objs = []
        for r in range(P):
            so, sv = jarray(np.concatenate([sentinel(dt, soff(r)), xs[r]]))
            rl = recv_len(r) if recv_len else n
            ro, rv = jarray(sentinel(dt, roff(r) + rl + 2))
            objs.append((so, ro, rv, rl))
        excs = run(lambda r: call(r, comms[r], objs[r][0], soff(r), objs[r][1], roff(r))[1])
        exp = expected(xs)
        bad = []
        for r in range(P):
            so, ro, rv, rl = objs[r]
            if excs[r] is not None:
                bad.append(f"rank {r}: {excs[r]}")
            elif exp[r] is not None and not same(rv[roff(r):roff(r) + rl], exp[r]):
                bad.append(f"rank {r}: result differs")
            elif not same(rv[roff(r) + rl:], sentinel(dt, 2)):
                bad.append(f"rank {r}: wrote past its window")
        res[name] = "ok" if not bad else "; ".join(bad)

    n = 100003
    case("rccl_allreduce_double_sum_offsets", O.DOUBLE, O.SUM, n,
         lambda r, c, s_, so, rr, ro: native("nativeAllreduce", c, s_, so, rr, ro, n, O.DOUBLE, O.SUM, 0),
         lambda xs: O.allreduce(xs, n, O.DOUBLE, O.SUM), soff=lambda r: r + 1, roff=lambda r: 2 * r)
    nb = (20 << 20) // 8 + 7
    case("rccl_allreduce_20MiB_host_pipeline", O.DOUBLE, O.SUM, nb,
         lambda r, c, s_, so, rr, ro: native("nativeAllreduce", c, s_, so, rr, ro, nb, O.DOUBLE, O.SUM, 0),
         lambda xs: O.allreduce(xs, nb, O.DOUBLE, O.SUM))
    case("rccl_reduce_float_max_last_root", O.FLOAT, O.MAX, n,
         lambda r, c, s_, so, rr, ro: native("nativeReduce", c, s_, so, rr, ro, n, O.FLOAT, O.MAX, P - 1, 0),
         lambda xs: [O.reduce(xs, n, O.FLOAT, O.MAX, P - 1)[P - 1] if r == P - 1 else None for r in range(P)])
    case("rccl_scan_long_sum", O.LONG, O.SUM, n,
         lambda r, c, s_, so, rr, ro: native("nativeScan", c, s_, so, rr, ro, n, O.LONG, O.SUM, 0),
         lambda xs: O.scan(xs, n, O.LONG, O.SUM), roff=lambda r: 1)
    rcs = [5003, 0, 40001][:P] + [777] * max(0, P - 3)
    tot = sum(rcs)

    def rs(r, c, s_, so, rr, ro):
        rco, _ = jarray(np.array(rcs, np.int32))
        return native("nativeReduceScatter", c, s_, so, rr, ro, rco, O.INT, O.BXOR, 0)
    case("rccl_reduce_scatter_int_bxor_ragged", O.INT, O.BXOR, tot, rs,
         lambda xs: O.reduce_scatter(xs, rcs, O.INT, O.BXOR)[0], recv_len=lambda r: rcs[r])
    # an invalid (op, type) pair on every rank: every rank's own MPIException, no RCCL call made; the
    # communicators are aborted (RcclTransport::abort_world), so a valid call after it raises too, naming
    # the abort, instead of pairing with a peer's pending exchange. Each rank its own arrays: the ranks of
    # an RCCL world are separate JVMs.
    abo = [(jarray(np.zeros(16, np.float64))[0], jarray(np.zeros(16, np.float64))[0]) for _ in range(P)]
    excs = run(lambda r: native("nativeAllreduce", comms[r], abo[r][0], 0, abo[r][1], 0, 16, O.DOUBLE, O.BXOR, 0)[1])
    res["rccl_invalid_pair_every_rank"] = "ok" if all(e and e[0] == "mpi/MPIException" for e in excs) else f"{excs}"
    excs = run(lambda r: native("nativeAllreduce", comms[r], abo[r][0], 0, abo[r][1], 0, 16, O.DOUBLE, O.SUM, 0)[1])
    res["rccl_aborted_communicator_raises"] = "ok" if all(
        e and e[0] == "mpi/MPIException" and "aborted" in e[1] for e in excs) else f"{excs}"
    run(lambda r: native("nativeFree", comms[r]))
    L.fj_copy_mode(0)
    cases.update(res)


def cpu(cases):
    """Without a GPU: the exception and bounds paths that need no device."""
    n = 16
    so, sv = jarray(np.arange(n, dtype=np.float64))
    ro, rv = jarray(np.full(n, 7.0))
    _, exc = native("nativeAllreduce", 0, so, 0, ro, 0, n, O.DOUBLE, O.SUM, 0)
    ok = exc is not None and exc[0] == "mpi/MPIException" and "comm is NULL" in exc[1] and same(rv, np.full(n, 7.0))
    cases["cpu_null_comm_raises_libmpjx_text"] = "ok" if ok and release_modes(ro) == [0, 0, 1] else \
        f"exc={exc} modes={release_modes(ro)}"
    short, _ = jarray(np.zeros(n - 1, np.float64))
    _, exc = native("nativeAllreduce", 0, short, 0, ro, 0, n, O.DOUBLE, O.SUM, 0)
    ok = exc is not None and "too short" in exc[1] and release_modes(short) == [0, 0, 0]
    cases["cpu_short_array_not_pinned"] = "ok" if ok else f"exc={exc} modes={release_modes(short)}"
    _, exc = native("nativeAllreduce", 0, so, 5, ro, 0, n, O.DOUBLE, O.SUM, 0)
    cases["cpu_offset_past_end"] = "ok" if exc is not None and "too short" in exc[1] else f"exc={exc}"
    _, exc = native("nativeScan", 0, so, -1, ro, 0, 4, O.DOUBLE, O.SUM, 0)
    cases["cpu_negative_offset"] = "ok" if exc is not None and "offset" in exc[1] else f"exc={exc}"
    io, _ = jarray(np.zeros(128, np.int8))
    do, _ = jarray(np.zeros(2, np.int32))
    _, exc = native("nativeInitSmp", io, 0, 4, do)
    cases["cpu_smp_devices_too_short"] = "ok" if exc is not None and "devices[]" in exc[1] else f"exc={exc}"
    short_id, _ = jarray(np.zeros(100, np.int8))
    _, exc = native("nativeInitRank", 0, 1, 0, short_id)
    cases["cpu_short_world_id"] = "ok" if exc is not None and "128 bytes" in exc[1] else f"exc={exc}"


def latency(out, P=4, calls=int(os.environ.get("MPJX_JNI_LATENCY_CALLS", "50"))):
    """What a JVM rank thread pays per call at BASELINE configs[0] (Allreduce SUM double, 1 MiB, P = 4)
    through the shim: multicore mode (nativeInitSmp; arrays copied in and out under short critical
    regions, then the host pipeline), each of P Python threads calling back to back; median of the
    slowest rank's per-call times; the last result checked against the oracle."""
    import time

    L.fj_copy_mode(0)  # critical regions in place, as HotSpot serves primitive arrays
    n = (1 << 20) // 8
    idv = np.random.default_rng(11).integers(-128, 127, 128, dtype=np.int8)
    xs = [rng_vals(O.DOUBLE, n, 700 + r) for r in range(P)]
    times = [None] * P
    res = [None] * P
    bar = threading.Barrier(P)

    # the same call straight into libmpjx's host entry point (no shim), from pageable and from page-locked
    # host arrays: how much of the per-call time is the shim's and how much the host staging's
    mx = ctypes.CDLL(os.path.join(ROOT, "mpjexpress_amd", "lib", "libmpjx.so"))
    mx.mpjx_allreduce_host.argtypes = [VP, VP, VP, I64, ctypes.c_int, ctypes.c_int, ctypes.c_uint]
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(VP), ctypes.c_size_t, ctypes.c_uint]

    def pinned(nbytes):
        p = VP()
        assert hip.hipHostMalloc(ctypes.byref(p), nbytes, 0) == 0
        return p.value

    def run(kind):
        def body(r):
            io, _ = jarray(idv)
            do, _ = jarray(np.zeros(P, np.int32))
            c = getattr(L, J + "nativeInitSmp")(ENV, SELF, io, r, P, do)
            so, _ = jarray(xs[r])
            ro, rv = jarray(np.zeros(n))
            if kind == "pageable":
                sp, rp = L.fj_data(so), L.fj_data(ro)
            elif kind == "pinned":
                sp, rp = pinned(8 * n), pinned(8 * n)
                ctypes.memmove(sp, L.fj_data(so), 8 * n)
            f = getattr(L, J + "nativeAllreduce")
            t = []
            for i in range(calls + 5):
                bar.wait()
                t0 = time.perf_counter()
                if kind == "shim":
                    f(ENV, SELF, c, so, 0, ro, 0, n, O.DOUBLE, O.SUM, 0)
                else:
                    rc = mx.mpjx_allreduce_host(c, sp, rp, n, O.DOUBLE, O.SUM, 0)
                    assert rc == 0, rc
                t.append(time.perf_counter() - t0)
            times[r] = t[5:]
            if kind == "pinned":
                ctypes.memmove(L.fj_data(ro), rp, 8 * n)
            res[r] = rv.copy()
            bar.wait()
            getattr(L, J + "nativeFree")(ENV, SELF, c)
        ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=300)
        per_call = [max(times[r][i] for r in range(P)) for i in range(calls)]
        exp = O.allreduce(xs, n, O.DOUBLE, O.SUM)
        ok = all(same(res[r], exp[r]) for r in range(P))
        return {"median": round(float(np.median(per_call)) * 1e6, 1), "min": round(min(per_call) * 1e6, 1),
                "calls": calls, "bit_exact": ok}

    only = os.environ.get("MPJX_JNI_LATENCY_ONLY")  # one kind alone (a profiler run of its kernels)
    for key, kind in (("multicore_p4_allreduce_1MiB_us", "shim"), ("direct_mpjx_allreduce_host_pageable_us", "pageable"),
                      ("direct_mpjx_allreduce_host_pinned_us", "pinned")):
        if not only or only == kind:
            out[key] = run(kind)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "gpu"
    if mode == "latency":
        out = {"MPJX_HOST_DIRECT": os.environ.get("MPJX_HOST_DIRECT", "1"),
               "MPJX_HOST_ONCE": os.environ.get("MPJX_HOST_ONCE", "1")}
        latency(out)
        print(json.dumps(out), flush=True)
        return
    cases, vlog = {}, []
    steps = [cpu] if mode == "cpu" else [rccl_ranks] if mode == "rccl" else [single, multicore]
    for step in steps:
        try:
            step(cases)
        except BaseException as e:  # noqa: BLE001
            cases[step.__name__] = f"raised {e!r}"
        nv, log = violations()
        if nv:
            vlog.append(f"{step.__name__}: {nv} JNI rule violation(s): {log}")
    print(json.dumps({"cases": cases, "violations": vlog}), flush=True)


if __name__ == "__main__":
    main()
