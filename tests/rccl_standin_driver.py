"""Drives libmpjx's RcclTransport at P > 1 on one GPU through the RCCL stand-in (VERDICT r5 "do this" #3):
tests/rccl/libmpjx_rccl_standin.so is the SAME libmpjx objects linked against tests/rccl/rccl_standin.hip
instead of librccl; P rank THREADS of this process each form their rank of an "RCCL" world with
mpjx_comm_init_rank and run the exchange engine exactly as one process per GPU would. Run as its own
process by tests/test_gpu_rccl_standin.py (MPJX_LIB_PATH selects the stand-in build before the package
loads it).

    python tests/rccl_standin_driver.py plan|full

plan: P = 2, 3, 5, 8 x {equal 256-B blocks, ragged blocks} x {default routing, MPJX_SLOT_SKEW=4096,
      MPJX_RCCL_P2P=1 (read at init), the two-lane chunk pipeline (MPJX_PIPE_CHUNK_MIB, ncclCommSplit),
      MPJX_RCCL_NATIVE=1}: Allreduce / Reduce (root P-1) / Reduce_scatter (equal, ragged, one empty
      block) / Scan / old-collectives Allreduce / faithful Reduce / the one-shot path / Bcast, Gather,
      Scatter / big-endian mpjbuf payloads / sub-block vectors with empty blocks and count 0 / the
      chunked host pipeline (mpjx_*_host, pageable and page-locked) / one rank failing (rejected arguments,
      a bad root, an injected ncclAllToAll or ncclAllGather failure) — every
      result against the oracle bit for bit; and the RCCL calls libmpjx made, from the
      stand-in's log: ncclAllToAll's count, ncclAllToAllv's exact sendcounts / sdispls / recvcounts /
      rdispls per rank (recomputed here from the block partition, csrc/mpjx_collectives.hip Blocks::even
      and scatter_blocks), the in-place ncclAllGather (sendbuff == recvbuff + rank * bytes), the grouped
      send/recv shapes, ncclCommSplit, the init-time routing agreement, ncclAllReduce's type and op.
full: BASELINE configs[2] (Allreduce SUM double, 256 MiB per rank), configs[3] (Reduce_scatter BAND and
      Scan BXOR int32, 64 MiB) and configs[4] (Allreduce MAX float, 1 GiB, 64 MiB chunk pipeline) at P = 8
      at their full sizes, on the GPU, checked on the device (MST grouping for the double SUM, order-free
      bitwise / MAX reductions for the rest).
Prints one JSON object: {"cases": {name: "ok" | error}, "calls": {rccl call: count}}.
"""
import ctypes
import faulthandler
import json
import os
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(HERE, "rccl", "libmpjx_rccl_standin.so")
os.environ["MPJX_LIB_PATH"] = SO  # before mpjexpress_amd loads its library
sys.path[:0] = [ROOT, HERE, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402  (the checker)
from mpjexpress_amd import _lib, mpi  # noqa: E402
from mpjexpress_amd.mpi import MPI  # noqa: E402
from util import make_input, same_bits  # noqa: E402

L = _lib.lib()
L.rsi_log.restype = ctypes.c_size_t
L.rsi_log.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
L.rsi_fail_next.argtypes = [ctypes.c_int, ctypes.c_char_p]
assert L.rsi_is_standin() == 1, "not the stand-in build"
faulthandler.enable()
if os.environ.get("RSI_WATCHDOG_S"):  # a hang prints every thread's stacks, then ends the run
    import watchdog

    watchdog.arm(os.environ["RSI_WATCHDOG_S"])
NCCL_INT32, NCCL_F64 = 2, 8  # ncclDataType_t / ncclRedOp_t codes the log reports (rccl/rccl.h)
NCCL_SUM, NCCL_MAX = 0, 2
CALLS = {}


def log():
    n = L.rsi_log(None, 0)
    buf = ctypes.create_string_buffer(n)
    L.rsi_log(buf, n)
    entries = json.loads(buf.value.decode())
    for e in entries:
        CALLS[e.get("op", "error")] = CALLS.get(e.get("op", "error"), 0) + 1
    return entries


class Env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def threads(P, body):
    out, err = [None] * P, [None] * P

    def th(r):
        try:
            torch.cuda.set_device(0)
            out[r] = body(r)
        except BaseException as e:  # noqa: BLE001
            err[r] = f"{type(e).__name__}: {e}"
    ts = [threading.Thread(target=th, args=(r,), name=f"rank{r}") for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    if any(t.is_alive() for t in ts):
        raise AssertionError("a rank thread hung")
    bad = [f"rank {r}: {e}" for r, e in enumerate(err) if e]
    if bad:
        raise AssertionError("; ".join(bad))
    return out


def world(P):
    """P ranks of one stand-in RCCL world (mpjx_comm_init_rank blocks until all arrived)."""
    uid = mpi.unique_id()

    def body(r):
        h = ctypes.c_void_p()
        _lib.call("mpjx_comm_init_rank", ctypes.byref(h), P, uid, r, 0)
        c = mpi.Intracomm(h.value)
        c._kind = "rccl"
        return c
    return threads(P, body)


def free(comms):
    threads(len(comms), lambda r: comms[r].Free())


def dev(a):
    if a.dtype.names:
        a = a.view(a.dtype[0])
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t, like):
    a = t.cpu().numpy()
    return a.view(like.dtype) if like.dtype.names else a


# ---- the plan libmpjx must issue (csrc/mpjx_collectives.hip), restated for the log checks -------------
def blocks_even(n, P, esz):
    a = 256 // esz
    per = -(-n // P)
    per = -(-per // a) * a
    off = [min(n, j * per) for j in range(P)]
    ln = [min(n, o + per) - o for o in off]
    return off, ln


def scatter_plan(n, P, esz, me, skew=0):
    """(equal, sendcounts, sdispls, recvcounts, rdispls) in bytes of exchange #1 for rank me."""
    off, ln = blocks_even(n, P, esz)
    stride = -(-ln[0] * esz // 256) * 256 + (-(-skew // 256) * 256 if skew > 0 else 0)
    equal = all(x == ln[0] for x in ln) and all(off[j] == j * ln[0] for j in range(P))
    eq = equal and stride == ln[0] * esz
    sc = [0 if (j == me and not eq) else ln[j] * esz for j in range(P)]
    sd = [off[j] * esz for j in range(P)]
    rc = [0 if (j == me and not eq) else ln[me] * esz for j in range(P)]
    rd = [j * stride for j in range(P)]
    return eq, equal, sc, sd, rc, rd


def entries(lg, op, world_id=None):
    return [e for e in lg if e.get("op") == op and (world_id is None or e["world"] == world_id)]


# ---- collectives on the stand-in world ---------------------------------------------------------------
def run_case(comms, kind, op, type_, n=None, recvcounts=None, root=0, flags=0, inplace=False, seed=0):
    P = len(comms)
    dt, opx = mpi.datatype(type_), mpi.OPS[op - 1]
    total = sum(recvcounts) if recvcounts is not None else n
    sends = [make_input(type_, total, 7907 * (r + 1) + total + seed, op=op) for r in range(P)]

    def body(r):
        c = comms[r]
        c.faithful = bool(flags & O.FLAG_FAITHFUL)
        MPI.isOldSelected = bool(flags & O.FLAG_OLD)
        s = dev(sends[r])
        try:
            if kind == "reduce_scatter":
                out = dev(np.zeros(max(1, recvcounts[r]), sends[r].dtype))
                c.Reduce_scatter(s, 0, out, 0, recvcounts, dt, opx)
                return host(out, sends[r])[: recvcounts[r]]
            out = s if inplace else dev(np.zeros(max(1, n), sends[r].dtype))
            if kind == "allreduce":
                c.Allreduce(s, 0, out, 0, n, dt, opx)
            elif kind == "reduce":
                c.Reduce(s, 0, out, 0, n, dt, opx, root)
            elif kind == "scan":
                c.Scan(s, 0, out, 0, n, dt, opx)
            elif kind == "bcast":
                c.Bcast(s, 0, n, dt, root)
                out = s
            return host(out, sends[r])[:n]
        finally:
            c.faithful = False
    MPI.isOldSelected = bool(flags & O.FLAG_OLD)
    try:
        got = threads(P, body)
    finally:
        MPI.isOldSelected = False
    if kind == "allreduce":
        exp = O.allreduce(sends, n, type_, op, flags=flags)
    elif kind == "reduce":
        exp = O.reduce(sends, n, type_, op, root, flags=flags)
    elif kind == "scan":
        exp = O.scan(sends, n, type_, op, flags=flags)
    elif kind == "bcast":
        exp = [sends[root]] * P
    else:
        exp = O.reduce_scatter(sends, list(recvcounts), type_, op, flags=flags)[0]
    for r in range(P):
        if kind == "reduce" and r != root and not (flags & O.FLAG_FAITHFUL):
            continue
        m = recvcounts[r] if kind == "reduce_scatter" else n
        if not same_bits(type_, op, got[r], np.asarray(exp[r])[:m]):
            raise AssertionError(f"{kind} {O.OP_NAMES[op]} {O.TYPE_NAMES[type_]} P={P} rank {r}: differs from the oracle")


def gather_scatter(comms, n=3001):
    P = len(comms)
    xs = [np.arange(n, dtype=np.int64) * (r + 3) for r in range(P)]
    root = P - 1

    def body(r):
        c = comms[r]
        s = dev(xs[r])
        g = torch.zeros(n * P, dtype=torch.int64, device="cuda")
        c.Gather(s, 0, n, g, 0, n, MPI.LONG, root)
        sc = torch.zeros(n, dtype=torch.int64, device="cuda")
        c.Scatter(g, 0, n, sc, 0, n, MPI.LONG, root)
        return g.cpu().numpy(), sc.cpu().numpy()
    got = threads(P, body)
    assert np.array_equal(got[root][0], np.concatenate(xs)), "gather"
    for r in range(P):
        assert np.array_equal(got[r][1], xs[r]), f"scatter rank {r}"


def split_create(comms, n=40961):
    """mpi.py's Split / Create on an RCCL world (Intracomm._kind "rccl"): the colors, keys and devices
    gathered and broadcast over the parent (Gather + Bcast through RcclTransport), the leader's RCCL unique
    id gathered to every member, one new RCCL world per group (mpjx_comm_init_rank), then an Allreduce on
    each — new ranks ordered by key, ties by parent rank (src/mpi/PureIntracomm.java:201-280, 302-309)."""
    P = len(comms)
    xs = [make_input(O.DOUBLE, n, 5100 + r, specials=False) for r in range(P)]

    def body(r):
        sub = comms[r].Split(r % 2, -r)
        out = torch.zeros(n, dtype=torch.float64, device="cuda")
        sub.Allreduce(dev(xs[r]), 0, out, 0, n, MPI.DOUBLE, MPI.SUM)
        res = (sub.Rank(), sub.Size(), out.cpu().numpy())
        sub.Free()
        grp = [P - 1, 0] if P > 2 else [1, 0]
        cr = comms[r].Create(grp)
        cres = None
        if cr is not None:
            o2 = torch.zeros(n, dtype=torch.float64, device="cuda")
            cr.Allreduce(dev(xs[r]), 0, o2, 0, n, MPI.DOUBLE, MPI.MAX)
            cres = (cr.Rank(), o2.cpu().numpy())
            cr.Free()
        return res, cres
    got = threads(P, body)
    for color in (0, 1):
        members = sorted([r for r in range(P) if r % 2 == color], key=lambda r: (-r, r))
        if not members:
            continue
        exp = O.allreduce([xs[r] for r in members], n, O.DOUBLE, O.SUM)
        for i, r in enumerate(members):
            rk, sz, out = got[r][0]
            assert (rk, sz) == (i, len(members)), (color, r, rk, sz)
            assert np.array_equal(out.view(np.uint64), exp[i].view(np.uint64)), ("split", color, r)
    grp = [P - 1, 0] if P > 2 else [1, 0]
    exp = O.allreduce([xs[r] for r in grp], n, O.DOUBLE, O.MAX)
    for r in range(P):
        c = got[r][1]
        if r not in grp:
            assert c is None, r
            continue
        i = grp.index(r)
        assert c[0] == i and np.array_equal(c[1].view(np.uint64), exp[i].view(np.uint64)), ("create", r)


def _bswap(a):
    return a.byteswap() if not a.dtype.names else a.view(a.dtype[0]).byteswap().view(a.dtype)


BE_CASES = [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.BXOR, O.INT), (O.PROD, O.LONG), (O.MINLOC, O.DOUBLE2)]


def big_endian(comms, n=70001):
    """mpjbuf payloads on the RCCL world (MPJX_FLAG_SEND_BIG_ENDIAN | MPJX_FLAG_RECV_BIG_ENDIAN, §8 f4):
    the byte swaps ride the combine kernels on both sides of RcclTransport's exchanges. Allreduce, Reduce
    (root P-1), ragged Reduce_scatter with an empty block and Scan through the C ABI, past the one-shot
    limit; the results swapped back must be the oracle's on the native values."""
    P = len(comms)
    fl = 0x4 | 0x8 | 0x10  # send BE, recv BE, blocking
    rc = [(n // P) + (1 if r < n % P else 0) for r in range(P)]
    rc[-1] += rc[0]
    rc[0] = 0
    root = P - 1
    for op, t in BE_CASES:
        sends = [make_input(t, n, 311 + 7 * r + t, op=op) for r in range(P)]
        ins = [_bswap(s) for s in sends]

        def body(r):
            h, s = comms[r].handle, dev(ins[r])
            outs = {}
            for name, fn, cnt in (("ar", "mpjx_allreduce", n), ("scan", "mpjx_scan", n)):
                d = dev(np.zeros_like(ins[r]))
                _lib.check(getattr(L, fn)(h, s.data_ptr(), d.data_ptr(), cnt, t, op, fl, None), name)
                outs[name] = d
            d = dev(np.zeros_like(ins[r]))
            _lib.check(L.mpjx_reduce(h, s.data_ptr(), d.data_ptr(), n, t, op, root, fl, None), "reduce")
            outs["red"] = d
            d = dev(np.zeros(max(rc[r], 1), ins[r].dtype))
            _lib.check(L.mpjx_reduce_scatter(h, s.data_ptr(), d.data_ptr(), (ctypes.c_int64 * P)(*rc), t, op, fl,
                                             None), "reduce_scatter")
            outs["rs"] = d
            _lib.check(L.mpjx_comm_synchronize(h), "sync")
            return {k: _bswap(host(v, ins[r])) for k, v in outs.items()}
        got = threads(P, body)
        exp_ar = O.allreduce(sends, n, t, op)
        exp_sc = O.scan(sends, n, t, op)
        exp_red = O.reduce(sends, n, t, op, root)[root]
        exp_rs = O.reduce_scatter(sends, rc, t, op)[0]
        for r in range(P):
            tag = f"{O.OP_NAMES[op]} {O.TYPE_NAMES[t]} P={P} rank {r}"
            assert same_bits(t, op, got[r]["ar"], exp_ar[r]), tag + " allreduce"
            assert same_bits(t, op, got[r]["scan"], exp_sc[r]), tag + " scan"
            assert r != root or same_bits(t, op, got[r]["red"], exp_red), tag + " reduce"
            assert same_bits(t, op, got[r]["rs"][:rc[r]], exp_rs[r]), tag + " reduce_scatter"


def tiny_exchange(comms):
    """The exchange engine with the one-shot path off (MPJX_ONESHOT_KIB=0) on vectors shorter than one
    256-B block per rank: block 0 holds everything, every other block is empty — ncclAllToAllv with zero
    counts to and from every rank but one, a grouped all-gather with one sender — and count 0 (nothing
    issued, nothing written). Returns the exchange #1 mismatches against the block plan."""
    P = len(comms)
    msgs = []
    with Env(MPJX_ONESHOT_KIB=0):
        for n in sorted({1, 3, max(1, P - 1)}):
            L.rsi_log_clear()
            run_case(comms, "allreduce", O.SUM, O.DOUBLE, n=n, seed=20 + n)
            lg = log()
            for me in range(P):
                eq, equal, sc, sd, rc, rd = scatter_plan(n, P, 8, me)
                v = [e for e in lg if e.get("rank") == me and e.get("op") == "AllToAllv"]
                if len(v) != 1 or (v[0]["sendcounts"], v[0]["sdispls"], v[0]["recvcounts"], v[0]["rdispls"]) != \
                        (sc, sd, rc, rd):
                    msgs.append(f"n={n} rank {me}: {v} != {(sc, sd, rc, rd)}")
            run_case(comms, "scan", O.MAX, O.FLOAT, n=n, seed=30 + n)
            run_case(comms, "reduce", O.PROD, O.LONG, n=n, root=P - 1, seed=40 + n)
        run_case(comms, "reduce_scatter", O.BOR, O.INT, recvcounts=[0] * (P - 1) + [5])
        L.rsi_log_clear()
        run_case(comms, "allreduce", O.SUM, O.DOUBLE, n=0)
        run_case(comms, "reduce_scatter", O.SUM, O.DOUBLE, recvcounts=[0] * P)
        issued = [e for e in log() if e.get("op") not in (None, "CommInitRank")]
        if issued:
            msgs.append(f"count 0 issued {issued[:4]}")
    return msgs


def host_calls(comms):
    """The host-resident entry points (mpjx_*_host, the JNI shim's path for Java arrays) over RcclTransport
    with the chunk pipeline forced small (MPJX_HOST_CHUNK_MIB=1, so 3+ chunks and a ragged last one):
    pageable operands (the drain thread's D2H copies) and page-locked ones from mpjx_host_alloc (straight
    D2H on the copy stream); Allreduce, Reduce at the last rank, Scan, Reduce_scatter with an empty block.
    RCCL worlds take the staged form (host form 1). Returns the mismatches."""
    P = len(comms)
    msgs = []
    n = (3 << 20) // 8 + 1234
    rc = [(n // P) + (1 if r < n % P else 0) for r in range(P)]
    rc[-1] += rc[0]
    rc[0] = 0
    pinned = []

    def pin(a):
        p = ctypes.c_void_p()
        _lib.call("mpjx_host_alloc", ctypes.byref(p), max(1, a.nbytes))
        pinned.append(p.value)
        v = np.frombuffer((ctypes.c_uint8 * max(1, a.nbytes)).from_address(p.value), dtype=a.dtype, count=a.size)
        v[:] = a
        return v
    try:
        with Env(MPJX_HOST_CHUNK_MIB=1):
            for mem in ("pageable", "pinned"):
                for kind, op, t in (("allreduce", O.SUM, O.DOUBLE), ("reduce", O.MAX, O.FLOAT),
                                    ("scan", O.PROD, O.DOUBLE), ("reduce_scatter", O.BXOR, O.INT)):
                    sends = [make_input(t, n, 4400 + 31 * r + t, op=op) for r in range(P)]
                    ins = [pin(s) if mem == "pinned" else s for s in sends]
                    outs = [np.zeros(max(1, rc[r] if kind == "reduce_scatter" else n), sends[r].dtype) for r in range(P)]
                    outs = [pin(o) if mem == "pinned" else o for o in outs]
                    root = P - 1

                    def body(r):
                        h, s, d = comms[r].handle, ins[r].ctypes.data, outs[r].ctypes.data
                        if kind == "allreduce":
                            _lib.call("mpjx_allreduce_host", h, s, d, n, t, op, 0)
                        elif kind == "reduce":
                            _lib.call("mpjx_reduce_host", h, s, d, n, t, op, root, 0)
                        elif kind == "scan":
                            _lib.call("mpjx_scan_host", h, s, d, n, t, op, 0)
                        else:
                            _lib.call("mpjx_reduce_scatter_host", h, s, d, (ctypes.c_int64 * P)(*rc), t, op, 0)
                        form = ctypes.c_int()
                        _lib.call("mpjx_comm_last_host_form", h, ctypes.byref(form))
                        return form.value
                    forms = threads(P, body)
                    if kind == "allreduce":
                        exp = O.allreduce(sends, n, t, op)
                    elif kind == "reduce":
                        exp = [O.reduce(sends, n, t, op, root)[root] if r == root else None for r in range(P)]
                    elif kind == "scan":
                        exp = O.scan(sends, n, t, op)
                    else:
                        exp = O.reduce_scatter(sends, rc, t, op)[0]
                    for r in range(P):
                        m = rc[r] if kind == "reduce_scatter" else n
                        if exp[r] is not None and not same_bits(t, op, outs[r][:m], np.asarray(exp[r])[:m]):
                            msgs.append(f"{mem} {kind} rank {r}: differs from the oracle")
                    if forms != [1] * P:
                        msgs.append(f"{mem} {kind}: host forms {forms}, expected staged (1) on every rank")
    finally:
        for p in pinned:
            _lib.call("mpjx_host_free", p)
    return msgs


FAILURES = {  # how rank 1 fails its part of an Allreduce / Reduce, and the status it gets
    "rejects": -2,          # BXOR on double: MPJX_ERR_OP_TYPE before any RCCL call (reject())
    "bad_root": -1,         # Reduce with root P: MPJX_ERR_ARG before any RCCL call (not a reject())
    "alltoall_fails": -4,   # its ncclAllToAll fails (injected): MPJX_ERR_RCCL, nothing exchanged
    "allgather_fails": -4,  # its ncclAllGather fails after its exchange #1 and combine: mid-collective
}


def rank_fails(P, how):
    """Rank 1 fails its part of a collective at P > 1 (FAILURES) while the other ranks make theirs. Its
    communicator is aborted (RcclTransport::abort_world / call_failed / failed_call), so its next call
    fails with MPJX_ERR_RCCL instead of pairing with the peers' pending exchange. Here the stand-in's
    ncclCommAbort also ends the peers' waits (real RCCL leaves them waiting until MPJX_RCCL_TIMEOUT_S),
    so they fail their call with MPJX_ERR_RCCL and abort too; every later call on every rank fails the
    same way, one ncclCommAbort per rank, and every communicator can still be destroyed. Returns the
    mismatches."""
    comms = world(P)
    L.rsi_log_clear()
    n = 65536 * P  # equal 256-B blocks: ncclAllToAll, combine, in-place ncclAllGather
    xs = [make_input(O.DOUBLE, n, 900 + r, op=O.SUM) for r in range(P)]
    if how == "alltoall_fails":
        L.rsi_fail_next(1, b"AllToAll")
    elif how == "allgather_fails":
        L.rsi_fail_next(1, b"AllGather")

    def body(r):
        h, s, d = comms[r].handle, dev(xs[r]), dev(np.zeros(n))
        res = []
        for first in (True, False):
            if first and how == "bad_root":
                rc = L.mpjx_reduce(h, s.data_ptr(), d.data_ptr(), n, O.DOUBLE, O.SUM, P if r == 1 else 0, 0x10, None)
            else:
                op = O.BXOR if (first and how == "rejects" and r == 1) else O.SUM
                rc = L.mpjx_allreduce(h, s.data_ptr(), d.data_ptr(), n, O.DOUBLE, op, 0x10, None)
            res.append((rc, L.mpjx_last_error().decode(errors="replace") if rc else ""))
        return res
    try:
        got = threads(P, body)
    finally:
        free(comms)
        L.rsi_fail_next(-1, b"")
    msgs = []
    for r, ((rc1, m1), (rc2, m2)) in enumerate(got):
        want1 = FAILURES[how] if r == 1 else -4  # the peers: MPJX_ERR_RCCL
        if rc1 != want1:
            msgs.append(f"rank {r}: first call {rc1} ({m1}), expected {want1}")
        if rc2 != -4 or "aborted" not in m2:
            msgs.append(f"rank {r}: later call {rc2} ({m2}), expected MPJX_ERR_RCCL on an aborted communicator")
    lg = log()
    aborts = entries(lg, "CommAbort")
    if sorted(e["rank"] for e in aborts) != list(range(P)):
        msgs.append(f"ncclCommAbort calls {aborts}")
    if how.endswith("_fails") and len(entries(lg, "InjectedFailure")) != 1:
        msgs.append(f"injected failures {entries(lg, 'InjectedFailure')}")
    ended = [e for e in lg if "error" in e]  # the peers' waits this world's abort ended: expected here
    if any("world aborted" not in e["error"] for e in ended):
        msgs.append(f"waits ended otherwise: {ended}")
    CALLS["error"] = CALLS.get("error", 0) - len(ended)
    if not CALLS["error"]:
        del CALLS["error"]
    return msgs


def plan(cases):
    for P in (2, 3, 5, 8):
        L.rsi_log_clear()  # the previous world's calls are not this world's
        esz = 8
        n_eq = 65536 * P            # 512 KiB per block: past the one-shot limit, equal 256-B blocks
        n_rag = n_eq + 4099         # ragged: the last block short
        # -- default routing: AllToAll + in-place AllGather (equal), AllToAllv + grouped send/recv (ragged)
        comms = world(P)
        lg = log()
        agree = entries(lg, "AllReduce")
        cases[f"P{P}_init_agreement"] = "ok" if len(agree) == P and all(
            e["count"] == 4 and e["datatype"] == NCCL_INT32 and e["redop"] == NCCL_MAX for e in agree) else \
            f"init AllReduce calls: {agree}"
        wid = agree[0]["world"] if agree else -1
        for name, n in (("equal", n_eq), ("ragged", n_rag)):
            L.rsi_log_clear()
            try:
                run_case(comms, "allreduce", O.SUM, O.DOUBLE, n=n, seed=1)
                lg = log()
                errs = [e for e in lg if "error" in e]
                msgs = []
                for me in range(P):
                    eq, equal, sc, sd, rc, rd = scatter_plan(n, P, esz, me)
                    mine = [e for e in lg if e.get("rank") == me and e.get("world") == wid]
                    ops = [e["op"] for e in mine]
                    if eq:
                        a2a = [e for e in mine if e["op"] == "AllToAll"]
                        ag = [e for e in mine if e["op"] == "AllGather"]
                        if ops != ["AllToAll", "AllGather"] or a2a[0]["count"] != sc[0] or a2a[0]["elem"] != 1:
                            msgs.append(f"rank {me}: {mine}")
                        elif not (ag[0]["in_place"] and ag[0]["send_minus_recv"] == me * ag[0]["bytes"]
                                  and ag[0]["bytes"] == blocks_even(n, P, esz)[1][0] * esz):
                            msgs.append(f"rank {me}: all-gather not in place at block {me}: {ag[0]}")
                    else:
                        v = [e for e in mine if e["op"] == "AllToAllv"]
                        if ops != ["AllToAllv", "Group"]:
                            msgs.append(f"rank {me}: calls {ops}")
                        elif (v[0]["sendcounts"], v[0]["sdispls"], v[0]["recvcounts"], v[0]["rdispls"]) != (sc, sd, rc, rd):
                            msgs.append(f"rank {me}: AllToAllv {v[0]} != {(sc, sd, rc, rd)}")
                        else:  # the ragged all-gather: my block to every peer, every peer's block from it
                            off, ln = blocks_even(n, P, esz)
                            g = [e for e in mine if e["op"] == "Group"][0]
                            want_s = [[j, ln[me] * esz] for j in range(P) if j != me and ln[me] > 0]
                            want_r = [[j, ln[j] * esz] for j in range(P) if j != me and ln[j] > 0]
                            if g["sends"] != want_s or g["recvs"] != want_r:
                                msgs.append(f"rank {me}: all-gather group {g} != {want_s}, {want_r}")
                cases[f"P{P}_allreduce_{name}_calls"] = "ok" if not msgs and not errs else "; ".join(msgs + [str(errs)])
            except Exception as e:  # noqa: BLE001
                cases[f"P{P}_allreduce_{name}_calls"] = repr(e)[:800]
        # -- skewed input slots: equal blocks through ncclAllToAllv with rdispls j * (block + 4 KiB)
        L.rsi_log_clear()
        try:
            with Env(MPJX_SLOT_SKEW=4096):
                run_case(comms, "allreduce", O.SUM, O.DOUBLE, n=n_eq, seed=2)
            lg = log()
            msgs = []
            for me in range(P):
                eq, equal, sc, sd, rc, rd = scatter_plan(n_eq, P, esz, me, skew=4096)
                v = [e for e in lg if e.get("rank") == me and e["op"] == "AllToAllv"]
                if eq or len(v) != 1 or (v[0]["sendcounts"], v[0]["sdispls"], v[0]["recvcounts"], v[0]["rdispls"]) != (sc, sd, rc, rd):
                    msgs.append(f"rank {me}: {v}")
            cases[f"P{P}_slot_skew_alltoallv"] = "ok" if not msgs else "; ".join(msgs)
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_slot_skew_alltoallv"] = repr(e)[:800]
        # -- every other collective of the path on the exchange engine, against the oracle
        rag = [(37 * r + 5) % 23 * 977 + 40000 for r in range(P)]
        rag[P // 2] = 0
        big = 70001
        for name, kw in (
                ("reduce_root_last", dict(kind="reduce", op=O.SUM, type_=O.DOUBLE, n=n_rag, root=P - 1)),
                ("reduce_faithful", dict(kind="reduce", op=O.PROD, type_=O.DOUBLE, n=n_rag, root=0, flags=O.FLAG_FAITHFUL)),
                ("allreduce_old", dict(kind="allreduce", op=O.SUM, type_=O.FLOAT, n=n_rag, flags=O.FLAG_OLD)),
                ("allreduce_inplace", dict(kind="allreduce", op=O.MAX, type_=O.FLOAT, n=n_rag, inplace=True)),
                ("allreduce_band_int", dict(kind="allreduce", op=O.BAND, type_=O.INT, n=n_eq)),
                ("allreduce_maxloc_double2", dict(kind="allreduce", op=O.MAXLOC, type_=O.DOUBLE2, n=big)),
                ("reduce_scatter_equal", dict(kind="reduce_scatter", op=O.BAND, type_=O.INT, recvcounts=[big] * P)),
                ("reduce_scatter_ragged_empty", dict(kind="reduce_scatter", op=O.SUM, type_=O.DOUBLE, recvcounts=rag)),
                ("reduce_scatter_faithful", dict(kind="reduce_scatter", op=O.SUM, type_=O.INT, recvcounts=rag,
                                                 flags=O.FLAG_FAITHFUL)),
                ("scan_bxor", dict(kind="scan", op=O.BXOR, type_=O.INT, n=n_rag)),
                ("scan_sum_double", dict(kind="scan", op=O.SUM, type_=O.DOUBLE, n=n_rag)),
                ("oneshot_allreduce", dict(kind="allreduce", op=O.SUM, type_=O.DOUBLE, n=1001)),
                ("oneshot_reduce", dict(kind="reduce", op=O.MIN, type_=O.FLOAT, n=1001, root=P - 1)),
                ("oneshot_scan", dict(kind="scan", op=O.PROD, type_=O.DOUBLE, n=1001)),
                ("bcast", dict(kind="bcast", op=O.SUM, type_=O.LONG, n=n_rag, root=P - 1))):
            try:
                run_case(comms, **kw)
                cases[f"P{P}_{name}"] = "ok"
            except Exception as e:  # noqa: BLE001
                cases[f"P{P}_{name}"] = repr(e)[:800]
        try:
            gather_scatter(comms)
            cases[f"P{P}_gather_scatter"] = "ok"
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_gather_scatter"] = repr(e)[:800]
        try:
            split_create(comms)
            cases[f"P{P}_split_create_rccl_subworlds"] = "ok"
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_split_create_rccl_subworlds"] = repr(e)[:800]
        try:
            big_endian(comms)
            cases[f"P{P}_big_endian_mpjbuf"] = "ok"
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_big_endian_mpjbuf"] = repr(e)[:800]
        try:
            msgs = tiny_exchange(comms)
            cases[f"P{P}_tiny_and_empty_exchange"] = "ok" if not msgs else "; ".join(msgs)[:800]
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_tiny_and_empty_exchange"] = repr(e)[:800]
        try:
            msgs = host_calls(comms)
            cases[f"P{P}_host_pipeline_chunked"] = "ok" if not msgs else "; ".join(msgs)[:800]
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_host_pipeline_chunked"] = repr(e)[:800]
        # -- the two-lane chunk pipeline: 1 MiB chunks, ragged last chunk, twice (the split lane is reused)
        L.rsi_log_clear()
        try:
            nf = (8 << 20) // 4 + 12345
            with Env(MPJX_PIPE_CHUNK_MIB=1):
                run_case(comms, "allreduce", O.MAX, O.FLOAT, n=nf, seed=3)
                run_case(comms, "allreduce", O.SUM, O.DOUBLE, n=(3 << 20) // 8 + 7, seed=4)
            lg = log()
            sp = entries(lg, "CommSplit")
            lane = {e["new_world"] for e in sp}
            ok = len(sp) == P and all(e["color"] == 0 and e["key"] == e["rank"] and e["new_rank"] == e["rank"]
                                      for e in sp) and len(lane) == 1
            nch = -(-nf // ((1 << 20) // 4))
            ag2 = [e for e in lg if e.get("op") in ("AllGather", "Group") and e["world"] in lane]
            x1 = [e for e in lg if e.get("op") in ("AllToAll", "AllToAllv") and e["world"] == wid]
            cases[f"P{P}_pipeline_two_lanes"] = "ok" if ok and len(ag2) >= P * nch and len(x1) >= P * nch and \
                not any("error" in e for e in lg) else f"split={sp} lane-2 gathers={len(ag2)} exchanges={len(x1)} nch={nch}"
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_pipeline_two_lanes"] = repr(e)[:800]
        free(comms)
        # -- MPJX_RCCL_P2P=1 (read at init): grouped ncclSend/ncclRecv for every exchange, no collectives
        with Env(MPJX_RCCL_P2P=1):
            comms = world(P)
        L.rsi_log_clear()
        try:
            run_case(comms, "allreduce", O.SUM, O.DOUBLE, n=n_eq, seed=5)
            run_case(comms, "allreduce", O.SUM, O.DOUBLE, n=n_rag, seed=6)
            run_case(comms, "reduce_scatter", O.SUM, O.DOUBLE, recvcounts=rag)
            run_case(comms, "scan", O.MIN, O.DOUBLE, n=n_rag)
            lg = log()
            kinds = {e["op"] for e in lg if "op" in e}
            groups = entries(lg, "Group")
            cases[f"P{P}_p2p_grouped_only"] = "ok" if kinds == {"Group"} and groups else f"calls {sorted(kinds)}"
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_p2p_grouped_only"] = repr(e)[:800]
        free(comms)
        # -- MPJX_RCCL_NATIVE=1 (read at init): one ncclAllReduce where the result is order-free
        with Env(MPJX_RCCL_NATIVE=1):
            comms = world(P)
        L.rsi_log_clear()
        try:
            run_case(comms, "allreduce", O.SUM, O.INT, n=n_rag, seed=7)
            run_case(comms, "allreduce", O.SUM, O.DOUBLE, n=n_rag, seed=8)
            lg = log()
            ar = [e for e in entries(lg, "AllReduce")]
            ints = [e for e in ar if e["datatype"] == NCCL_INT32 and e["redop"] == NCCL_SUM and e["count"] == n_rag]
            dbl = [e for e in ar if e["datatype"] == NCCL_F64]
            want_dbl = P if P == 2 else 0  # double SUM only at P <= 2 (one commutative add per element)
            x1 = entries(lg, "AllToAllv") + entries(lg, "AllToAll")
            ok = len(ints) == P and len(dbl) == want_dbl and (P == 2 or len(x1) == P)
            cases[f"P{P}_rccl_native_routing"] = "ok" if ok else f"int={len(ints)} double={len(dbl)} exch={len(x1)}"
        except Exception as e:  # noqa: BLE001
            cases[f"P{P}_rccl_native_routing"] = repr(e)[:800]
        free(comms)
        for how in FAILURES:
            try:
                msgs = rank_fails(P, how)
                cases[f"P{P}_rank_{how}_comm_aborted"] = "ok" if not msgs else "; ".join(msgs)[:800]
            except Exception as e:  # noqa: BLE001
                cases[f"P{P}_rank_{how}_comm_aborted"] = repr(e)[:800]


def full(cases):
    """configs[2] / [3] / [4] at P = 8 at full size, checked on the device."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth as S  # the bench's counter streams

    P = 8
    comms = world(P)
    try:
        # configs[2]: Allreduce SUM double, 256 MiB per rank (equal 32 MiB blocks: AllToAll + AllGather)
        n = (256 << 20) // 8
        L.rsi_log_clear()
        sends = [S.uniform_torch(n, S.seed(2, r), torch.device("cuda", 0)) for r in range(P)]

        def mst(vals, lo, hi, root):
            if lo == hi:
                return vals[lo]
            mid = (lo + hi) // 2
            if root <= mid:
                own, other = mst(vals, lo, mid, root), mst(vals, mid + 1, hi, hi)
            else:
                own, other = mst(vals, mid + 1, hi, root), mst(vals, lo, mid, lo)
            return other + own
        exp = mst(sends, 0, P - 1, 0)
        outs = [torch.empty_like(s) for s in sends]
        threads(P, lambda r: comms[r].Allreduce(sends[r], 0, outs[r], 0, n, MPI.DOUBLE, MPI.SUM))
        bad = [r for r in range(P) if not torch.equal(outs[r].view(torch.int64), exp.view(torch.int64))]
        lg = log()
        calls = sorted({e["op"] for e in lg if e.get("op")})
        cases["P8_configs2_allreduce_sum_double_256MiB"] = "ok" if not bad and calls == ["AllGather", "AllToAll"] \
            else f"ranks differing {bad}, calls {calls}"
        del sends, outs, exp
        # configs[3]: Reduce_scatter BAND + Scan BXOR int32, 64 MiB per rank
        n = (64 << 20) // 4
        g = [torch.randint(-2 ** 31, 2 ** 31 - 1, (n,), dtype=torch.int32, device="cuda",
                           generator=torch.Generator("cuda").manual_seed(40 + r)) for r in range(P)]
        band = [x | torch.roll(x, 1) | torch.roll(x, 2) for x in g]  # dense ones: the AND keeps bits
        rc = [n // P] * P
        outs = [torch.empty(n // P, dtype=torch.int32, device="cuda") for _ in range(P)]
        threads(P, lambda r: comms[r].Reduce_scatter(band[r], 0, outs[r], 0, rc, MPI.INT, MPI.BAND))
        tot = band[0].clone()
        for x in band[1:]:
            tot &= x
        bad = [r for r in range(P) if not torch.equal(outs[r], tot[r * (n // P):(r + 1) * (n // P)])]
        cases["P8_configs3_reduce_scatter_band_int32_64MiB"] = "ok" if not bad else f"ranks differing {bad}"
        del band, outs, tot
        outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(P)]
        threads(P, lambda r: comms[r].Scan(g[r], 0, outs[r], 0, n, MPI.INT, MPI.BXOR))
        acc = torch.zeros_like(g[0])
        bad = []
        for r in range(P):
            acc ^= g[r]
            if not torch.equal(outs[r], acc):
                bad.append(r)
        cases["P8_configs3_scan_bxor_int32_64MiB"] = "ok" if not bad else f"ranks differing {bad}"
        del g, outs, acc
        # configs[4]: Allreduce MAX float, 1 GiB per rank, the 64 MiB chunk pipeline (bench's rccl_pipe64)
        n = (1 << 30) // 4
        L.rsi_log_clear()
        xs = [torch.rand(n, dtype=torch.float32, device="cuda", generator=torch.Generator("cuda").manual_seed(90 + r)) - 0.5
              for r in range(P)]
        outs = [torch.empty_like(x) for x in xs]
        with Env(MPJX_PIPE_CHUNK_MIB=64):
            threads(P, lambda r: comms[r].Allreduce(xs[r], 0, outs[r], 0, n, MPI.FLOAT, MPI.MAX))
        mx = xs[0].clone()
        for x in xs[1:]:
            torch.maximum(mx, x, out=mx)
        bad = [r for r in range(P) if not torch.equal(outs[r], mx)]
        lg = log()
        nsplit = len(entries(lg, "CommSplit"))
        cases["P8_configs4_allreduce_max_float_1GiB_pipelined"] = "ok" if not bad and nsplit == P and \
            not any("error" in e for e in lg) else f"ranks differing {bad}, splits {nsplit}"
        del xs, outs, mx
    finally:
        free(comms)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "plan"
    cases = {}
    try:
        (plan if mode == "plan" else full)(cases)
    except BaseException as e:  # noqa: BLE001
        cases[mode] = f"raised {e!r}"[:2000]
    print(json.dumps({"cases": cases, "calls": CALLS}), flush=True)


if __name__ == "__main__":
    main()
