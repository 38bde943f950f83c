"""A second, independent restatement of the reference collectives — P ranks as threads exchanging
messages through queues, each running the per-rank program of src/mpi/PureIntracomm.java with a
typed Op that keeps its own `arr` exactly as the generated classes do (createInitialBuffer copies the
rank's buffer into arr, perform does arr[i] = buf[i] (op) arr[i] after each recv, getResultant copies
arr back; src/mpi/SumDouble.java:49-67). The C oracle restates the same algorithms as fold orders
over P inputs; here they run as the message pattern itself. The two must agree bit for bit for
float and double — this is what pins the oracle's float combine ORDERS beyond source reading of
the order tables (no JVM exists in this image to run the reference).

  MST_Reduce      src/mpi/PureIntracomm.java:1943-1992 (recursive halving, sub-root sends to root)
  Reduce          :1923-1941 (arraycopy send -> recv, then MST_Reduce on recv)
  Allreduce       :2168-2185 (Reduce to 0 + Bcast: every rank holds rank 0's result)
  FT_Reduce       :1994-2057 (root folds ranks 0..P-1, skipping itself, in ascending order)
  FT_Allreduce    :2187-2314 (every rank does the FT fold; EXOTIC_ALLREDUCE is false, :2059)
  Scan            :2495-2545 (rank r folds ranks 0..r-1 in ascending order)
  BKT_Reduce_scatter :2377-2439 (the ring as written; pins the FAITHFUL defect A9, and A3 no-ops)
"""
import queue
import threading

import numpy as np
import pytest

import oracle as O


class Net:
    """Point-to-point channels (src, dst, tag) -> FIFO, like the device's matched send/recv."""

    def __init__(self):
        self.lock = threading.Lock()
        self.q = {}

    def _chan(self, key):
        with self.lock:
            return self.q.setdefault(key, queue.Queue())

    def send(self, buf, src, dst, tag):
        self._chan((src, dst, tag)).put(buf.copy())

    def recv(self, buf, src, dst, tag):
        buf[:] = self._chan((src, dst, tag)).get(timeout=30)


def combine(op, x, acc):
    """One element-wise step acc = x (op) acc with the Java rules (typed classes, MAX/MIN by compare)."""
    if op == O.SUM:
        return x + acc
    if op == O.PROD:
        return x * acc
    if op == O.MAX:
        return np.where(x > acc, x, acc)
    if op == O.MIN:
        return np.where(x < acc, x, acc)
    raise ValueError(op)


class TypedOp:
    """opx of src/mpi/<Op><Type>.java: arr is the op's private accumulator."""

    def __init__(self, op):
        self.op, self.arr = op, None

    def createInitialBuffer(self, buf):
        self.arr = buf.copy()

    def perform(self, buf):
        self.arr = combine(self.op, buf, self.arr)

    def getResultant(self, buf):
        buf[:] = self.arr


def mst_reduce(net, me, buf, op, root, left, right, tag=1):
    if left == right:
        return
    mid = (left + right) // 2
    srce = right if root <= mid else left
    if me <= mid and root <= mid:
        mst_reduce(net, me, buf, op, root, left, mid, tag)
    elif me <= mid and root > mid:
        mst_reduce(net, me, buf, op, srce, left, mid, tag)
    elif me > mid and root <= mid:
        mst_reduce(net, me, buf, op, srce, mid + 1, right, tag)
    else:
        mst_reduce(net, me, buf, op, root, mid + 1, right, tag)
    if me == srce:
        net.send(buf, me, root, tag)
    if me == root:
        opx = TypedOp(op)
        opx.createInitialBuffer(buf)
        net.recv(buf, srce, me, tag)
        opx.perform(buf)
        opx.getResultant(buf)


def run_ranks(P, program):
    out, err = [None] * P, []
    net = Net()

    def body(r):
        try:
            out[r] = program(net, r)
        except BaseException as e:  # noqa: BLE001
            err.append(e)

    th = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise err[0]
    return out


def sim_reduce(sends, op, root):
    P = len(sends)

    def prog(net, me):
        recv = sends[me].copy()  # arraycopy(sendbuf -> recvbuf)
        mst_reduce(net, me, recv, op, root, 0, P - 1)
        return recv

    return run_ranks(P, prog)[root]


def sim_allreduce(sends, op):
    res = sim_reduce(sends, op, 0)
    return [res.copy() for _ in sends]  # MST_Broadcast moves rank 0's bits unchanged


def sim_ft(sends, op, root_of):
    """FT_Reduce at `root`, or FT_Allreduce (every rank is a root): isend to the roots, fold in order."""
    P = len(sends)

    def prog(net, me):
        opx = TypedOp(op)
        opx.createInitialBuffer(sends[me])
        roots = root_of(me)
        for dst in range(P):
            if dst != me and (dst in roots if roots is not None else True):
                net.send(sends[me], me, dst, 2)
        recv = np.zeros_like(sends[me])
        if roots is None or me in roots:
            for i in range(P):
                if i == me:
                    continue
                net.recv(recv, i, me, 2)
                opx.perform(recv)
        opx.getResultant(recv)
        return recv

    return run_ranks(P, prog)


def sim_scan(sends, op):
    P = len(sends)

    def prog(net, me):
        opx = TypedOp(op)
        opx.createInitialBuffer(sends[me])
        for i in range(P - 1, me, -1):
            net.send(sends[me], me, i, 3)
        recv = np.zeros_like(sends[me])
        for i in range(me):
            net.recv(recv, i, me, 3)
            opx.perform(recv)
        opx.getResultant(recv)
        return recv

    return run_ranks(P, prog)


def _inputs(P, n, dt, op, seed):
    rng = np.random.default_rng(seed)
    xs = []
    for r in range(P):
        x = rng.uniform(-1, 1, n).astype(dt)
        if op == O.PROD:
            x = (np.sign(x) * (0.5 + np.abs(x))).astype(dt)
        x[r % n] = np.nan if op in (O.MAX, O.MIN) and r % 3 == 0 else x[r % n]
        x[(r + 5) % n] = dt(-0.0) if r % 2 else dt(0.0)
        xs.append(x)
    return xs


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    u = np.uint32 if a.dtype == np.float32 else np.uint64
    return np.array_equal(a.view(u), b.view(u))


CASES = [(op, t) for op in (O.SUM, O.PROD, O.MAX, O.MIN) for t in (O.FLOAT, O.DOUBLE)]


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("op,type_", CASES)
def test_message_passing_restatement_matches_oracle(P, op, type_):
    dt = np.float32 if type_ == O.FLOAT else np.float64
    n = 257
    sends = _inputs(P, n, dt, op, 1000 * P + op)
    for root in range(P):
        exp = O.reduce(sends, n, type_, op, root)[root]
        assert _same(sim_reduce(sends, op, root), exp), ("reduce", root)
        exp = O.reduce(sends, n, type_, op, root, flags=O.FLAG_OLD)[root]
        assert _same(sim_ft(sends, op, lambda me, root=root: [root])[root], exp), ("ft_reduce", root)
    for got, exp in zip(sim_allreduce(sends, op), O.allreduce(sends, n, type_, op)):
        assert _same(got, exp), "allreduce"
    for got, exp in zip(sim_ft(sends, op, lambda me: None), O.allreduce(sends, n, type_, op, flags=O.FLAG_OLD)):
        assert _same(got, exp), "ft_allreduce"
    for got, exp in zip(sim_scan(sends, op), O.scan(sends, n, type_, op)):
        assert _same(got, exp), "scan"


class NoopOp(TypedOp):
    """Bor*/Bxor* declare perform(Object, Object, int), which does not override Op.perform(Object,
    int, int) (src/mpi/BorInt.java:50): the base class's empty methods run instead."""

    def createInitialBuffer(self, buf):
        pass

    def perform(self, buf):
        pass

    def getResultant(self, buf):
        pass


def combine_int(op, x, acc):
    if op == O.BAND:
        return x & acc
    return combine(op, x, acc)


class IntOp(TypedOp):
    def perform(self, buf):
        self.arr = combine_int(self.op, buf, self.arr)


def sim_bkt_reduce_scatter(sends, recvcounts, op, faithful_noop=False):
    """BKT_Reduce_scatter (src/mpi/PureIntracomm.java:2377-2439) as written: every round isends the
    same block `prev` of buf, irecvs block `me` from `next` into a zero temporary, and the typed op
    combines the WHOLE temporary into arr (then copies arr over buf)."""
    P = len(sends)
    count = sum(recvcounts)
    bufs = [s.copy() for s in sends]

    def prog(net, me):
        prev, nxt = (me - 1) % P, (me + 1) % P
        isend_off = sum(recvcounts[:prev])
        irecv_off = sum(recvcounts[:me])
        buf = bufs[me]
        opx = NoopOp(op) if faithful_noop else IntOp(op)
        opx.createInitialBuffer(buf)
        tmp = np.zeros(count, dtype=buf.dtype)
        for _ in range(P - 1):
            net.send(buf[isend_off:isend_off + recvcounts[prev]], me, prev, 4)
            blk = tmp[irecv_off:irecv_off + recvcounts[me]]
            net.recv(blk, nxt, me, 4)
            opx.perform(tmp)
            opx.getResultant(buf)
        return buf[irecv_off:irecv_off + recvcounts[me]].copy()

    return run_ranks(P, prog), bufs


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("op,type_", [(O.SUM, O.DOUBLE), (O.SUM, O.INT), (O.PROD, O.FLOAT), (O.MAX, O.DOUBLE),
                                      (O.MIN, O.FLOAT), (O.BAND, O.INT), (O.BOR, O.INT), (O.BXOR, O.INT)])
def test_bkt_reduce_scatter_defect_as_message_pattern(P, op, type_):
    """The oracle's FAITHFUL Reduce_scatter (SURVEY A9, and A3 for BOR/BXOR) equals the BKT ring run as
    messages: results and the overwritten send buffers, ragged recvcounts."""
    rng = np.random.default_rng(77 * P + op)
    dt = O.NP_DTYPE[type_]
    rc = [3 + (r * 5) % 7 for r in range(P)]
    n = sum(rc)
    if type_ in (O.FLOAT, O.DOUBLE):
        sends = [rng.uniform(-2, 2, n).astype(dt) for _ in range(P)]
    else:
        sends = [rng.integers(-1000, 1000, n).astype(dt) for _ in range(P)]
    got, bufs = sim_bkt_reduce_scatter(sends, rc, op, faithful_noop=op in (O.BOR, O.BXOR))
    exp, exp_bufs = O.reduce_scatter([s.copy() for s in sends], rc, type_, op, flags=O.FLAG_FAITHFUL)
    for r in range(P):
        assert np.array_equal(np.asarray(got[r]).view(np.uint8), np.asarray(exp[r]).view(np.uint8)), ("recv", r)
        assert np.array_equal(bufs[r].view(np.uint8), np.asarray(exp_bufs[r]).view(np.uint8)), ("sendbuf", r)
