"""CPU, multi-process (gloo, world sizes 2, 3 and 5): the N>1 plan of libmpjx, carried out with real
message passing.

libmpjx replaces the reference's tree/ring message patterns (src/mpi/PureIntracomm.java) by
  exchange #1 (block j of every rank -> rank j) -> per-block combine in the reference's ORDER ->
  exchange #2 (all-gather, result scatter or gather-to-root).
These tests run that plan across processes with gloo point-to-point, doing each rank's block
combine with the oracle's own collective on the P received slices, and check the reassembled
result against the oracle's whole-vector reference algorithm: the claim that slicing commutes with
the MST / FT / Scan orders, for the exact block partition the engine uses (256-B aligned even
split; ragged recvcounts for Reduce_scatter).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from util import make_input, same_bits


def even_blocks(n, P, esz):
    """Same partition as Blocks::even in csrc/mpjx_collectives.hip."""
    a = 256 // esz
    per = -(-n // P)
    per = -(-per // a) * a
    off = [min(n, j * per) for j in range(P)]
    ln = [min(n, off[j] + per) - off[j] for j in range(P)]
    return off, ln


def mst_subtree(P, root, r):
    """Same walk as mst_subtree in csrc/mpjx_collectives.hip: the interval whose MST partial rank r's
    recvbuf holds after MST_Reduce (PureIntracomm.java:1943-1992)."""
    lo, hi, rt = 0, P - 1, root
    while r != rt:
        mid = (lo + hi) // 2
        srce = hi if rt <= mid else lo
        if r <= mid:
            rt, hi = (rt if rt <= mid else srce), mid
        else:
            rt, lo = (rt if rt > mid else srce), mid + 1
    return lo, hi


def test_mst_subtree_intervals():
    """Every rank's interval contains it, the root's is everything, and the intervals nest (a tree)."""
    for P in range(1, 14):
        for root in range(P):
            iv = [mst_subtree(P, root, r) for r in range(P)]
            assert iv[root] == (0, P - 1)
            for r, (a, b) in enumerate(iv):
                assert a <= r <= b
                for (c, d) in iv:
                    assert b < c or d < a or (a <= c and d <= b) or (c <= a and b <= d)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def exchange(sends, recvs):
    """Grouped point-to-point: sends/recvs are lists of (peer, numpy array) (like Transport::exchange)."""
    import torch

    reqs = []
    bufs = []
    for peer, arr in recvs:
        t = torch.empty(arr.nbytes, dtype=torch.uint8)
        bufs.append((t, arr))
        reqs.append(dist.irecv(t, src=peer))
    for peer, arr in sends:
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy()), dst=peer))
    for r in reqs:
        r.wait()
    for t, arr in bufs:
        arr.view(np.uint8)[:] = t.numpy()


def _worker(rank, P, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        q.put((rank, _plans(rank, P)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, e))
    finally:
        dist.destroy_process_group()


def _plans(me, P):
    errors = []
    cases = [(O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.PROD, O.FLOAT), (O.BXOR, O.INT), (O.SUM, O.CHAR)]
    for op, t in cases:
        esz = np.dtype(O.NP_DTYPE[t]).itemsize
        n = 3001
        xs = [make_input(t, n, 11 * (r + 1), op=op) for r in range(P)]  # every rank knows all inputs
        off, ln = even_blocks(n, P, esz)
        blk = lambda r, j: xs[r][off[j]:off[j] + ln[j]]  # noqa: E731
        # exchange #1
        recv = {j: np.empty(ln[me], xs[0].dtype) for j in range(P) if j != me}
        exchange([(j, blk(me, j)) for j in range(P) if j != me and ln[j]],
                 [(j, recv[j]) for j in range(P) if j != me and ln[me]])
        slices = [blk(me, me) if j == me else recv[j] for j in range(P)]
        for flags in (0, O.FLAG_OLD):
            # Allreduce: my block in the reference order, then all-gather
            mine = O.allreduce(slices, ln[me], t, op, flags=flags)
            res = np.empty(n, xs[0].dtype)
            if flags & O.FLAG_OLD:  # FT: every rank's own order -> rank me computes all P results
                outs = mine
                res[off[me]:off[me] + ln[me]] = outs[me]
                exchange([(j, outs[j]) for j in range(P) if j != me and ln[me]],
                         [(j, res[off[j]:off[j] + ln[j]]) for j in range(P) if j != me and ln[j]])
            else:
                res[off[me]:off[me] + ln[me]] = mine[0]
                exchange([(j, mine[0]) for j in range(P) if j != me and ln[me]],
                         [(j, res[off[j]:off[j] + ln[j]]) for j in range(P) if j != me and ln[j]])
            exp = O.allreduce(xs, n, t, op, flags=flags)[me]
            if not same_bits(t, op, res, exp):
                errors.append(("allreduce", op, t, flags))
        # Scan: rank me computes block me of every rank's prefix and scatters them back
        outs = O.scan(slices, ln[me], t, op)
        res = np.empty(n, xs[0].dtype)
        res[off[me]:off[me] + ln[me]] = outs[me]
        exchange([(j, outs[j]) for j in range(P) if j != me and ln[me]],
                 [(j, res[off[j]:off[j] + ln[j]]) for j in range(P) if j != me and ln[j]])
        if not same_bits(t, op, res, O.scan(xs, n, t, op)[me]):
            errors.append(("scan", op, t))
        # Reduce at every root: gather-to-root of the rooted-tree blocks
        for root in range(P):
            part = O.reduce(slices, ln[me], t, op, root)[root]
            res = np.empty(n, xs[0].dtype)
            if me == root:
                res[off[me]:off[me] + ln[me]] = part
            exchange([(root, part)] if me != root and ln[me] else [],
                     [(j, res[off[j]:off[j] + ln[j]]) for j in range(P) if me == root and j != root and ln[j]])
            if me == root and not same_bits(t, op, res, O.reduce(xs, n, t, op, root)[root]):
                errors.append(("reduce", op, t, root))
        # Faithful Reduce (MPJX_FLAG_FAITHFUL): block me of EVERY rank's recvbuf — rank r's MST sub-tree
        # partial (mst_subtree, as csrc/mpjx_collectives.hip) — then each block to its rank
        for root in range(P):
            parts = {}
            for r in range(P):
                a, b = mst_subtree(P, root, r)
                parts[r] = O.reduce(slices[a:b + 1], ln[me], t, op, r - a, flags=O.FLAG_FAITHFUL)[r - a][:ln[me]]
            res = np.empty(n, xs[0].dtype)
            res[off[me]:off[me] + ln[me]] = parts[me]
            exchange([(j, parts[j]) for j in range(P) if j != me and ln[me]],
                     [(j, res[off[j]:off[j] + ln[j]]) for j in range(P) if j != me and ln[j]])
            if not same_bits(t, op, res, O.reduce(xs, n, t, op, root, flags=O.FLAG_FAITHFUL)[me]):
                errors.append(("faithful_reduce_partials", op, t, root))
        # Reduce_scatter with ragged recvcounts
        rc = [5 + 37 * j for j in range(P)]
        tot = sum(rc)
        ys = [make_input(t, tot, 5 * (r + 3), op=op) for r in range(P)]
        roff = np.cumsum([0] + rc[:-1]).tolist()
        got = {j: np.empty(rc[me], ys[0].dtype) for j in range(P) if j != me}
        exchange([(j, ys[me][roff[j]:roff[j] + rc[j]]) for j in range(P) if j != me],
                 [(j, got[j]) for j in range(P) if j != me])
        sl = [ys[me][roff[me]:roff[me] + rc[me]] if j == me else got[j] for j in range(P)]
        exp, _ = O.reduce_scatter(ys, rc, t, op)
        if P <= 2:
            mine = O.apply(op, t, sl[me].copy(), sl[(me + 1) % P])  # BKT order: acc = own block
        else:
            mine = O.reduce(sl, rc[me], t, op, 0)[0]               # MST root-0 block
        if not same_bits(t, op, mine, exp[me]):
            errors.append(("reduce_scatter", op, t))
    return errors


@pytest.mark.parametrize("P", [2, 3, 5, 8])
def test_exchange_plan_matches_reference_algorithms(P):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, P, port, q)) for r in range(P)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(P))
    for p in procs:
        p.join(timeout=60)
    for r in range(P):
        assert not isinstance(res[r], Exception), res[r]
        assert res[r] == [], f"rank {r}: {res[r]}"


def test_even_blocks_partition():
    for n in (0, 1, 31, 32, 33, 1000, 33554432):
        for P in (1, 2, 3, 7, 8):
            for esz in (1, 2, 4, 8):
                off, ln = even_blocks(n, P, esz)
                assert sum(ln) == n
                assert all(o * esz % 256 == 0 or lnj == 0 for o, lnj in zip(off, ln))
                assert all(off[j] + ln[j] <= n for j in range(P))
