"""Time the P-way combine kernels (mpjx_combine_multi) on one GPU: HBM GB/s per order and P.

  python tools/bench_pway.py [--mib-per-slice 32] [--iters 20] [--cases MST:8,SCAN:2,FOLD:2]
                             [--big-endian] [--copies] [--combine] [--rotate R]
Slices are separate 256-B aligned device buffers of random doubles (as after exchange #1).
Algorithmic bytes: MST/FOLD (P + 1) * slice, SCAN 2P * slice. --big-endian passes
MPJX_FLAG_SEND_BIG_ENDIAN | MPJX_FLAG_RECV_BIG_ENDIAN (operands and results byte-swapped inside the
kernel; same algorithmic bytes). --copies also times k_copies (the copy kernel behind the IPC push
and Reduce's arraycopy at P = 1): mpjx_combine_multi FOLD with P = 1 is one copy, 2 * slice bytes.
--combine also times the headline in-place mpjx_combine (inout = in + inout, 3 * slice bytes).
--rotate R cycles every case over R independent buffer sets, so no launch finds its operands in the
256 MiB Infinity Cache from the previous launch (R sets of >= 512 MiB leave nothing to reuse).
Each case is timed with HIP events on the stream it is launched on; run
the same command under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE for the counter traffic.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mpjexpress_amd import _lib  # noqa: E402

ORDERS = {"FOLD": 0, "MST": 1, "SCAN": 2}
DEFAULT = "MST:3,MST:4,MST:8,FOLD:2,FOLD:3,FOLD:4,FOLD:8,SCAN:2,SCAN:3,SCAN:4,SCAN:8"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib-per-slice", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cases", default=DEFAULT)
    ap.add_argument("--big-endian", action="store_true")
    ap.add_argument("--copies", action="store_true")
    ap.add_argument("--combine", action="store_true")
    ap.add_argument("--rotate", type=int, default=1, help="independent buffer sets cycled per launch")
    ap.add_argument("--op", type=int, default=3, help="op code (SUM = 3)")
    ap.add_argument("--type", type=lambda v: int(v, 0), default=8, help="type code (DOUBLE = 8; pairs 0x103..0x108)")
    ap.add_argument("--mpjbuf", action="store_true",
                    help="also time mpjx_mpjbuf_combine: acc (slice) = payload of a one-section mpjbuf image (op) acc")
    a = ap.parse_args()
    L = _lib.lib()
    esz = {1: 1, 2: 2, 3: 2, 4: 1, 5: 4, 6: 8, 7: 4, 8: 8, 0x103: 4, 0x105: 8, 0x106: 16, 0x107: 8, 0x108: 16}[a.type]
    nbytes = a.mib_per_slice * (1 << 20)
    n = nbytes // esz  # elements of the chosen type per slice (random bits: a timing run)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    flags = 0xC if a.big_endian else 0
    cases = [(c.split(":")[0], int(c.split(":")[1])) for c in a.cases.split(",") if c]
    if a.copies:
        cases.append(("COPY", 1))
    if a.mpjbuf:
        cases.append(("MPJBUF", 2))
    if a.combine:
        cases.append(("COMBINE", 2))
    R = max(1, a.rotate)
    for oname, P in cases:
        if oname == "MPJBUF":
            print(json.dumps(mpjbuf_case(L, n, dev, st, sp, a.iters, a.mib_per_slice, R)), flush=True)
            continue
        order = ORDERS.get(oname, 0)
        Q = P if oname == "SCAN" else 1
        if oname == "COMBINE":
            Q = 0
        def buf():
            return torch.randint(0, 2 if a.type == 4 else 256, (nbytes,), dtype=torch.uint8, device=dev)

        if (a.op, a.type) == (3, 8):
            buf = lambda: torch.rand(n, dtype=torch.float64, device=dev)  # noqa: E731
        ins = [[buf() for _ in range(P)] for _ in range(R)]
        outs = [[torch.empty_like(ins[0][0]) for _ in range(Q)] for _ in range(R)]
        pin = [(ctypes.c_void_p * P)(*[t.data_ptr() for t in s]) for s in ins]
        pout = [(ctypes.c_void_p * max(Q, 1))(*[t.data_ptr() for t in s]) for s in outs]
        torch.cuda.synchronize()

        def go(k):
            k %= R
            if oname == "COMBINE":
                _lib.check(L.mpjx_combine(a.op, a.type, ins[k][0].data_ptr(), ins[k][1].data_ptr(), n, sp), "combine")
                return
            _lib.check(L.mpjx_combine_multi(a.op, a.type, order, P, pin[k], pout[k], n, 0, flags if oname != "COPY" else 0,
                                            sp), "combine_multi")

        for k in range(max(3, R)):
            go(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(a.iters):
            go(k)
        e1.record(st)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / a.iters / 1e3
        byts = (P + max(Q, 1)) * nbytes
        r = {"order": oname, "P": P, "slice_MiB": a.mib_per_slice, "rotate": R, "op": a.op, "type": a.type,
             "big_endian": bool(flags) and oname not in ("COPY", "COMBINE"),
             "us": round(t * 1e6, 1), "algorithmic_bytes": byts, "GBps": round(byts / t / 1e9, 1),
             "frac_8TBps": round(byts / t / 8e12, 3)}
        print(json.dumps(r), flush=True)
        del ins, outs


def mpjbuf_case(L, n, dev, st, sp, iters, mib, R=1):
    """acc = payload (op SUM) acc, the payload a one-section big-endian mpjbuf image of n doubles
    (8-byte header, elements from byte 8), the section walked by the kernel; R (acc, image) sets cycled."""
    sets = []
    for _ in range(R):
        acc = torch.rand(n, dtype=torch.float64, device=dev)
        img = torch.zeros(8 + n * 8 + 8, dtype=torch.uint8, device=dev)
        hdr = torch.tensor([7, 0, 0, 0] + list(int(n).to_bytes(4, "big")), dtype=torch.uint8)
        img[:8] = hdr.to(dev)
        img[8:8 + n * 8] = torch.rand(n, dtype=torch.float64, device=dev).view(torch.uint8)
        sets.append((acc, img))
    st_dev = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def go(k):
        acc, img = sets[k % R]
        _lib.check(L.mpjx_mpjbuf_combine(3, 8, acc.data_ptr(), img.data_ptr(), img.numel(), n, st_dev.data_ptr(), 0, sp),
                   "mpjx_mpjbuf_combine")

    for k in range(max(3, R)):
        go(k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for k in range(iters):
        go(k)
    e1.record(st)
    torch.cuda.synchronize()
    assert int(st_dev.item()) == 0
    t = e0.elapsed_time(e1) / iters / 1e3
    byts = 3 * n * 8
    return {"order": "MPJBUF", "P": 2, "slice_MiB": mib, "rotate": R, "big_endian": True, "us": round(t * 1e6, 1),
            "algorithmic_bytes": byts, "GBps": round(byts / t / 1e9, 1), "frac_8TBps": round(byts / t / 8e12, 3)}


if __name__ == "__main__":
    main()
