"""Time the P-way combine kernels (mpjx_combine_multi) on one GPU: HBM GB/s per order and P.

  python tools/bench_pway.py [--mib-per-slice 32] [--iters 20]
Slices are separate 256-B aligned device buffers of random doubles (as after exchange #1).
Algorithmic bytes: MST/FOLD (P + 1) * slice, SCAN 2P * slice.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib-per-slice", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    L = _lib.lib()
    n = a.mib_per_slice * (1 << 20) // 8
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    res = []
    for order, oname in ((1, "MST"), (0, "FOLD"), (2, "SCAN")):
        for P in (2, 3, 4, 8):
            if order == 1 and P == 2:
                continue
            ins = [torch.rand(n, dtype=torch.float64, device=dev) for _ in range(P)]
            Q = P if order == 2 else 1
            outs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(Q)]
            pin = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
            pout = (ctypes.c_void_p * Q)(*[t.data_ptr() for t in outs])
            torch.cuda.synchronize()

            def go():
                _lib.check(L.mpjx_combine_multi(3, 8, order, P, pin, pout, n, 0, 0, sp), "combine_multi")

            for _ in range(3):
                go()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
            for e0, e1 in ev:
                e0.record(st)
                go()
                e1.record(st)
            torch.cuda.synchronize()
            t = sum(e0.elapsed_time(e1) for e0, e1 in ev) / a.iters / 1e3
            byts = (P + Q) * n * 8
            r = {"order": oname, "P": P, "slice_MiB": a.mib_per_slice, "us": round(t * 1e6, 1),
                 "GBps": round(byts / t / 1e9, 1), "frac_8TBps": round(byts / t / 8e12, 3)}
            res.append(r)
            print(json.dumps(r), flush=True)
            del ins, outs


if __name__ == "__main__":
    main()
