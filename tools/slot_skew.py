"""Does the placement of the P operand slices in one allocation matter?

The exchange engine's P input slots are one scratch allocation with a stride of exactly the block
size (S/P, a power of two at the BASELINE shapes), so the P streams of a P-way kernel sit at the same
offset modulo 32/64/128 MiB. If HBM channel interleaving repeats at such strides the streams collide.
This times K_MST / K_FOLD / K_SCAN through mpjx_combine_multi with the slices of each set placed at
base + p * (slice + skew) in ONE buffer, for several skews, on cold operands (R sets cycled, >= 1 GiB
between two uses of a set), HIP events on the launch stream.

  python tools/slot_skew.py [--iters 30]
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

SHAPES = [("FOLD", 2, 128), ("MST", 4, 64), ("MST", 8, 32), ("SCAN", 8, 32)]
SKEWS = [0, 256, 4096, 65536, (2 << 20) + 4096, 3 << 20]
if os.environ.get("SKEW_SET") == "fine":
    SHAPES = [("MST", 8, 32), ("SCAN", 8, 32), ("MST", 4, 64), ("SCAN", 4, 64), ("MST", 8, 4), ("SCAN", 2, 128)]
    SKEWS = [0, 1024, 2048, 4096, 4096 + 256, 8192, 12288, 16384, 32768]
if os.environ.get("SKEW_SET") == "pol":  # the engines' 4 KiB skew, P = 3..4 streaming shapes (POL rule)
    SHAPES = [("MST", 4, 64), ("MST", 3, 64), ("MST", 4, 32), ("MST", 4, 16), ("FOLD", 4, 64), ("FOLD", 3, 64),
              ("SCAN", 4, 64), ("SCAN", 3, 64), ("MST", 8, 32), ("FOLD", 2, 128)]
    SKEWS = [4096]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    order_code = {"FOLD": 0, "MST": 1, "SCAN": 2}
    for kind, P, mib in SHAPES:
        slice_b = mib << 20
        n = slice_b // 8
        nout = P if kind == "SCAN" else 1
        for skew in SKEWS:
            stride = slice_b + skew
            set_b = (P + nout) * stride
            R = max(2, -(-(1 << 30) // set_b) + 1)
            bufs = [torch.empty((P + nout) * stride // 8, dtype=torch.float64, device=dev).uniform_(-1, 1)
                    for _ in range(R)]
            torch.cuda.synchronize()
            ins, outs = [], []
            for b in bufs:
                base = b.data_ptr()
                ins.append((ctypes.c_void_p * P)(*[base + p * stride for p in range(P)]))
                outs.append((ctypes.c_void_p * nout)(*[base + (P + q) * stride for q in range(nout)]))

            def go(i):
                k = i % R
                _lib.check(L.mpjx_combine_multi(3, 8, order_code[kind], P, ins[k], outs[k], n, 0, 0, sp), "multi")

            for i in range(R):
                go(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(a.iters):
                go(i)
            e1.record(st)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / a.iters / 1e3
            alg = (P + nout) * slice_b
            print(json.dumps({"kind": kind, "P": P, "slice_MiB": mib, "skew": skew, "sets": R,
                              "us": round(t * 1e6, 2), "frac": round(alg / t / 8e12, 4)}), flush=True)
            del bufs, ins, outs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
