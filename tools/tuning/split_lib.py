"""The library's P-way combine at the engines' combine shapes (round 3 also ran it with
MPJX_PWAY_SPLIT_KIB, a launch-splitting knob the library had for that experiment only; removed after
the null result, the variable is now ignored), cold (R sets cycled), operands in one allocation
per set at slice + 4 KiB (the engines' skewed layout). Run once per setting (the knob is read once per
process); one JSON line per shape. Usage: [SKEW=0] python tools/tuning/split_lib.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mpjexpress_amd import _lib  # noqa: E402

SHAPES = [("MST", 4, 64), ("SCAN", 8, 32), ("MST", 8, 32), ("FOLD", 2, 128), ("SCAN", 4, 64), ("FOLD", 2, 256)]
SK = int(os.environ.get("SKEW", "4096"))  # slot skew; 0 = contiguous slots (the RCCL engine's input layout)


def main():
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    code = {"FOLD": 0, "MST": 1, "SCAN": 2}
    iters = int(os.environ.get("ITERS", "30"))
    split = os.environ.get("MPJX_PWAY_SPLIT_KIB", "")
    for trial in range(3):
        for kind, P, mib in SHAPES:
            slice_b = mib << 20
            Q = P if kind == "SCAN" else 1
            stride = slice_b + SK
            R = max(3, -(-(3 << 29) // ((P + Q) * stride)) + 1)
            sets = []
            for _ in range(R):
                b = torch.empty((P * stride + Q * (slice_b + 4096)) // 8, dtype=torch.float64, device=dev).uniform_(-1, 1)
                ins = [b.data_ptr() + p * stride for p in range(P)]
                outs = [b.data_ptr() + P * stride + q * (slice_b + 4096) for q in range(Q)]  # output slots always skewed
                sets.append(((ctypes.c_void_p * P)(*ins), (ctypes.c_void_p * Q)(*outs), b))
            torch.cuda.synchronize()

            def go(i):
                ins, outs, _ = sets[i % R]
                _lib.check(L.mpjx_combine_multi(3, 8, code[kind], P, ins, outs, slice_b // 8, 0, 0, sp), "multi")

            for i in range(R):
                go(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(iters):
                go(i)
            e1.record(st)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / iters / 1e3
            print(json.dumps({"split_KiB": split or None, "skew": SK, "trial": trial, "kind": kind, "P": P, "slice_MiB": mib,
                              "sets": R, "us": round(t * 1e6, 2), "frac": round((P + Q) * slice_b / t / 8e12, 4)}),
                  flush=True)
            del sets
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
