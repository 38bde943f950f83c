"""Where should the P-way kernel's operands live? (follow-up of tools/slot_skew.py)

For each shape, time the kernel (cold: R independent sets cycled, >= 1 GiB between two uses of a
set; HIP events on the launch stream) under several layouts of the P inputs and Q outputs of a set:
  contig_sepout   inputs: one allocation, stride = slice (the RCCL engine's exchange slots);
                  outputs: their own allocation(s)
  skew_sepout     inputs: one allocation, stride = slice + 4 KiB (IPC push slots); outputs separate
  skew_inout      inputs and outputs: one allocation, stride = slice + 4 KiB (tools/slot_skew.py)
  separate        every slice its own torch allocation (tools/bench_pway.py, bench.py before round 3)
  contig_outskew  inputs contiguous; outputs: one allocation, stride slice + 4 KiB, placed after the inputs
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mpjexpress_amd import _lib  # noqa: E402

SHAPES = [("MST", 8, 32), ("SCAN", 8, 32), ("MST", 4, 64), ("SCAN", 4, 64), ("FOLD", 2, 128), ("MST", 8, 4)]
LAYOUTS = ["contig_sepout", "skew_sepout", "skew_inout", "separate", "contig_outskew"]
SK = 4096


def sets_for(layout, P, Q, slice_b, R, dev):
    """R sets of (list of P input addresses, list of Q output addresses, keep-alive tensors)."""
    out = []
    for _ in range(R):
        keep, ins, outs = [], [], []
        if layout == "separate":
            for _p in range(P):
                t = torch.empty(slice_b // 8, dtype=torch.float64, device=dev).uniform_(-1, 1)
                keep.append(t)
                ins.append(t.data_ptr())
            for _q in range(Q):
                t = torch.empty(slice_b // 8, dtype=torch.float64, device=dev)
                keep.append(t)
                outs.append(t.data_ptr())
        else:
            stride = slice_b + (SK if layout.startswith("skew") else 0)
            nslots = P + Q if layout == "skew_inout" else P
            b = torch.empty(nslots * stride // 8, dtype=torch.float64, device=dev).uniform_(-1, 1)
            keep.append(b)
            ins = [b.data_ptr() + p * stride for p in range(P)]
            if layout == "skew_inout":
                outs = [b.data_ptr() + (P + q) * stride for q in range(Q)]
            elif layout == "contig_outskew":
                o = torch.empty(Q * (slice_b + SK) // 8, dtype=torch.float64, device=dev)
                keep.append(o)
                outs = [o.data_ptr() + q * (slice_b + SK) for q in range(Q)]
            else:
                for _q in range(Q):
                    t = torch.empty(slice_b // 8, dtype=torch.float64, device=dev)
                    keep.append(t)
                    outs.append(t.data_ptr())
        out.append(((ctypes.c_void_p * P)(*ins), (ctypes.c_void_p * Q)(*outs), keep))
    return out


def main():
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    code = {"FOLD": 0, "MST": 1, "SCAN": 2}
    iters = int(os.environ.get("ITERS", "30"))
    for trial in range(2):
        for kind, P, mib in SHAPES:
            slice_b = mib << 20
            Q = P if kind == "SCAN" else 1
            R = max(2, -(-(1 << 30) // ((P + Q) * slice_b)) + 1)
            for layout in LAYOUTS:
                sets = sets_for(layout, P, Q, slice_b, R, dev)
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
                print(json.dumps({"trial": trial, "kind": kind, "P": P, "slice_MiB": mib, "layout": layout, "sets": R,
                                  "us": round(t * 1e6, 2), "frac": round((P + Q) * slice_b / t / 8e12, 4)}), flush=True)
                del sets
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
