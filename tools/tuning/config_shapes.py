"""The library's P-way combine at the shapes BASELINE configs[3] (Reduce_scatter BAND / Scan BXOR,
int32, 64 MiB per rank) and configs[4] (Allreduce MAX float, 1 GiB per rank) run at N = 2, 4, 8, in the
RCCL exchange engine's layout: input slots contiguous in one allocation (one ncclAllToAll), output slots
4 KiB apart (mpjx_collectives.hip make_slots). Cold: R sets cycled so >= 1 GiB streams between two uses
of a set. One JSON line per shape; MPJX_NT_MIN_MIB etc. apply as in the library.
MODE=after_write: the same sets, but before every combine a device copy rewrites the input slots (the
exchange #1 that lands them in the engine), and only the combine is timed — what the combine sees when
its operands were written a moment ago (the Infinity Cache may still hold them), beside the cold figure.
MODE=sizes: RS BAND int32 K_MST P=8, cold, slices 4 KiB .. 64 MiB: the launch's fixed cost (intercept of
time over bytes) and its streaming rate (slope), which bound the fraction a launch of a given size reaches.
Usage: [MODE=cold|after_write|sizes] python tools/tuning/config_shapes.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mpjexpress_amd import _lib  # noqa: E402

MAX, BAND, BXOR = 1, 6, 10
INT, FLOAT = 5, 7
FOLD, MST, SCAN = 0, 1, 2
# (label, op, type, kind, P, slice bytes): Reduce_scatter at P >= 3 is the MST(0) block, at P = 2 the
# bucket fold; Scan is K_SCAN; Allreduce MST (P >= 3) or the 2-operand fold
SHAPES = [("configs[3] RS BAND int32 N=8", BAND, INT, MST, 8, 8 << 20),
          ("configs[3] Scan BXOR int32 N=8", BXOR, INT, SCAN, 8, 8 << 20),
          ("configs[4] MAX float N=8", MAX, FLOAT, MST, 8, 128 << 20),
          ("configs[3] RS BAND int32 N=4", BAND, INT, MST, 4, 16 << 20),
          ("configs[3] Scan BXOR int32 N=4", BXOR, INT, SCAN, 4, 16 << 20),
          ("configs[4] MAX float N=4", MAX, FLOAT, MST, 4, 256 << 20),
          ("configs[3] RS BAND int32 N=2", BAND, INT, FOLD, 2, 32 << 20),
          ("configs[3] Scan BXOR int32 N=2", BXOR, INT, SCAN, 2, 32 << 20),
          ("configs[4] MAX float N=2", MAX, FLOAT, FOLD, 2, 512 << 20)]
OSK = 4096


SIZES = [("RS BAND int32 K_MST P=8, %s slices" % (("%d KiB" % (sb >> 10)) if sb < (1 << 20) else ("%d MiB" % (sb >> 20))),
          BAND, INT, MST, 8, sb) for sb in (4 << 10, 64 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20,
                                             32 << 20, 64 << 20)]


def main():
    mode = os.environ.get("MODE", "cold")
    shapes = SIZES if mode == "sizes" else SHAPES
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    iters = int(os.environ.get("ITERS", "20"))
    for trial in range(2):
        for label, op, typ, kind, P, sb in shapes:
            Q = P if kind == SCAN else 1
            R = max(2, -(-(1 << 30) // ((P + Q) * sb)) + 1)
            sets = []
            for _ in range(R):
                b = torch.randint(-2**31, 2**31 - 1, (P * sb // 4,), dtype=torch.int32, device=dev)
                o = torch.empty(Q * (sb + OSK) // 4, dtype=torch.int32, device=dev)
                ins = [b.data_ptr() + p * sb for p in range(P)]
                outs = [o.data_ptr() + q * (sb + OSK) for q in range(Q)]
                sets.append(((ctypes.c_void_p * P)(*ins), (ctypes.c_void_p * Q)(*outs), b, o))
            src = sets[-1][2].clone() if mode == "after_write" else None
            n = sb // 4
            torch.cuda.synchronize()

            def go(i):
                ins, outs, _, _ = sets[i % R]
                _lib.check(L.mpjx_combine_multi(op, typ, kind, P, ins, outs, n, 0, 0, sp), label)

            for i in range(R):
                go(i)
            torch.cuda.synchronize()
            if mode == "after_write":
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
                with torch.cuda.stream(st):
                    for i in range(iters):
                        sets[i % R][2].copy_(src)  # exchange #1 lands the slots
                        ev[i][0].record(st)
                        go(i)
                        ev[i][1].record(st)
                torch.cuda.synchronize()
                t = sum(a.elapsed_time(b) for a, b in ev) / iters / 1e3
            else:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for i in range(iters):
                    go(i)
                e1.record(st)
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / iters / 1e3
            print(json.dumps({"trial": trial, "mode": mode, "shape": label, "P": P, "slice_KiB": sb >> 10,
                              "sets": R, "bytes": (P + Q) * sb, "us": round(t * 1e6, 2),
                              "frac": round((P + Q) * sb / t / 8e12, 4)}), flush=True)
            del sets
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
