"""Worker for test_gpu_combine.py::test_streaming_form_every_instantiation, run as a child process with
MPJX_NT_MIN_MIB=0 (read once per process by libmpjx), so that every vector launch takes a streaming
form — with MPJX_SHORT_MAX_MIB=0 the 1024/512-lane non-temporal tiles that otherwise run only for
launches streaming >= 256 MiB, without it the short-launch forms of 64-256 MiB launches (deep K_SCAN
tiles, persistent grids) (mpjx_kernels.hpp launch_pw) — at sizes the oracle checks in seconds. Covers every (op, type) pair's
2-operand fold, FOLD/MST/SCAN at P = 2..8 for one pair per element width (the narrow types at large P
take the 512-lane instantiation), MAXLOC/MINLOC at P = 8, and big-endian operands and results.
Prints one line per failure and exits nonzero if there was any."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), HERE]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402  (the checker)
from util import flat, make_input, same_bits  # noqa: E402

from mpjexpress_amd import _lib, mpi  # noqa: E402

BE = 0xC  # MPJX_FLAG_SEND_BIG_ENDIAN | MPJX_FLAG_RECV_BIG_ENDIAN


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def bswap(a, type_):
    return flat(a, type_).byteswap().view(a.dtype)


def main():
    assert os.environ.get("MPJX_NT_MIN_MIB") == "0", "run with MPJX_NT_MIN_MIB=0"
    L = _lib.lib()
    bad = []
    # every pair's in-place fold (mpjx_combine), sizes around the 1024-lane tile and its tail
    for op, t in O.valid_pairs():
        for n in (1, 1000, 16384 + 3, 70001):
            acc, inp = make_input(t, n, 11 + n, op=op), make_input(t, n, 23 + n, op=op)
            exp = O.apply(op, t, acc.copy(), inp)
            ta, tb = dev(acc), dev(inp)
            mpi.combine(mpi.OPS[op - 1], mpi.DATATYPES[t - 1], ta, tb)
            torch.cuda.synchronize()
            if not same_bits(t, op, ta.cpu().numpy(), exp):
                bad.append(f"combine {O.OP_NAMES[op]} {O.TYPE_NAMES[t]} n={n}")
    # FOLD / MST (root 0 and the last; every root for the pair types) / SCAN at P = 2..8, one pair per
    # element width plus the MAXLOC/MINLOC pairs
    n = 40003
    cases = [(O.SUM, O.BYTE), (O.MAX, O.SHORT), (O.PROD, O.CHAR), (O.BXOR, O.INT), (O.MIN, O.FLOAT),
             (O.SUM, O.DOUBLE), (O.BAND, O.LONG), (O.LOR, O.BOOLEAN)] + list(O.loc_pairs())
    for op, t in cases:
        for P in range(2, 9):
            xs = [make_input(t, n, 131 * p + P, op=op) for p in range(P)]
            for swap in (0, BE):
                if swap and t == O.BOOLEAN:
                    continue
                src = [bswap(x, t) if swap else x for x in xs]
                ds = [dev(flat(x, t)) for x in src]
                pin = (ctypes.c_void_p * P)(*[d.data_ptr() for d in ds])
                tag = f"{O.OP_NAMES[op]} {O.TYPE_NAMES[t]} P={P} be={bool(swap)}"
                roots = range(P) if t in O.PAIR_BASE else sorted({0, P - 1})  # pairs: per-root bodies
                kinds = [(1, r) for r in roots] if P >= 3 else []
                kinds += [(0, 0), (2, 0)]
                for kind, root in kinds:
                    Q = P if kind == 2 else 1
                    outs = [torch.empty_like(ds[0]) for _ in range(Q)]
                    pout = (ctypes.c_void_p * Q)(*[o.data_ptr() for o in outs])
                    _lib.check(L.mpjx_combine_multi(op, t, kind, P, pin, pout, n, root, swap, None), tag)
                    torch.cuda.synchronize()
                    if kind == 1:
                        exp = [O.reduce(xs, n, t, op, root)[root]]
                    elif kind == 0:
                        exp = [O.reduce(xs, n, t, op, 0, flags=O.FLAG_OLD)[0]]
                    else:
                        exp = O.scan(xs, n, t, op)
                    for q in range(Q):
                        got = outs[q].cpu().numpy().view(xs[0].dtype)
                        if swap:
                            got = bswap(got, t)
                        ok = (np.array_equal(got.view(np.uint8), exp[q].view(np.uint8)) if t in O.PAIR_BASE
                              else same_bits(t, op, got, exp[q]))
                        if not ok:
                            bad.append(f"multi kind={kind} root={root} q={q} {tag}")
    # the persistent grid of the short-launch form (one block per CU, grid-strided): enough tiles that
    # every block loops several times (and a ragged last tile), FOLD P=2 and MST P=4/8
    for op, t in [(O.BAND, O.INT), (O.SUM, O.DOUBLE), (O.MAX, O.FLOAT), (O.MAXLOC, O.DOUBLE2)]:
        esz = 16 if t in O.PAIR_BASE else np.dtype(O.NP_DTYPE[t]).itemsize
        big = 3 * 256 * 1024 * (16 // esz) + 5
        for P, kind in ((2, 0), (4, 1), (8, 1)):
            xs = [make_input(t, big, 977 * p + P, op=op) for p in range(P)]
            ds = [dev(flat(x, t)) for x in xs]
            pin = (ctypes.c_void_p * P)(*[d.data_ptr() for d in ds])
            out = torch.empty_like(ds[0])
            pout = (ctypes.c_void_p * 1)(out.data_ptr())
            tag = f"persistent {O.OP_NAMES[op]} {O.TYPE_NAMES[t]} P={P} n={big}"
            _lib.check(L.mpjx_combine_multi(op, t, kind, P, pin, pout, big, 0, 0, None), tag)
            torch.cuda.synchronize()
            exp = (O.reduce(xs, big, t, op, 0)[0] if kind == 1
                   else O.reduce(xs, big, t, op, 0, flags=O.FLAG_OLD)[0])
            got = out.cpu().numpy().view(xs[0].dtype)
            ok = (np.array_equal(got.view(np.uint8), exp.view(np.uint8)) if t in O.PAIR_BASE
                  else same_bits(t, op, got, exp))
            if not ok:
                bad.append(tag)
    for b in bad:
        print("MISMATCH", b)
    print(f"streaming form: {len(bad)} mismatches")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
