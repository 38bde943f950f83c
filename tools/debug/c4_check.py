"""Debug: why does bench.py's configs[3] Reduce_scatter check report a mismatch at world size 1?"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import torch  # noqa: E402

import bench  # noqa: E402
from mpjexpress_amd import _lib  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda", 0)
n4 = (64 << 20) // 4
band, bxor = bench.c4_inputs(n4, 0, dev)
band2, bxor2 = bench.c4_inputs(n4, 0, dev)
torch.cuda.synchronize()
print("inputs deterministic:", torch.equal(band, band2), torch.equal(bxor, bxor2), flush=True)
arr = (ctypes.c_void_p * 1)()
devs = (ctypes.c_int * 1)(0)
_lib.check(L.mpjx_comm_init_smp(arr, 1, devs), "init")
c = ctypes.c_void_p(arr[0])
cs = ctypes.c_void_p()
_lib.check(L.mpjx_comm_stream(c, ctypes.byref(cs)), "stream")
for trial, sp in (("comm stream", cs), ("NULL", None)):
    y = torch.empty(n4, dtype=torch.int32, device=dev)
    rc = (ctypes.c_int64 * 1)(n4)
    torch.cuda.synchronize()
    for _ in range(3):
        _lib.check(L.mpjx_reduce_scatter(c, band.data_ptr(), y.data_ptr(), rc, 5, 6, 0, sp), "rs")
    _lib.check(L.mpjx_comm_synchronize(c), "sync")
    torch.cuda.synchronize()
    bad = (y != band).nonzero().flatten()
    print(trial, "mismatches", bad.numel(), "first", bad[:8].tolist(),
          [(int(y[i]), int(band[i])) for i in bad[:4].tolist()], flush=True)
    z = torch.empty(n4, dtype=torch.int32, device=dev)
    for _ in range(3):
        _lib.check(L.mpjx_scan(c, bxor.data_ptr(), z.data_ptr(), n4, 5, 10, 0, sp), "scan")
    _lib.check(L.mpjx_comm_synchronize(c), "sync")
    torch.cuda.synchronize()
    print(trial, "scan mismatches", int((z != bxor).sum()), flush=True)
    for n in (n4 - 4, n4 // 2, 1 << 20):
        y2 = torch.empty(n, dtype=torch.int32, device=dev)
        rc2 = (ctypes.c_int64 * 1)(n)
        _lib.check(L.mpjx_reduce_scatter(c, band.data_ptr(), y2.data_ptr(), rc2, 5, 6, 0, sp), "rs")
        _lib.check(L.mpjx_comm_synchronize(c), "sync")
        torch.cuda.synchronize()
        print(trial, n, "rs mismatches", int((y2 != band[:n]).sum()), flush=True)
L.mpjx_comm_destroy(c)
