"""End-to-end (host-resident) rate of the reduction path: host arrays in, host arrays out, through
mpjx_allreduce_host (what the JNI shim calls with pinned Java arrays), plus the raw PCIe and host
memcpy rates that bound it. World size 1 over RCCL (the one-GPU box).

  python tools/e2e_bench.py [--mib 256] [--iters 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpjexpress_amd import _lib, mpi  # noqa: E402


def timeit(f, iters):
    f()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", choices=["pageable", "pinned"], help="time just this e2e path (for traces)")
    a = ap.parse_args()
    S = a.mib << 20
    n = S // 8
    L = _lib.lib()
    out = {"bytes": S}
    src = np.random.default_rng(1).uniform(-1, 1, n)
    dst = np.empty_like(src)
    if a.only:
        c = mpi.Init(0, 1, 0, mpi.unique_id())
        if a.only == "pinned":
            s_, d_ = torch.from_numpy(src).pin_memory(), torch.zeros(n, dtype=torch.float64).pin_memory()
            sp, rp = s_.data_ptr(), d_.data_ptr()
        else:
            sp, rp = src.ctypes.data, dst.ctypes.data
        t = timeit(lambda: _lib.check(L.mpjx_allreduce_host(c.handle, sp, rp, n, 8, 3, 0), "allreduce_host"), a.iters)
        print(json.dumps({"only": a.only, "e2e_GBps": round(S / t / 1e9, 2), "ms": round(t * 1e3, 3)}))
        c.Free()
        return
    # raw rates
    dev = torch.empty(n, dtype=torch.float64, device="cuda")
    pin = torch.empty(n, dtype=torch.float64, pin_memory=True)
    pag = torch.from_numpy(src)
    out["h2d_pinned_GBps"] = S / timeit(lambda: (dev.copy_(pin, non_blocking=True), torch.cuda.synchronize()), a.iters) / 1e9
    out["d2h_pinned_GBps"] = S / timeit(lambda: (pin.copy_(dev, non_blocking=True), torch.cuda.synchronize()), a.iters) / 1e9
    out["h2d_pageable_GBps"] = S / timeit(lambda: (dev.copy_(pag), torch.cuda.synchronize()), a.iters) / 1e9
    dev2 = torch.empty_like(dev)
    pin2 = torch.empty_like(pin, pin_memory=True)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def bidir():
        with torch.cuda.stream(s1):
            dev.copy_(pin, non_blocking=True)
        with torch.cuda.stream(s2):
            pin2.copy_(dev2, non_blocking=True)
        torch.cuda.synchronize()

    out["bidir_pinned_each_GBps"] = S / timeit(bidir, a.iters) / 1e9
    pag_out = torch.from_numpy(dst)
    out["d2h_pageable_GBps"] = S / timeit(lambda: (pag_out.copy_(dev), torch.cuda.synchronize()), a.iters) / 1e9
    out["host_memcpy_1thread_GBps"] = S / timeit(lambda: np.copyto(dst, src), a.iters) / 1e9
    # e2e through libmpjx
    c = mpi.Init(0, 1, 0, mpi.unique_id())
    sp, rp = src.ctypes.data, dst.ctypes.data

    def ar():
        _lib.check(L.mpjx_allreduce_host(c.handle, sp, rp, n, 8, 3, 0), "allreduce_host")

    t = timeit(ar, a.iters)
    assert np.array_equal(dst, src)
    out["e2e_allreduce_host_P1_GBps"] = S / t / 1e9
    out["e2e_allreduce_host_P1_ms"] = t * 1e3
    # the pipeline chunk (MPJX_HOST_CHUNK_MIB, read per call)
    sweep = {}
    for mib in (8, 16, 32):
        os.environ["MPJX_HOST_CHUNK_MIB"] = str(mib)
        dst.fill(0)
        t = timeit(ar, a.iters)
        assert np.array_equal(dst, src)
        sweep[f"chunk{mib}MiB"] = round(S / t / 1e9, 2)
    os.environ.pop("MPJX_HOST_CHUNK_MIB")
    out["e2e_pageable_chunk_sweep_GBps"] = sweep
    # page-locked caller buffers: copied directly, no ring — torch's pinned allocator, and hipHostMalloc
    psrc = torch.from_numpy(src).pin_memory()
    pdst = torch.zeros(n, dtype=torch.float64).pin_memory()

    def ar_pinned(sp_, rp_):
        _lib.check(L.mpjx_allreduce_host(c.handle, sp_, rp_, n, 8, 3, 0), "allreduce_host")

    for mib in (8, 16, 32):
        os.environ["MPJX_HOST_CHUNK_MIB"] = str(mib)
        t = timeit(lambda: ar_pinned(psrc.data_ptr(), pdst.data_ptr()), a.iters)
        assert np.array_equal(pdst.numpy(), src)
        out[f"e2e_allreduce_host_P1_torch_pinned_chunk{mib}MiB_GBps"] = S / t / 1e9
    try:
        hip = L  # dlsym through libmpjx's handle resolves the HIP runtime it (and torch) already bound
        hs, hd = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(hs), ctypes.c_size_t(S), 0) == 0
        assert hip.hipHostMalloc(ctypes.byref(hd), ctypes.c_size_t(S), 0) == 0
        hsrc = np.ctypeslib.as_array((ctypes.c_double * n).from_address(hs.value))
        hdst = np.ctypeslib.as_array((ctypes.c_double * n).from_address(hd.value))
        hsrc[:] = src
        for mib in (8, 16, 32):
            os.environ["MPJX_HOST_CHUNK_MIB"] = str(mib)
            hdst.fill(0)
            t = timeit(lambda: ar_pinned(hs.value, hd.value), a.iters)
            assert np.array_equal(hdst, src)
            out[f"e2e_allreduce_host_P1_hipHostMalloc_chunk{mib}MiB_GBps"] = S / t / 1e9
        os.environ.pop("MPJX_HOST_CHUNK_MIB")
        del hsrc, hdst
        hip.hipHostFree(hs)
        hip.hipHostFree(hd)
    except Exception as e:  # noqa: BLE001
        out["hipHostMalloc_error"] = str(e)[:200]
    # the same with a big-endian (mpjbuf) payload in and the result back big-endian: the byte swap
    # happens inside the device kernels (MPJX_FLAG_SEND/RECV_BIG_ENDIAN), the host only copies
    sbe = src.byteswap()

    def ar_be():
        _lib.check(L.mpjx_allreduce_host(c.handle, sbe.ctypes.data, rp, n, 8, 3, 0xC), "allreduce_host BE")

    t = timeit(ar_be, a.iters)
    assert np.array_equal(dst.view(np.uint64), sbe.view(np.uint64))
    out["e2e_allreduce_host_P1_big_endian_GBps"] = S / t / 1e9
    c.Free()
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}))


if __name__ == "__main__":
    main()
