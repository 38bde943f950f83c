"""configs[4] pipeline check: Allreduce MAX float 1 GiB per rank, P = 8 multicore ranks on one GPU
through the exchange engine (MPJX_SMP_COPY=1: the RCCL engine's code path — exchange #1, P-way
combine on the communicator's combine stream, all-gather — with device copies as the transport).

  python tools/c5_overlap.py [--calls 3]              time pipelined (64 MiB chunks) vs unchunked
  python tools/c5_overlap.py --trace-run              two pipelined calls (run under rocprofv3 --kernel-trace)
  python tools/c5_overlap.py --analyze KERNEL_TRACE.csv
      from a rocprofv3 kernel trace: time during which a combine kernel (k_pway, on a combine stream)
      runs while an exchange copy (the runtime's copy kernels, on the collective streams) runs
"""
import argparse
import csv
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]


def run(calls, trace_run):
    import torch

    import synth
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    os.environ["MPJX_SMP_COPY"] = "1"
    P, n = 8, (1 << 30) // 4
    dev = torch.device("cuda", 0)
    sends = [synth.uniform_torch(n, 0x4D504A00 + 5000 + r, dev, -1e3, 1e3).to(torch.float32) for r in range(P)]
    recvs = [torch.empty_like(s) for s in sends]
    torch.cuda.synchronize()
    comms = mpi.smp_world(P, [0] * P)
    out = {}
    modes = [("pipelined_64MiB", "64")] if trace_run else [("pipelined_64MiB", "64"), ("unchunked", "0"),
                                                          ("pipelined_64MiB_again", "64")]
    try:
        for name, chunk in modes:
            os.environ["MPJX_PIPE_CHUNK_MIB"] = chunk
            k = 2 if trace_run else calls

            def body(c):
                r = c.Rank()
                c.Allreduce(sends[r], 0, recvs[r], 0, n, MPI.FLOAT, MPI.MAX)  # warm-up (scratch growth)
                c.Barrier()
                t0 = time.perf_counter()
                for _ in range(k):
                    c.Allreduce(sends[r], 0, recvs[r], 0, n, MPI.FLOAT, MPI.MAX)
                c.Barrier()
                return (time.perf_counter() - t0) / k

            ts = mpi.run_multicore(comms, body)
            out[name] = {"ms": round(max(ts) * 1e3, 3), "calls": k}
        # bit-exactness of the last call against a torch max over the ranks (MAX is order-independent
        # for these finite inputs)
        ref = sends[0].clone()
        for s in sends[1:]:
            torch.maximum(ref, s, out=ref)
        out["bit_exact_vs_elementwise_max"] = all(bool(torch.equal(r.view(torch.int32), ref.view(torch.int32)))
                                                  for r in recvs)
    finally:
        for c in comms:
            c.Free()
    out["config"] = "configs[4]: Allreduce MAX float 1 GiB per rank, 8 multicore ranks on one MI355X, exchange engine"
    print(json.dumps(out), flush=True)


def lanes(P, chunk_mib, calls):
    """Round 3: the pipeline's two exchange lanes. One instrumented call per
    repetition (mpjx_comm_phase_timing + mpjx_comm_pipeline_trace on rank 0): per chunk the intervals
    of exchange #1 (call stream), combine (combine stream) and all-gather (gather stream, the second
    lane); reports how long an all-gather ran while some exchange #1 ran, and the call time pipelined vs
    unchunked. configs[4] data: Allreduce MAX float 1 GiB per rank, P multicore ranks on one GPU,
    exchange engine (MPJX_SMP_COPY=1, device copies as the transport)."""
    import ctypes

    import torch

    import synth
    from mpjexpress_amd import _lib, mpi
    from mpjexpress_amd.mpi import MPI

    os.environ["MPJX_SMP_COPY"] = "1"
    L = _lib.lib()
    n = (1 << 30) // 4
    dev = torch.device("cuda", 0)
    sends = [synth.uniform_torch(n, 0x4D504A00 + 5000 + r, dev, -1e3, 1e3).to(torch.float32) for r in range(P)]
    recvs = [torch.empty_like(s) for s in sends]
    torch.cuda.synchronize()
    comms = mpi.smp_world(P, [0] * P)
    out = {"P": P, "chunk_MiB": chunk_mib, "config": "configs[4] Allreduce MAX float 1 GiB per rank, multicore "
                                                        "ranks on one MI355X, exchange engine"}
    try:
        times = {}
        for name, chunk in (("unchunked", "0"), ("pipelined", str(chunk_mib))):
            os.environ["MPJX_PIPE_CHUNK_MIB"] = chunk

            def body(c):
                r = c.Rank()
                c.Allreduce(sends[r], 0, recvs[r], 0, n, MPI.FLOAT, MPI.MAX)  # warm-up
                c.Barrier()
                t0 = time.perf_counter()
                for _ in range(calls):
                    c.Allreduce(sends[r], 0, recvs[r], 0, n, MPI.FLOAT, MPI.MAX)
                c.Barrier()
                return (time.perf_counter() - t0) / calls

            times[name] = round(max(mpi.run_multicore(comms, body)) * 1e3, 3)
        out["ms_per_call"] = times

        def traced(c):
            r = c.Rank()
            _lib.check(L.mpjx_comm_phase_timing(c.handle, 1), "phase on")
            c.Allreduce(sends[r], 0, recvs[r], 0, n, MPI.FLOAT, MPI.MAX)
            res = None
            if r == 0:
                ms = (ctypes.c_float * (6 * 64))()
                nch = ctypes.c_int()
                _lib.check(L.mpjx_comm_pipeline_trace(c.handle, ms, 6 * 64, ctypes.byref(nch)), "trace")
                res = [list(ms[6 * k:6 * k + 6]) for k in range(nch.value)]
            _lib.check(L.mpjx_comm_phase_timing(c.handle, 0), "phase off")
            return res

        tr = mpi.run_multicore(comms, traced)[0]
        ex1 = [(a[0], a[1]) for a in tr]
        comb = [(a[2], a[3]) for a in tr]
        gat = [(a[4], a[5]) for a in tr]

        def inter(x, y):
            return max(0.0, min(x[1], y[1]) - max(x[0], y[0]))

        g_with_e = sum(sum(inter(g, e) for e in ex1) for g in gat)
        c_with_x = sum(sum(inter(cb, e) for e in ex1 + gat) for cb in comb)
        out["trace_chunks"] = len(tr)
        out["exchange1_busy_ms"] = round(sum(e[1] - e[0] for e in ex1), 3)
        out["allgather_busy_ms"] = round(sum(g[1] - g[0] for g in gat), 3)
        out["combine_busy_ms"] = round(sum(cb[1] - cb[0] for cb in comb), 3)
        out["allgather_while_exchange1_ms"] = round(g_with_e, 3)
        out["combine_while_an_exchange_ms"] = round(c_with_x, 3)
        out["call_span_ms"] = round(max(g[1] for g in gat), 3)
        out["intervals_ms_rank0"] = [[round(v, 3) for v in a] for a in tr]
        ref = sends[0].clone()
        for x in sends[1:]:
            torch.maximum(ref, x, out=ref)
        out["bit_exact_vs_elementwise_max"] = all(bool(torch.equal(r.view(torch.int32), ref.view(torch.int32)))
                                                  for r in recvs)
    finally:
        for c in comms:
            c.Free()
    print(json.dumps(out), flush=True)


def analyze(path):
    comb, copy = [], []
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            iv = (int(row["Start_Timestamp"]), int(row["End_Timestamp"]))
            if "k_pway" in name:
                comb.append(iv)
            elif "copyBuffer" in name or "k_copies" in name:
                copy.append(iv)

    def union(ivs):
        out = []
        for s, e in sorted(ivs):
            if out and s <= out[-1][1]:
                out[-1][1] = max(out[-1][1], e)
            else:
                out.append([s, e])
        return out

    uc, ux = union(comb), union(copy)
    both = 0
    i = j = 0
    while i < len(uc) and j < len(ux):
        s, e = max(uc[i][0], ux[j][0]), min(uc[i][1], ux[j][1])
        both += max(0, e - s)
        if uc[i][1] < ux[j][1]:
            i += 1
        else:
            j += 1
    tc = sum(e - s for s, e in uc)
    tx = sum(e - s for s, e in ux)
    span = (max(e for _, e in comb + copy) - min(s for s, _ in comb + copy)) if comb and copy else 0
    print(json.dumps({"combine_kernels": len(comb), "copy_kernels": len(copy), "combine_busy_us": round(tc / 1e3, 1),
                      "copy_busy_us": round(tx / 1e3, 1), "overlap_us": round(both / 1e3, 1),
                      "overlap_frac_of_combine": round(both / tc, 3) if tc else None,
                      "span_us": round(span / 1e3, 1), "serial_sum_us": round((tc + tx) / 1e3, 1)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--trace-run", action="store_true")
    ap.add_argument("--analyze")
    ap.add_argument("--lanes", type=int, default=0, help="P: the two-lane pipeline trace (round 3)")
    ap.add_argument("--chunk-mib", type=int, default=64)
    a = ap.parse_args()
    if a.lanes:
        lanes(a.lanes, a.chunk_mib, a.calls)
    elif a.analyze:
        analyze(a.analyze)
    else:
        run(a.calls, a.trace_run)


if __name__ == "__main__":
    main()
