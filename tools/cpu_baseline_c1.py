"""BASELINE configs[0]: Allreduce SUM double[] 1 MiB, -np 4 multicore — the reference's CPU path,
timed as the oracle's restatement (MST_Reduce + MST_Bcast, 4 ranks as 4 pinned threads, big-endian
mpjbuf pack/unpack on every hop; oracle/mpjx_oracle.c ora_time_allreduce_mst) next to libmpjx in
multicore mode on one GPU (4 ranks as threads, device-resident) for the same shape.

  python tools/cpu_baseline_c1.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402  (the CPU restatement, timed as a baseline)
from mpjexpress_amd import mpi  # noqa: E402
from mpjexpress_amd.mpi import MPI  # noqa: E402

P, n = 4, (1 << 20) // 8
out = {"config": "configs[0]: Allreduce SUM double[] 1 MiB, 4 ranks", "bytes": n * 8}
t = oracle.time_allreduce_mst(P, n, 50, pin=True)
out["cpu_reference_restatement_ms"] = round(t * 1e3, 4)
out["cpu_algbw_GBps"] = round(n * 8 / t / 1e9, 3)
if torch.cuda.is_available():
    comms = mpi.smp_world(P, [0] * P)

    def body(c):
        s = torch.rand(n, dtype=torch.float64, device="cuda")
        d = torch.empty_like(s)
        for _ in range(5):
            c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
        c.Barrier()
        t0 = time.perf_counter()
        for _ in range(50):
            c.Allreduce(s, 0, d, 0, n, MPI.DOUBLE, MPI.SUM)
        c.Barrier()
        return (time.perf_counter() - t0) / 50

    ts = mpi.run_multicore(comms, body)
    out["gpu_multicore_1gpu_ms"] = round(max(ts) * 1e3, 4)  # direct engine (default in multicore mode)
    os.environ["MPJX_SMP_COPY"] = "1"
    for name, kib in (("two_exchange", "0"), ("oneshot_allgather", "4096")):
        os.environ["MPJX_ONESHOT_KIB"] = kib
        ts = mpi.run_multicore(comms, body)
        out[f"gpu_multicore_1gpu_copy_engine_{name}_ms"] = round(max(ts) * 1e3, 4)
    del os.environ["MPJX_SMP_COPY"], os.environ["MPJX_ONESHOT_KIB"]
    for c in comms:
        c.Free()
    out["note"] = "GPU multicore ranks share one MI355X; per-call latency includes the host rendezvous"
print(json.dumps(out))
