"""One rank of a multi-process libmpjx world (mpjx_comm_init_ipc), driven by tests/test_gpu_ipc.py.

    python tests/ipc_worker.py RANK P UID_HEX CASES_JSON OUT_DIR

Ranks are separate processes (as niodev ranks started by the reference's runtime are), all on
cuda:0 here: the IPC engine maps every other rank's buffers, so the collectives run exactly as they
do with one process per GPU, only with the peers' memory on the same device. Each case's inputs are
regenerated from its seed by the parent, which checks the saved outputs against the oracle.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")]
if os.environ.get("MPJX_TEST_STALL_REPORT_S"):  # a world far past its usual 3-6 s: where each rank waits
    import watchdog

    watchdog.arm(os.environ["MPJX_TEST_STALL_REPORT_S"], exit_after=False)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from util import make_input  # noqa: E402  (seeded inputs; oracle constants only, no oracle calls)


def case_input(case, total, rank, rep):
    """Rank `rank`'s send vector of a case: seeded edge-value inputs (tests/util.py), or BASELINE's
    synthetic streams (case["synth"] = config number: tools/synth.py, as bench.py generates them)."""
    if "synth" in case:
        import synth

        return synth.uniform_np(np.arange(total, dtype=np.uint64), synth.seed(case["synth"], rank))
    return make_input(case["type"], total, case["seed"] * 1000 + rank + 100 * rep, op=case["op"])


def tensor(a, host=None):
    """The buffer a rank passes: a device tensor, or (host = "pageable" | "pinned") a host numpy array,
    which mpi.py routes to the mpjx_*_host entry points (niodev ranks' Java arrays)."""
    if a.dtype.names:
        a = a.view(a.dtype[0])
    if host == "pageable":
        return np.array(a, copy=True)
    if host == "pinned":  # page-locked (hipHostMalloc'd by torch); the array keeps the tensor alive
        return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run_case(comm, case, rank, P, out_dir):
    from mpjexpress_amd import mpi
    from mpjexpress_amd.mpi import MPI

    for k, v in case.get("env", {}).items():
        os.environ[k] = v
    MPI.isOldSelected = bool(case.get("flags", 0) & 1)
    comm.faithful = bool(case.get("flags", 0) & 2)  # MPJX_FLAG_FAITHFUL (every rank's Reduce recvbuf)
    dt, op = mpi.datatype(case["type"]), mpi.OPS[case["op"] - 1]
    kind, n, rc = case["kind"], case.get("n", 0), case.get("recvcounts")
    total = sum(rc) if rc is not None else n
    s = out = None
    host = case.get("host")
    for rep in range(case.get("reps", 1)):
        # rep > 0: new data in the same buffers, or (realloc) fresh buffers — new HIP allocations
        x = case_input(case, total, rank, rep)
        like = x[:1]
        off = case.get("off", 0)  # element offset into both buffers (misaligned device pointers)
        xo = np.concatenate([np.zeros(off, x.dtype), x]) if off else x
        if s is None or case.get("realloc"):
            # new tensors from torch's caching allocator; device memory is never handed back to the
            # driver while the world lives (no empty_cache): on a GPU oversubscribed by rank processes,
            # a kernel can read a stale translation of a freed and re-allocated page
            s = out = None
            torch.cuda.synchronize()
            s = tensor(xo, host)
            if kind == "reduce_scatter":
                out = tensor(np.zeros(off + max(1, rc[rank]), x.dtype), host)
            elif kind != "bcast":
                out = s if case.get("inplace") else tensor(np.zeros(off + max(1, n), x.dtype), host)
        elif host:
            np.copyto(s, xo.view(s.dtype))
        else:
            s.copy_(tensor(xo))
        bo = off * dt.size  # offsets are in base elements (Java array indices)
        if kind == "reduce_scatter":
            comm.Reduce_scatter(s, bo, out, bo, rc, dt, op)
            m = rc[rank]
        else:
            if kind == "allreduce":
                comm.Allreduce(s, bo, out, bo, n, dt, op)
            elif kind == "reduce":
                comm.Reduce(s, bo, out, bo, n, dt, op, case["root"])
            elif kind == "scan":
                comm.Scan(s, bo, out, bo, n, dt, op)
            elif kind == "bcast":
                comm.Bcast(s, bo, n, dt, case["root"])
                out = s
            m = n
        if case.get("nosave"):  # large-size smoke: finish, report, keep no output
            torch.cuda.synchronize()
            print(f"rank {rank} {case['id']} pass {rep} done", flush=True)
            continue
        res = np.array(out, copy=True) if host else out.cpu().numpy()
        res = res.view(like.dtype) if like.dtype.names else res
        np.save(os.path.join(out_dir, f"{case['id']}_r{rank}_p{rep}.npy"), res[off:off + m])
        if comm.faithful and kind == "reduce_scatter":  # the BKT ring's sendbuf overwrite
            sv = np.array(s, copy=True) if host else s.cpu().numpy()
            np.save(os.path.join(out_dir, f"{case['id']}_send_r{rank}_p{rep}.npy"), sv[off:off + total])
    del s, out
    torch.cuda.synchronize()
    comm.faithful = False
    for k in case.get("env", {}):
        os.environ.pop(k, None)


def main():
    rank, P, uid_hex, cases_json, out_dir = sys.argv[1:6]
    rank, P = int(rank), int(P)
    torch.cuda.set_device(0)
    # tools/queue_census.py: streams of the rank process's own beside torch's and the communicator's, each
    # used once so the HIP runtime gives it a hardware queue (up to GPU_MAX_HW_QUEUES per process)
    extra = [torch.cuda.Stream() for _ in range(int(os.environ.get("MPJX_TEST_EXTRA_STREAMS", "0")))]
    for st in extra:
        with torch.cuda.stream(st):
            torch.ones(1, device="cuda").add_(1)
    torch.cuda.synchronize()
    from mpjexpress_amd import mpi

    cases = json.load(open(cases_json))
    if cases and cases[0]["kind"] == "init_refused":  # the world must refuse to form: record why
        try:
            mpi.InitIPC(rank, P, 0, bytes.fromhex(uid_hex))
            rc, msg = 0, ""
        except mpi.MPIException as e:
            rc, msg = -1, str(e)
        with open(os.path.join(out_dir, f"init_r{rank}.txt"), "w") as f:
            f.write(f"{rc} {msg}")
        return
    import time

    t0 = time.perf_counter()
    comm = mpi.InitIPC(rank, P, 0, bytes.fromhex(uid_hex))
    print(f"rank {rank} init {time.perf_counter() - t0:.2f} s", flush=True)
    for case in cases:
        # progress on stdout (tests/test_gpu_ipc.py launch() shows every rank's last lines on a timeout)
        print(f"rank {rank} {case.get('id')} start t={time.perf_counter() - t0:.2f} s", flush=True)
        if case["kind"] == "fail":  # rank `root` passes a host pointer: every rank must get an error
            import ctypes

            from mpjexpress_amd import _lib

            n = 1024
            buf = torch.zeros(n, dtype=torch.float64, device="cuda")
            host = np.zeros(n)
            send = host.ctypes.data if rank == case["root"] else buf.data_ptr()
            rc = _lib.lib().mpjx_allreduce(comm.handle, ctypes.c_void_p(send), ctypes.c_void_p(buf.data_ptr()),
                                           n, 8, 3, 0, None)
            if rc == 0:  # MPJX_IPC_SYNC=device: the call is enqueued; a failed peer shows at the sync
                rc = _lib.lib().mpjx_comm_synchronize(comm.handle)
            with open(os.path.join(out_dir, f"{case['id']}_r{rank}.txt"), "w") as f:
                f.write(f"{rc} {_lib.lib().mpjx_last_error().decode()}")
            continue
        if case["kind"] == "split":  # Split of the IPC world: each sub-world is an IPC world of its own
            color = rank % case["colors"]
            sub = comm.Split(color, -rank)  # key -rank: new ranks in descending parent order
            x = case_input(case, case["n"], rank, 0)
            s = tensor(x)
            out = torch.zeros_like(s)
            from mpjexpress_amd import mpi as _m

            sub.Allreduce(s, 0, out, 0, case["n"], _m.datatype(case["type"]), _m.OPS[case["op"] - 1])
            np.save(os.path.join(out_dir, f"{case['id']}_r{rank}.npy"), out.cpu().numpy())
            with open(os.path.join(out_dir, f"{case['id']}_r{rank}.txt"), "w") as f:
                f.write(f"{sub.Rank()} {sub.Size()}")
            sub.Free()
            continue
        run_case(comm, case, rank, P, out_dir)
    comm.Free()
    print(f"rank {rank} done", flush=True)


if __name__ == "__main__":
    main()
