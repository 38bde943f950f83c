"""Probe: can the RCCL exchange engine run with two rank processes on ONE GPU? (The multi-GPU path's
RCCL calls — AllToAll, AllGather, grouped Send/Recv — have otherwise run only at world size 1 here.)

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29531 tools/rccl_two_rank_probe.py

Each rank: gloo for the unique id, mpjx_comm_init_rank on cuda:0, then Allreduce / Reduce_scatter /
Scan of SUM double at a few sizes (equal blocks -> ncclAllToAll + ncclAllGather; ragged ->
ncclAllToAllv / grouped p2p) and MPJX_RCCL_P2P=1, every result checked bit for bit against the
oracle on rank 0. Buffers are allocated once and never freed while the world lives.
Rank 0 prints one JSON line: {"ok": bool, ...} or the error RCCL gave."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
os.environ.setdefault("MPJX_RCCL_TIMEOUT_S", "30")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle as O  # noqa: E402  (the checker)
from mpjexpress_amd import _lib  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = _lib.lib()
    buf = ctypes.create_string_buffer(128)
    if rank == 0:
        _lib.check(L.mpjx_get_unique_id(buf), "uid")
    uid = [buf.raw if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    torch.cuda.set_device(0)
    c = ctypes.c_void_p()
    rc = L.mpjx_comm_init_rank(ctypes.byref(c), world, uid[0], rank, 0)
    res = {"world": world, "init_rc": rc}
    if rc != 0:
        res["error"] = (L.mpjx_last_error() or b"").decode()
        out = [None] * world
        dist.all_gather_object(out, res)
        if rank == 0:
            print(json.dumps({"ok": False, "ranks": out}), flush=True)
        return 0
    bad, cases = [], []
    for n in (1000, 1 << 20, (1 << 20) + 7):
        rng = np.random.default_rng(1234 + n)
        xs = [rng.uniform(-1, 1, n) for _ in range(world)]
        send = torch.from_numpy(xs[rank]).cuda()
        recv = torch.empty_like(send)
        for p2p in ("0", "1"):
            os.environ["MPJX_RCCL_P2P"] = p2p
            r1 = L.mpjx_allreduce(c, send.data_ptr(), recv.data_ptr(), n, 8, 3, 0, None)
            r2 = L.mpjx_comm_synchronize(c)
            got = recv.cpu().numpy()
            exp = O.allreduce(xs, n, O.DOUBLE, O.SUM)[rank]
            ok = r1 == 0 and r2 == 0 and np.array_equal(got.view(np.uint64), exp.view(np.uint64))
            cases.append({"op": "allreduce", "n": n, "p2p": p2p, "ok": bool(ok)})
            counts = [n // world + (1 if j < n % world else 0) for j in range(world)]
            rcv = torch.empty(counts[rank], dtype=torch.float64, device="cuda")
            cnt = (ctypes.c_int64 * world)(*counts)
            r1 = L.mpjx_reduce_scatter(c, send.data_ptr(), rcv.data_ptr(), cnt, 8, 3, 0, None)
            r2 = L.mpjx_comm_synchronize(c)
            exp = O.reduce_scatter(xs, counts, O.DOUBLE, O.SUM)[0][rank]
            ok = r1 == 0 and r2 == 0 and np.array_equal(rcv.cpu().numpy().view(np.uint64), exp.view(np.uint64))
            cases.append({"op": "reduce_scatter", "n": n, "p2p": p2p, "ok": bool(ok)})
            r1 = L.mpjx_scan(c, send.data_ptr(), recv.data_ptr(), n, 8, 3, 0, None)
            r2 = L.mpjx_comm_synchronize(c)
            exp = O.scan(xs, n, O.DOUBLE, O.SUM)[rank]
            ok = r1 == 0 and r2 == 0 and np.array_equal(recv.cpu().numpy().view(np.uint64), exp.view(np.uint64))
            cases.append({"op": "scan", "n": n, "p2p": p2p, "ok": bool(ok)})
    bad = [k for k in cases if not k["ok"]]
    out = [None] * world
    dist.all_gather_object(out, {"rank": rank, "bad": bad, "n_cases": len(cases)})
    if rank == 0:
        print(json.dumps({"ok": all(not o["bad"] for o in out), "ranks": out}), flush=True)
    L.mpjx_comm_destroy(c)
    return 0


if __name__ == "__main__":
    sys.exit(main())
