#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Allreduce(SUM,double) GB/s, device-resident, 256 MiB.

  python bench.py --gpus 1 --steps K --warmup W           # N = 1 (default)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

Workloads (a "step" = one pass of the hot path over one batch of resident synthetic input):
  N = 1: BASELINE configs[1] — local Op.SUM combine of two 256 MiB double[] on one MI355X
         (inout[i] = in[i] + inout[i], one mpjx_combine = one typed Op.perform over the buffer).
  N > 1: BASELINE configs[2] at N ranks — Allreduce SUM double, 256 MiB per rank, one process per
         GPU, libmpjx over RCCL/xGMI (exchange -> MST-order P-way HIP combine -> all-gather).
value = aggregate algorithm bandwidth = (sum over ranks of the 256 MiB vector each rank reduces) /
time per step (nccl-tests "algbw", summed over ranks). Inputs are resident in HBM before timing.
Rank 0 prints one JSON line. See DESIGN.md "Measurement" for every field.
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (before libmpjx: one HIP runtime per process)

HBM_PEAK_GBPS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBPS = 153.6    # per link per the brief / SURVEY §8d; 7 links per GPU
METRIC = "Allreduce(SUM,double) GB/s device-resident @256 MiB, 1/2/4/8 MI355X"
MPJX_SUM, MPJX_DOUBLE = 3, 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mib", type=int, default=256, help="bytes per rank buffer, MiB")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true", help="N>1: skip the comparison timings")
    return ap.parse_args()


def seed(cfg, rank):
    return 0x4D504A00 + 1000 * cfg + rank


def synth(n, s, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(s)
    return torch.rand(n, dtype=torch.float64, device=dev, generator=g) * 2.0 - 1.0


def traffic_from_profiles(kernel_tag):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(p))
        return d.get(kernel_tag, {}).get("hbm_bytes_per_launch")
    except Exception:  # noqa: BLE001
        return None


def cpu_baseline(n, budget_s):
    """The reference's host combine (typed-class round trip) timed on this host: oracle port."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU restatement, timed as the baseline only

    t1 = oracle.time_combine(oracle.SUM, oracle.DOUBLE, n, 1)
    reps = max(3, min(50, int(budget_s / max(t1, 1e-6))))
    t = oracle.time_combine(oracle.SUM, oracle.DOUBLE, n, reps)
    return {"value": round(n * 8 / t / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x full-size combine of 2 x {n * 8 >> 20} MiB double[] "
                      f"(new T[] + arraycopy + perform loop + getResultant, SumDouble.java:49-67), "
                      f"median {t * 1e3:.1f} ms, host {platform.processor() or platform.machine()}"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        a.gpus = world if world > 1 else a.gpus
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from mpjexpress_amd import _lib

    L = _lib.lib()
    n = a.mib * (1 << 20) // 8
    S = n * 8
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if dist is not None:
            dist.barrier()

    if world == 1:
        # ---- configs[1]: inout = in + inout, 2 x 256 MiB double, one kernel per step ----------
        stream = torch.cuda.Stream(device=dev)
        sp = ctypes.c_void_p(stream.cuda_stream)
        inout = synth(n, seed(2, 0), dev)
        inp = synth(n, seed(2, 1), dev)
        torch.cuda.synchronize()

        def step():
            _lib.check(L.mpjx_combine(MPJX_SUM, MPJX_DOUBLE, inout.data_ptr(), inp.data_ptr(), n, sp),
                       "mpjx_combine")

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            for i in range(a.steps):
                ev[i][0].record(stream)
                step()
                ev[i][1].record(stream)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / a.steps
        kern_s = sum(s.elapsed_time(e) for s, e in ev) / a.steps / 1e3
        alg = 3 * S  # read in, read inout, write inout
        achieved = alg / kern_s / 1e9
        traffic = traffic_from_profiles("combine_sum_f64_256MiB")
        out = {
            "metric": METRIC, "value": round(S / t / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(t * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: U[-1,1) doubles from torch.Generator, seed 0x4D504A00+1000*cfg+rank",
            "config": {"workload": "configs[1]: local Op.SUM combine of two 256 MiB double[] on 1 MI355X "
                                   "(kernel only, no RCCL)",
                       "elements": n, "bytes_per_operand": S, "op": "SUM", "datatype": "DOUBLE",
                       "parallelism": "single GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "kernel": "k_pway<Sum<double>,2,K_FOLD,2,4>",
                         "algorithmic_bytes_per_launch": alg, "kernel_us": round(kern_s * 1e6, 2)},
        }
        if not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(n, a.cpu_seconds)
        print(json.dumps(out), flush=True)
        return

    # ---- N > 1: configs[2] Allreduce SUM double 256 MiB per rank over RCCL/xGMI ----------------
    uid = [None]
    if rank == 0:
        uid[0] = _lib_unique_id(L)
    dist.broadcast_object_list(uid, src=0)
    comm = ctypes.c_void_p()
    _lib.check(L.mpjx_comm_init_rank(ctypes.byref(comm), world, uid[0], rank, local), "mpjx_comm_init_rank")
    sp = ctypes.c_void_p()
    _lib.check(L.mpjx_comm_stream(comm, ctypes.byref(sp)), "mpjx_comm_stream")
    send = synth(n, seed(3, rank), dev)
    recv = torch.empty_like(send)
    torch.cuda.synchronize()

    def step():
        _lib.check(L.mpjx_allreduce(comm, send.data_ptr(), recv.data_ptr(), n, MPJX_DOUBLE, MPJX_SUM, 0, sp),
                   "mpjx_allreduce")

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        _lib.check(L.mpjx_comm_synchronize(comm), "sync")
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        _lib.check(L.mpjx_comm_synchronize(comm), "sync")
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        barrier()
        return el.item() / steps

    t = timed(step, a.steps, a.warmup)
    algbw = S / t / 1e9
    busbw = algbw * 2 * (world - 1) / world
    peak = (world - 1) * XGMI_LINK_GBPS
    # comparison timings for tuning (not the reported value): same call with the chunk pipeline
    # off, with grouped ncclSend/ncclRecv exchanges, and RCCL's own ncclAllReduce (not order-faithful)
    variants = {}
    if not a.no_variants:
        for name, env in (("no_pipeline", {"MPJX_PIPE_CHUNK_MIB": "0"}), ("rccl_p2p", {"MPJX_RCCL_P2P": "1"})):
            try:
                old_env = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                tv = timed(step, max(3, a.steps // 2), 2)
                variants[name] = {"ms": round(tv * 1e3, 4), "busbw_GBps": round(S / tv / 1e9 * 2 * (world - 1) / world, 2)}
            except Exception as e:  # noqa: BLE001
                variants[name] = {"error": str(e)[:200]}
            finally:
                for k, v in old_env.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
        try:
            g = dist.new_group(backend="nccl")
            ref = send.clone()

            def rstep():
                dist.all_reduce(ref, group=g)

            tv = timed(rstep, max(3, a.steps // 2), 2)
            variants["rccl_native_allreduce"] = {"ms": round(tv * 1e3, 4),
                                                 "busbw_GBps": round(S / tv / 1e9 * 2 * (world - 1) / world, 2),
                                                 "note": "torch RCCL all_reduce, ring order: not bit-exact vs the reference"}
        except Exception as e:  # noqa: BLE001
            variants["rccl_native_allreduce"] = {"error": str(e)[:200]}
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(world * algbw, 2), "unit": "GB/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(t * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: U[-1,1) doubles from torch.Generator, seed 0x4D504A00+1000*cfg+rank",
            "config": {"workload": f"configs[2] at {world} ranks: Allreduce SUM double 256 MiB per rank, "
                                   "one process per MI355X via libmpjx over RCCL/xGMI",
                       "elements": n, "bytes_per_rank": S, "op": "SUM", "datatype": "DOUBLE",
                       "parallelism": f"rccl-xgmi x{world}"},
            "algbw_GBps_per_rank": round(algbw, 2), "busbw_GBps": round(busbw, 2),
            "roofline": {"bound": "xgmi", "achieved": round(busbw, 1), "peak": round(peak, 1),
                         "unit": "GB/s", "frac": round(busbw / peak, 4), "traffic": None,
                         "note": "busBW = algBW*2(P-1)/P against (P-1) direct xGMI links"},
            "variants": variants,
        }
        print(json.dumps(out), flush=True)
    L.mpjx_comm_destroy(comm)
    dist.destroy_process_group()


def _lib_unique_id(L):
    buf = ctypes.create_string_buffer(128)
    from mpjexpress_amd import _lib

    _lib.check(L.mpjx_get_unique_id(buf), "mpjx_get_unique_id")
    return buf.raw


if __name__ == "__main__":
    main()
