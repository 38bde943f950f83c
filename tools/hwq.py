"""Hardware-queue budget of rank processes that share ONE GPU (one-GPU rehearsals of the multi-process
engines: tests/test_gpu_ipc.py worlds, `bench.py --one-device`). DESIGN.md §6 "The P = 8 push-world stall".

The GPU's scheduler (HWS, KFD sched_policy 0) maps at most `num_cp_queues` user compute queues at once
(KFD topology of the MI355X node: 24, each mapped on all 8 XCCs in SPX mode); with more queues active the
runlist is over-subscribed and the HWS time-slices them, so a rank whose queue is not mapped makes no
progress until its turn while every other rank waits for it at the call's rendezvous. HIP gives a process
up to GPU_MAX_HW_QUEUES hardware queues (one per stream until the cap; 4 is HIP's default and this box's
setting). So P rank processes plus one launching process that already holds a GPU context (the pytest
process: up to 4 queues) stay within the mapped set iff P * q + 4 <= num_cp_queues: the cap below.
Copy engines likewise: the node has num_sdma_engines x num_sdma_queues_per_engine = 2 x 8 user SDMA
queues, and every process that copies between host and device may open its own; rehearsal ranks run
with HSA_ENABLE_SDMA=0 (their copies become blit kernels on their compute queues), so they open none."""
import glob

KFD_CP_QUEUES_DEFAULT = 24   # MI355X KFD topology (profiles/r06/census_f.json)
PARENT_RESERVE = 4           # a launching process's own queues (HIP's default cap)
HIP_DEFAULT = 4


def cp_queues():
    """The GPU node's num_cp_queues from the KFD topology (the first GPU node), else the MI355X value."""
    for props in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        try:
            kv = dict(ln.split()[:2] for ln in open(props) if len(ln.split()) >= 2)
        except OSError:
            continue
        if kv.get("simd_count", "0") != "0" and kv.get("num_cp_queues", "0").isdigit():
            return int(kv["num_cp_queues"])
    return KFD_CP_QUEUES_DEFAULT


def per_process_cap(nprocs, cp=None):
    """GPU_MAX_HW_QUEUES for each of `nprocs` rank processes sharing one GPU: at most HIP's default, at
    least 1, and nprocs * cap + PARENT_RESERVE <= the queues the GPU maps at once."""
    cp = cp_queues() if cp is None else cp
    return max(1, min(HIP_DEFAULT, (cp - PARENT_RESERVE) // max(1, nprocs)))


def rehearsal_env(nprocs, env=None):
    """Environment for `nprocs` rank processes sharing one GPU: capped compute queues, no SDMA queues."""
    env = env if env is not None else {}
    cur = int(env.get("GPU_MAX_HW_QUEUES", str(HIP_DEFAULT)) or HIP_DEFAULT)
    return {"GPU_MAX_HW_QUEUES": str(min(cur, per_process_cap(nprocs))), "HSA_ENABLE_SDMA": "0"}
