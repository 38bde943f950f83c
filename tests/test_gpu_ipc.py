"""GPU: the cross-process direct engine (mpjx_comm_init_ipc) — ranks are separate processes that map
each other's device buffers through HIP IPC, as one process per GPU does on an 8-GPU node.

Here every rank process sits on cuda:0 (the box has one GPU), so the code path is the multi-process
one end to end — shared-memory rendezvous, IPC handle export/open/cache, one P-way kernel per rank
reading every rank's send block and writing every rank's recv block — with the peers' memory on the
same device instead of across xGMI. Results are compared bit-exactly with the oracle's restatement
of the reference algorithms (src/mpi/PureIntracomm.java), float/double included.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from ipc_worker import case_input
from util import same_bits


pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(HERE)


def cases_for(P):
    rc = [(37 * r + 5) % 23 * 41 for r in range(P)]  # ragged, one block may be empty
    rc[P // 2] = 0
    return [
        dict(id="ar_sum_f64", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=100003, seed=1),
        dict(id="ar_sum_f64_old", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=4099, seed=2, flags=O.FLAG_OLD),
        dict(id="ar_max_f32", kind="allreduce", op=O.MAX, type=O.FLOAT, n=4099, seed=3),
        dict(id="ar_band_i32", kind="allreduce", op=O.BAND, type=O.INT, n=65541, seed=4),
        dict(id="ar_sum_char", kind="allreduce", op=O.SUM, type=O.CHAR, n=1037, seed=5),
        dict(id="ar_maxloc_d2", kind="allreduce", op=O.MAXLOC, type=O.DOUBLE2, n=2053, seed=6),
        dict(id="ar_inplace", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=8191, seed=7, inplace=True),
        dict(id="ar_realloc", kind="allreduce", op=O.PROD, type=O.FLOAT, n=3001, seed=8, realloc=True, reps=3),
        dict(id="ar_reuse", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=50021, seed=18, reps=3),
        dict(id="rs_reuse", kind="reduce_scatter", op=O.MAX, type=O.LONG, recvcounts=[777] * P, seed=19,
             reps=2),
        dict(id="ar_exchange", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=100003, seed=9,
             env={"MPJX_SMP_COPY": "1"}),
        dict(id="ar_big", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=(16 << 20) // 8 + 3, seed=10),
        dict(id="red_root_last", kind="reduce", op=O.SUM, type=O.DOUBLE, n=7777, root=P - 1, seed=11),
        dict(id="red_min_root0_old", kind="reduce", op=O.MIN, type=O.FLOAT, n=777, root=0, seed=12,
             flags=O.FLAG_OLD),
        dict(id="rs_ragged", kind="reduce_scatter", op=O.SUM, type=O.DOUBLE, recvcounts=rc, seed=13),
        dict(id="rs_bxor", kind="reduce_scatter", op=O.BXOR, type=O.INT, recvcounts=[1000] * P, seed=14),
        dict(id="scan_sum_f64", kind="scan", op=O.SUM, type=O.DOUBLE, n=3001, seed=15),
        dict(id="scan_lor", kind="scan", op=O.LOR, type=O.BOOLEAN, n=513, seed=16),
        dict(id="bcast", kind="bcast", op=O.SUM, type=O.DOUBLE, n=5000, root=P - 1, seed=17),
        # misaligned device pointers (2-, 4- and 1-byte offsets): the unaligned copy/combine paths
        dict(id="ar_char_off1", kind="allreduce", op=O.MAX, type=O.CHAR, n=70001, seed=24, off=1),
        dict(id="rs_int_off3", kind="reduce_scatter", op=O.BXOR, type=O.INT, recvcounts=[3001] * P, seed=25, off=3),
        dict(id="scan_byte_off5", kind="scan", op=O.SUM, type=O.BYTE, n=9999, seed=26, off=5),
        # larger than a 1 MiB staging window (test_ipc_windows): windowed calls / exchange rounds
        dict(id="rs_big", kind="reduce_scatter", op=O.SUM, type=O.DOUBLE,
             recvcounts=[(r + 1) * 50021 for r in range(P)], seed=20),
        dict(id="scan_big", kind="scan", op=O.MIN, type=O.FLOAT, n=400003, seed=21),
        dict(id="red_big", kind="reduce", op=O.PROD, type=O.DOUBLE, n=300007, root=1 % P, seed=22),
        dict(id="bcast_big", kind="bcast", op=O.SUM, type=O.LONG, n=300001, root=0, seed=23),
        # exactly one 1 MiB staging window (one window since the slot-rounding slack), and one element more
        dict(id="ar_stage_exact", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=(1 << 20) // 8, seed=27),
        dict(id="ar_stage_plus1", kind="allreduce", op=O.MAX, type=O.DOUBLE, n=(1 << 20) // 8 + 1, seed=28),
    ]


def expected(case, P, rep=0):
    t, op, flags = case["type"], case["op"], case.get("flags", 0)
    rc = case.get("recvcounts")
    total = sum(rc) if rc is not None else case["n"]
    sends = [case_input(case, total, r, rep) for r in range(P)]
    if case.get("inplace"):
        sends = [s.copy() for s in sends]
    k, n = case["kind"], case.get("n")
    if k == "allreduce":
        return O.allreduce(sends, n, t, op, flags=flags)
    if k == "reduce":
        return O.reduce(sends, n, t, op, case["root"], flags=flags)
    if k == "scan":
        return O.scan(sends, n, t, op, flags=flags)
    if k == "bcast":
        return [sends[case["root"]]] * P
    exp, _ = O.reduce_scatter(sends, list(rc), t, op, flags=flags)
    return exp


def launch(P, cases, tmp_path, env_extra=None, timeout=None):
    """Run the case list in P rank processes on this GPU; returns every rank's output. Worlds with two
    rank processes on one GPU are refused by default (mpjx_comm_init_ipc); the workers
    never release device memory while their world exists, which is what makes such a world safe, so
    they opt in with MPJX_IPC_OVERSUBSCRIBE=1 (tests/conftest.py)."""
    # Every world here runs in 3-6 s (P = 8 included, profiles/r06/pytest_ipc_file_i.txt); 180 s is the
    # limit at every P (DESIGN.md §6 "The P = 8 one-GPU stalls").
    if timeout is None:
        timeout = 180
    uid = os.urandom(128).hex()
    cj = tmp_path / "cases.json"
    cj.write_text(json.dumps(cases))
    # a rank still running 45 s in (every world here takes 3-6 s) reports once, and runs on: its blocking
    # system call and native + Python stacks (tests/watchdog.py) land in its output and so in the
    # slow-world record below (DESIGN.md §6 "The P = 8 one-GPU stalls")
    env = dict(os.environ, MPJX_IPC_OVERSUBSCRIBE="1", MPJX_TEST_STALL_REPORT_S="45")
    env.update(env_extra or {})
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "ipc_worker.py"), str(r), str(P), uid,
                               str(cj), str(tmp_path)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True, env=env) for r in range(P)]
    import threading
    import time

    outs = [""] * P
    # read every rank's output as it comes (progress lines), so a timeout can show where each rank was
    def reader(r):
        outs[r] = "".join(procs[r].stdout)
    readers = [threading.Thread(target=reader, args=(r,), daemon=True) for r in range(P)]
    for t in readers:
        t.start()
    deadline = time.monotonic() + timeout
    try:
        for p in procs:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for t in readers:
            t.join(timeout=10)
        _slow_world_record(P, timeout, env_extra, outs, "timed out")
        raise AssertionError(f"P={P} rank processes still running after {timeout} s; last output per rank:\n" +
                             "\n".join(f"rank {r}: ...{outs[r][-400:]}" for r in range(P))) from None
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for t in readers:
        t.join(timeout=10)
    bad = [r for r, p in enumerate(procs) if p.returncode != 0]
    assert not bad, "\n".join(f"rank {r} exit {procs[r].returncode}:\n{outs[r][-2500:]}" for r in bad)
    took = timeout - (deadline - time.monotonic())
    if took > 30:
        _slow_world_record(P, took, env_extra, outs, "finished")
    return outs


def _slow_world_record(P, took, env_extra, outs, how):
    """A slow or timed-out world on the GPU box: keep every rank's whole output (progress lines and, past
    45 s, the stall report) under gpurun_out/slow_worlds/."""
    if not os.environ.get("GRAFT_REPO_ROOT"):
        return
    d = os.path.join(ROOT_DIR, "gpurun_out", "slow_worlds")
    os.makedirs(d, exist_ok=True)
    name = os.environ.get("PYTEST_CURRENT_TEST", "world").split(" ")[0].replace("/", "_").replace("::", "-")
    # whether this (launching) process held a GPU context: the round-5 slow worlds ran after the
    # in-process suite had given it one
    ctx = "torch" in sys.modules and sys.modules["torch"].cuda.is_initialized()
    with open(os.path.join(d, f"{name}.txt"), "w") as f:
        f.write(f"P={P} {took:.1f} s ({how}) env={env_extra} parent_gpu_context={ctx}\n" +
                "\n".join(f"--- rank {r}\n{outs[r]}" for r in range(P)))


@pytest.mark.parametrize("mode", ["push", "pull"])
@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_ipc_collectives_match_oracle(P, mode, tmp_path):
    """push: each rank writes block j of its send into rank j's region, kernels read local HBM;
    pull: each rank stages its own send, kernels read the peers' regions."""
    cases = cases_for(P)
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_MODE": mode})
    _check(P, cases, tmp_path)


@pytest.mark.parametrize("alloc", ["coarse", "uncached"])
def test_ipc_staging_alloc_classes(alloc, tmp_path):
    """The staging region is fine-grained by default; MPJX_IPC_STAGE_ALLOC selects coarse-grained
    (hipMalloc) or uncached memory instead, with the same results."""
    P = 4
    cases = [c for c in cases_for(P) if c["id"] in ("ar_sum_f64", "ar_reuse", "rs_ragged", "scan_sum_f64", "ar_big")]
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_MODE": "push", "MPJX_IPC_STAGE_ALLOC": alloc})
    _check(P, cases, tmp_path)


def _check(P, cases, tmp_path):
    for case in cases:
        for rep in range(case.get("reps", 1)):
            exp = expected(case, P, rep)
            for r in range(P):
                if case["kind"] == "reduce" and r != case["root"] and not case.get("flags", 0) & O.FLAG_FAITHFUL:
                    continue  # recvbuf is significant at the root only (every rank's under FAITHFUL)
                got = np.load(tmp_path / f"{case['id']}_r{r}_p{rep}.npy")
                e = exp[r]
                m = case["recvcounts"][r] if case["kind"] == "reduce_scatter" else case["n"]
                assert same_bits(case["type"], case["op"], got, e[:m]), \
                    f"{case['id']} rank {r} pass {rep} P={P}: {_diagnose(case, P, rep, r, got, m)}"


def _diagnose(case, P, rep, r, got, m):
    """On a mismatch: is the result the oracle's with one rank's input replaced by another rank's
    (a block read from the wrong rank's memory)? Run only when a check has failed."""
    t, op = case["type"], case["op"]
    rc = case.get("recvcounts")
    total = sum(rc) if rc is not None else case["n"]
    sends = [case_input(case, total, q, rep) for q in range(P)]
    for j in range(P):
        for q in range(P):
            if q == j:
                continue
            alt = list(sends)
            alt[j] = sends[q]
            try:
                e = _expected_from(case, alt, P)
            except Exception:  # noqa: BLE001
                return "no diagnosis"
            if same_bits(t, op, got, e[r][:m]):
                return f"equals the oracle with rank {j}'s input replaced by rank {q}'s"
    bad = int(np.count_nonzero(got.view(np.uint8) != expected(case, P, rep)[r][:m].view(np.uint8)))
    return f"{bad} bytes differ; not a one-rank substitution"


def _expected_from(case, sends, P):
    t, op, flags, k = case["type"], case["op"], case.get("flags", 0), case["kind"]
    if k == "allreduce":
        return O.allreduce(sends, case["n"], t, op, flags=flags)
    if k == "reduce":
        return O.reduce(sends, case["n"], t, op, case["root"], flags=flags)
    if k == "scan":
        return O.scan(sends, case["n"], t, op, flags=flags)
    if k == "bcast":
        return [sends[case["root"]]] * P
    return O.reduce_scatter(sends, list(case["recvcounts"]), t, op, flags=flags)[0]


@pytest.mark.parametrize("host,sync", [("pageable", "host"), ("pinned", "host"), ("pageable", "device-shared"),
                                       ("pinned", "device-shared")])
def test_ipc_host_buffers(host, sync, tmp_path):
    """Rank processes passing HOST arrays (niodev ranks' Java heap arrays through the JNI shim's
    mpjx_*_host calls, north_star's host-to-host path) on the IPC engine: 1 MiB host chunks, so the
    larger cases run the chunk pipeline (H2D / collective / D2H overlapped, one IPC collective per chunk,
    enqueued without a host barrier under device sync) and the smaller ones one staged call. Pageable
    arrays and page-locked ones (copied back without the drain thread); every result bit-exact."""
    P = 4
    cases = [dict(c, host=host) for c in cases_for(P) if c["kind"] != "bcast" and "env" not in c]
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_MODE": "push", "MPJX_IPC_SYNC": sync,
                                          "MPJX_HOST_CHUNK_MIB": "1"})
    _check(P, cases, tmp_path)


@pytest.mark.parametrize("mode", ["push", "pull"])
@pytest.mark.parametrize("P", [3])
def test_ipc_windows(P, mode, tmp_path):
    """A 1 MiB staging region: vectors longer than it run as consecutive windows (Allreduce, Reduce,
    Scan; Reduce_scatter windows over the whole vector with per-window recvcounts) and exchange()
    moves blocks in rounds — results identical to the unwindowed oracle."""
    cases = cases_for(P)
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_STAGE_MIB": "1", "MPJX_IPC_MODE": mode})
    _check(P, cases, tmp_path)


@pytest.mark.parametrize("mode", ["push", "pull"])
@pytest.mark.parametrize("P", [2, 4, 8])
def test_ipc_device_sync(P, mode, tmp_path):
    """MPJX_IPC_SYNC=device-shared (device sync although every rank sits on this one GPU; plain
    "device" falls back to host sync when ranks share a GPU): the ranks order each direct call through sequence flags their kernels
    store into each other's staging regions (no host barrier, no stream synchronisation inside the
    call) — same results as the host-synchronised engine, every case of the list."""
    cases = cases_for(P)
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_MODE": mode, "MPJX_IPC_SYNC": "device-shared"})
    _check(P, cases, tmp_path)


@pytest.mark.parametrize("fused", ["fence", "share", "0"])
def test_ipc_device_sync_unfused_paths(fused, tmp_path):
    """The device-synchronised engine with its launches unfused, for comparison runs (tools/latency): the
    default stores the fence flag from the combine kernel's tail and fuses the wait into the copy-out
    launch (calls <= 2 MiB, MPJX_IPC_FUSE_KIB); MPJX_IPC_FUSED=fence stores the flag in the copy-out launch instead, =share
    keeps round 3's separate fence flag kernel, =0 separates the share() copies and flags too. Same results
    as the oracle every way."""
    P = 4
    cases = cases_for(P)
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_MODE": "push", "MPJX_IPC_SYNC": "device-shared",
                                          "MPJX_IPC_FUSED": fused})
    _check(P, cases, tmp_path)


@pytest.mark.parametrize("limit_kib", [None, 32768])
def test_ipc_device_sync_fuse_limits(limit_kib, tmp_path):
    """P = 8 rank processes on this one GPU, device sync, at the fused forms' size limit and one element
    past it: the tail signal is armed for calls of at most MPJX_IPC_FUSE_KIB (2 MiB by
    default; 32 MiB, its cap, in the second run) and the copy-out launch waits for the peers' flags in
    every block. Eight ranks whose fused launches spin while the last rank's combine kernel — which
    stores the flag they wait on — still needs CU slots: the copy-out grid is bounded (64 blocks per
    rank) so the call completes at the cap too, bit-exact, and well within the wait limit."""
    P = 8
    lim = (limit_kib or 2048) << 10
    cases = [dict(id="ar_fuse_exact", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=lim // 8, seed=61),
             dict(id="ar_fuse_plus1", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=lim // 8 + 1, seed=62),
             dict(id="scan_fuse_exact", kind="scan", op=O.MAX, type=O.FLOAT, n=lim // 4, seed=63),
             dict(id="scan_fuse_plus1", kind="scan", op=O.MAX, type=O.FLOAT, n=lim // 4 + 1, seed=64),
             dict(id="rs_fuse_exact", kind="reduce_scatter", op=O.BXOR, type=O.INT, recvcounts=[lim // 4 // P] * P,
                  seed=65)]
    env = {"MPJX_IPC_MODE": "push", "MPJX_IPC_SYNC": "device-shared", "MPJX_IPC_TIMEOUT_S": "60"}
    if limit_kib:
        env["MPJX_IPC_FUSE_KIB"] = str(limit_kib)
    launch(P, cases, tmp_path, env_extra=env)
    _check(P, cases, tmp_path)


@pytest.mark.parametrize("mode", ["push", "pull"])
def test_ipc_device_sync_windows(mode, tmp_path):
    """Device-synchronised windows interleaved with host-synchronised exchange() rounds (1 MiB
    staging region)."""
    P = 3
    cases = cases_for(P)
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_STAGE_MIB": "1", "MPJX_IPC_MODE": mode,
                                          "MPJX_IPC_SYNC": "device-shared"})
    _check(P, cases, tmp_path)


def test_ipc_device_sync_falls_back_on_a_shared_gpu(tmp_path):
    """MPJX_IPC_SYNC=device with every rank on this GPU: the world notices the shared PCI bus id and
    runs host-synchronised calls, with the same results."""
    P = 4
    cases = [c for c in cases_for(P) if c["id"] in ("ar_sum_f64", "rs_ragged", "scan_sum_f64", "red_root_last")]
    outs = launch(P, cases, tmp_path, env_extra={"MPJX_IPC_SYNC": "device", "MPJX_IPC_DEBUG": "1"})
    _check(P, cases, tmp_path)
    # the fallback fired on every rank (host sync and device sync give the same bits, so the results
    # alone cannot tell)
    for r, o in enumerate(outs):
        assert "share GPU" in o and "host-synchronised calls" in o, f"rank {r}: no fallback line:\n{o[-1500:]}"


def test_ipc_device_sync_failed_rank(tmp_path):
    """Device waits watch the world's failed mark: a rank that leaves the call early makes every
    rank's call fail promptly, not after MPJX_IPC_TIMEOUT_S."""
    import time

    P = 3
    t0 = time.time()
    launch(P, [dict(id="fail", kind="fail", root=1)], tmp_path,
           env_extra={"MPJX_IPC_TIMEOUT_S": "60", "MPJX_IPC_SYNC": "device-shared"}, timeout=90)
    assert time.time() - t0 < 45
    for r in range(P):
        rc, msg = (tmp_path / f"fail_r{r}.txt").read_text().split(" ", 1)
        assert int(rc) < 0, f"rank {r} returned {rc}"


def test_ipc_failed_rank_errors_every_rank(tmp_path):
    """A rank whose call fails (host pointer as sendbuf) marks the world: every rank's call returns
    an error promptly instead of waiting on the rendezvous."""
    P = 3
    launch(P, [dict(id="fail", kind="fail", root=1)], tmp_path, env_extra={"MPJX_IPC_TIMEOUT_S": "60"}, timeout=90)
    for r in range(P):
        rc, msg = (tmp_path / f"fail_r{r}.txt").read_text().split(" ", 1)
        assert int(rc) < 0, f"rank {r} returned {rc}"


def test_ipc_refuses_oversubscribed_gpu(tmp_path):
    """Round 1's one wrong IPC result: rank 0's rs_ragged block held rank 0's own block 0 where rank
    2's belonged (profiles/r01/pytest_gpu_reentry_failure.txt). Cause: with 8+ processes
    on one MI355X, a kernel can be served the stale translation of a 2 MiB page its process freed and
    re-allocated at the same virtual address — rank 2's push read its fresh send buffer through the
    old page, which by then held rank 0's send (tools/va_alias_probe.cpp reproduces it without
    libmpjx, at 8 processes and at 4 beside a fifth). A world with two rank processes on one GPU is
    therefore refused on every rank unless the caller opts in (MPJX_IPC_OVERSUBSCRIBE=1: no rank
    frees device memory meanwhile)."""
    P = 2
    launch(P, [dict(id="init", kind="init_refused")], tmp_path, env_extra={"MPJX_IPC_OVERSUBSCRIBE": "0"})
    for r in range(P):
        rc, msg = (tmp_path / f"init_r{r}.txt").read_text().split(" ", 1)
        assert int(rc) < 0, f"rank {r}: a 2-process world on one GPU formed"
        assert "share one GPU" in msg and "MPJX_IPC_OVERSUBSCRIBE" in msg, msg


def test_ipc_refuses_mixed_modes(tmp_path):
    """MPJX_IPC_MODE is read once, at init, and must agree: a pushing rank reads the slots its peers
    push into, a pulling rank overwrites them — a mixed world would be silently wrong, so it is refused."""
    P = 2
    uid = os.urandom(128).hex()
    cj = tmp_path / "cases.json"
    cj.write_text(json.dumps([dict(id="init", kind="init_refused")]))
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "ipc_worker.py"), str(r), str(P), uid,
                               str(cj), str(tmp_path)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                              env=dict(os.environ, MPJX_IPC_MODE="push" if r == 0 else "pull"))
             for r in range(P)]
    try:
        for p in procs:
            p.communicate(timeout=120)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r in range(P):
        rc, msg = (tmp_path / f"init_r{r}.txt").read_text().split(" ", 1)
        assert int(rc) < 0 and "MPJX_IPC_MODE" in msg, f"rank {r}: {rc} {msg}"


@pytest.mark.parametrize("mode", ["push", "pull"])
def test_config0_allreduce_sum_double_1mib_4_processes(mode, tmp_path):
    """configs[0] at its own shape over 4 rank PROCESSES (the HIP-IPC direct engine, the multi-process
    deployment's code path on one GPU): Allreduce SUM double 1 MiB, SURVEY §8d C1 streams, three calls
    in the same world, bit-exact against the oracle."""
    P = 4
    cases = [dict(id="c0", kind="allreduce", op=O.SUM, type=O.DOUBLE, n=(1 << 20) // 8, synth=1, reps=3)]
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_MODE": mode})
    _check(P, cases, tmp_path)


@pytest.mark.parametrize("P", [4, 5])
def test_ipc_split_forms_ipc_subworlds(P, tmp_path):
    """Intracomm.Split on a world of rank PROCESSES (mpi.InitIPC) forms each sub-communicator as an
    IPC world of its members (the leader's id gathered to every rank), not an in-process multicore
    world: colors rank % 2, key -rank, then an Allreduce on each sub-world."""
    case = dict(id="split", kind="split", colors=2, op=O.SUM, type=O.DOUBLE, n=20011, seed=41)
    launch(P, [case], tmp_path)
    for color in range(2):
        members = sorted([r for r in range(P) if r % 2 == color], key=lambda r: -r)
        sends = [case_input(case, case["n"], r, 0) for r in members]
        exp = O.allreduce(sends, case["n"], O.DOUBLE, O.SUM)
        for i, r in enumerate(members):
            got = np.load(tmp_path / f"split_r{r}.npy")
            assert same_bits(O.DOUBLE, O.SUM, got, exp[i]), (color, r)
            assert (tmp_path / f"split_r{r}.txt").read_text() == f"{i} {len(members)}"


@pytest.mark.parametrize("mode,host", [("push", None), ("pull", None), ("push", "pageable")])
@pytest.mark.parametrize("P", [3, 4])
def test_ipc_faithful_buffers(P, mode, host, tmp_path):
    """MPJX_FLAG_FAITHFUL over the HIP-IPC engine: every rank's Reduce recvbuf holds its MST sub-tree
    partial (through the staging out-regions and fence's copy-out), and the BKT ring's sendbuf overwrite
    lands in every rank's send buffer, both against the oracle's faithful mode — with device buffers,
    and with host arrays (the *_host calls copy the rewritten staged sendbuf back to the caller's)."""
    rc = [700 + 37 * r for r in range(P)]
    cases = [dict(id="fred_sum_f64", kind="reduce", op=O.SUM, type=O.DOUBLE, n=5003, root=P - 1, seed=51,
                  flags=O.FLAG_FAITHFUL),
             dict(id="fred_max_i32_root0", kind="reduce", op=O.MAX, type=O.INT, n=4099, root=0, seed=52,
                  flags=O.FLAG_FAITHFUL),
             dict(id="frs_sum_i32", kind="reduce_scatter", op=O.SUM, type=O.INT, recvcounts=rc, seed=53,
                  flags=O.FLAG_FAITHFUL),
             dict(id="frs_prod_f64", kind="reduce_scatter", op=O.PROD, type=O.DOUBLE, recvcounts=rc, seed=54,
                  flags=O.FLAG_FAITHFUL)]
    cases = [dict(c, host=host) for c in cases]
    launch(P, cases, tmp_path, env_extra={"MPJX_IPC_MODE": mode})
    _check(P, cases, tmp_path)
    for case in cases[2:]:
        total = sum(case["recvcounts"])
        sends = [case_input(case, total, r, 0) for r in range(P)]
        _, exp_send = O.reduce_scatter(sends, case["recvcounts"], case["type"], case["op"], flags=O.FLAG_FAITHFUL)
        for r in range(P):
            got = np.load(tmp_path / f"{case['id']}_send_r{r}_p0.npy")
            assert same_bits(case["type"], case["op"], got, exp_send[r]), (case["id"], r)
