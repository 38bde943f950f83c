"""bench.py's own checkers, on the CPU: the splitmix64 input streams (GPU/torch twin == host/numpy
twin, bit for bit) and the sampled-parity MST grouping (== the oracle's Allreduce order)."""
import os
import sys

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)


def test_splitmix_twins_agree():
    import synth

    assert int(synth.bits_np([0], 0)[0]) == 0xE220A8397B1DCDAF  # splitmix64 from state 0
    for cfg, rank in [(2, 0), (2, 1), (3, 7)]:
        s = synth.seed(cfg, rank)
        t = synth.uniform_torch(50000, s, "cpu").numpy()
        h = synth.uniform_np(np.arange(50000), s)
        assert np.array_equal(t.view(np.uint64), h.view(np.uint64))
        assert t.min() >= -1.0 and t.max() < 1.0
        idx = np.array([0, 17, 49999])
        assert np.array_equal(synth.uniform_np(idx, s), h[idx])


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8])
def test_bench_mst_grouping_matches_oracle(P):
    import bench
    import synth

    n = 4096
    sends = [synth.uniform_np(np.arange(n), synth.seed(3, r)) for r in range(P)]
    exp = O.allreduce(sends, n, O.DOUBLE, O.SUM)[0]
    got = bench.mst_sum(sends, 0, P - 1, 0)
    assert np.array_equal(np.asarray(got).view(np.uint64), exp.view(np.uint64))


def test_checksum_fingerprint():
    """bench.checksum: (XOR, wrapping sum) of 64-bit words — equal for equal bits, changed by one bit,
    the byte tail zero-padded into a last word."""
    import bench

    a = np.arange(1001, dtype=np.float64)
    c0 = bench.checksum(a)
    assert bench.checksum(a.copy()) == c0
    b = a.copy()
    b.view(np.uint64)[500] ^= np.uint64(1)
    assert bench.checksum(b) != c0
    w = int.from_bytes(bytes([1, 2, 3, 0, 0, 0, 0, 0]), "little")
    assert bench.checksum(np.array([1, 2, 3], np.uint8)) == (w, w)
    assert bench.checksum(np.array([2 ** 63, 2 ** 63], dtype=np.uint64)) == (0, 0)  # xor cancels, sum wraps


def _preflight_worker(rank, P, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        q.put((rank, bench.ipc_preflight(dist, rank, P, 0)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_ipc_preflight_verdict_without_gpu():
    """bench.py's child-process check of the IPC engine at world size 2 over gloo: without a GPU the
    children fail, and every rank gets the same verdict (skip the IPC engines) instead of an error."""
    import socket

    import torch
    import torch.multiprocessing as mp

    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present: tests/test_gpu_cpp.py covers the passing case")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_preflight_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert isinstance(res[r], dict), res[r]
        assert res[r]["ok"] is False and res[r]["msg"], res[r]


def test_c4_inputs_and_mismatch_counter():
    """configs[3] inputs (bench.c4_inputs, on the CPU device here): int32 = the low 32 bits of the 64-bit
    stream (a bit view), BAND words with about 7/8 of their bits set; bench._mismatch counts and
    locates differing elements bit for bit (NaN payloads and -0.0 included)."""
    import torch

    import bench
    import synth

    n = 1 << 16
    band, bxor = bench.c4_inputs(n, 3, torch.device("cpu"))
    s = synth.seed(4, 3)
    low = (synth.bits_np(np.arange(n), s + 0x300) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
    assert np.array_equal(bxor.numpy(), low)
    ones = np.unpackbits(band.numpy().view(np.uint8)).mean()
    assert 0.86 < ones < 0.89, ones
    a = torch.tensor([1.0, -0.0, float("nan"), 3.0], dtype=torch.float32)
    b = torch.tensor([1.0, 0.0, float("nan"), 4.0], dtype=torch.float32)
    assert bench._mismatch(a, b) == (2, 1)
    assert bench._mismatch(a, a.clone()) == (0, None)


def test_plan_engines_after_preflights():
    """bench.plan_engines: an engine is timed only if its own child-process preflight passed; every RCCL
    variant rides on the plain "rccl" world; the IPC and RCCL verdicts are independent."""
    import bench

    allx = ["rccl", "ipc", "ipc_pull", "ipc_dsync", "rccl_pipe64", "rccl_pipe32"]
    ok = {"ok": True, "msg": "ok"}
    bad = {"ok": False, "msg": "rank 1: forced failure"}
    ipc_ok = {"ok": True, "dsync_ok": True, "msg": "ipc preflight ok"}
    names, var, skip = bench.plan_engines(allx, ipc_ok, {v: ok for v in bench.RCCL_VARIANTS})
    assert names == allx and var == ["rccl_p2p", "rccl_skew"] and skip == {}
    # one pipeline fails: only it goes
    rpf = dict({v: ok for v in bench.RCCL_VARIANTS}, rccl_pipe32=bad)
    names, var, skip = bench.plan_engines(allx, ipc_ok, rpf)
    assert names == [e for e in allx if e != "rccl_pipe32"] and set(skip) == {"rccl_pipe32"}
    # the base RCCL world fails: every RCCL engine and variant goes, the IPC engines are still timed
    rpf = dict({v: ok for v in bench.RCCL_VARIANTS}, rccl=bad)
    names, var, skip = bench.plan_engines(allx, ipc_ok, rpf)
    assert names == ["ipc", "ipc_pull", "ipc_dsync"] and var == []
    assert set(skip) == {"rccl", "rccl_pipe64", "rccl_pipe32", "rccl_p2p", "rccl_skew"}
    assert "forced failure" in skip["rccl_pipe64"]
    # IPC fails, device sync alone fails
    names, _, skip = bench.plan_engines(allx, {"ok": False, "dsync_ok": False, "msg": "x"}, {"rccl": ok})
    assert names == ["rccl", "rccl_pipe64", "rccl_pipe32"] and {"ipc", "ipc_pull", "ipc_dsync"} <= set(skip)
    names, _, skip = bench.plan_engines(allx, {"ok": True, "dsync_ok": False, "msg": "x"}, None)
    assert "ipc_dsync" not in names and "ipc" in names and set(skip) == {"ipc_dsync"}
    # no preflight run (--no-preflight): nothing skipped
    assert bench.plan_engines(allx, None, None) == (allx, ["rccl_p2p", "rccl_skew"], {})
    # RCCL's own ncclAllReduce (rccl_native) is never an engine: passed in, it is dropped;
    # at world <= 2 it is a comparison VARIANT riding on the plain world and its own preflight
    alln = allx + ["rccl_native"]
    names, var, skip = bench.plan_engines(alln, ipc_ok, {v: ok for v in bench.RCCL_VARIANTS}, world=2)
    assert names == allx and var == ["rccl_p2p", "rccl_skew", "rccl_native"] and "rccl_native" not in skip
    names, var, skip = bench.plan_engines(alln, ipc_ok, {v: ok for v in bench.RCCL_VARIANTS}, world=4)
    assert names == allx and "rccl_native" not in var and "not a libmpjx HIP-combine engine" in skip["rccl_native"]
    names, var, skip = bench.plan_engines(allx, ipc_ok, {v: ok for v in bench.RCCL_VARIANTS}, world=8)
    assert var == ["rccl_p2p", "rccl_skew"]  # bit-exact only at P <= 2: not timed at 8
    names, var, skip = bench.plan_engines(allx, ipc_ok, dict({v: ok for v in bench.RCCL_VARIANTS}, rccl_native=bad),
                                          world=1)
    assert names == allx and "rccl_native" not in var and set(skip) == {"rccl_native"}
    names, var, skip = bench.plan_engines(allx, ipc_ok, dict({v: ok for v in bench.RCCL_VARIANTS}, rccl=bad), world=2)
    assert "rccl_native" not in var and "rccl_native" in skip


def test_reported_engine_is_always_a_hip_combine_engine():
    """bench.pick_reported: the line's engine is the fastest bit-exact one among libmpjx's HIP-combine
    engines — never rccl_native (RCCL's own reduction kernel, SURVEY 8(e): a ceiling reference), even
    when it is the fastest and bit-exact; the CLI does not offer it as an engine."""
    import bench

    assert "rccl_native" not in bench.HEADLINE_ENGINES
    eng = {"rccl": {"t": 2.0, "mismatches": 0, "full_checksum_match": True},
           "ipc": {"t": 1.5, "mismatches": 0, "full_checksum_match": True},
           "rccl_native": {"t": 0.5, "mismatches": 0, "full_checksum_match": True},
           "ipc_pull": {"t": 1.0, "mismatches": 3, "full_checksum_match": False}}
    names = list(eng)
    assert bench.pick_reported(names, eng) == "ipc"
    assert bench.pick_reported(["rccl_native"], eng) is None
    del eng["ipc"]
    assert bench.pick_reported(list(eng), eng) == "rccl"
    # nothing bit-exact: the first HIP-combine engine that ran (its parity fields flag it)
    bad = {"rccl_native": dict(eng["rccl_native"]), "ipc_pull": dict(eng["ipc_pull"]),
           "rccl": {"t": 3.0, "mismatches": 1, "full_checksum_match": False}}
    assert bench.pick_reported(["rccl_native", "ipc_pull", "rccl"], bad) == "ipc_pull"
    assert bench.pick_reported(["rccl"], {"rccl": {"error": "x"}}) is None
    with pytest.raises(SystemExit):
        bench.parse(["--engine", "rccl_native"])


FAKE_CHILD = r'''
import os, sys, time
rank, P, dev, variant, uid = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
if rank == 0:
    open(uid + ".tmp", "wb").write(os.urandom(128)); os.rename(uid + ".tmp", uid)
else:
    t0 = time.time()
    while not os.path.exists(uid):
        if time.time() - t0 > 20: sys.exit("uid file never published")
        time.sleep(0.01)
if variant == os.environ.get("FAKE_FAIL_VARIANT") and rank == int(os.environ.get("FAKE_FAIL_RANK", "-1")):
    sys.exit("element 7 = 1.5, MST(0) = 2.5")
if variant == os.environ.get("FAKE_HANG_VARIANT"):
    time.sleep(600)
print("rccl preflight ok: %s P=%d" % (variant, P))
'''


def _rccl_preflight_worker(rank, P, port, exe, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MPJX_RCCL_PREFLIGHT_EXE=exe,
                      MPJX_BENCH_PREFLIGHT_TIMEOUT_S="8", FAKE_FAIL_VARIANT="rccl_pipe32", FAKE_FAIL_RANK="1",
                      FAKE_HANG_VARIANT="rccl_p2p")
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        q.put((rank, bench.rccl_preflight(dist, rank, P, 0, ["rccl", "rccl_pipe32", "rccl_p2p", "rccl_skew"])))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P", [2, 8])
def test_rccl_preflight_protocol_gloo(P, tmp_path):
    """bench.rccl_preflight at world size 2 and 8 (the SCALE run's) over gloo with a stand-in child
    (MPJX_RCCL_PREFLIGHT_EXE): the unique-id file handshake, one world per variant, a failure on ONE rank
    reported on every rank with that rank's message, a hanging child killed at the time limit, and the
    variants after it still run."""
    import socket
    import stat

    import torch.multiprocessing as mp

    exe = tmp_path / "fake_child"
    exe.write_text("#!" + sys.executable + "\n" + FAKE_CHILD)
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rccl_preflight_worker, args=(r, P, port, str(exe), q)) for r in range(P)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(P))
    for p in procs:
        p.join(timeout=60)
    for r in range(P):
        v = res[r]
        assert isinstance(v, dict), v
        assert v["rccl"]["ok"] and "rccl preflight ok" in v["rccl"]["msg"], v
        assert not v["rccl_pipe32"]["ok"] and v["rccl_pipe32"]["failed_ranks"] == 1, v
        assert "rank 1" in v["rccl_pipe32"]["msg"] and "MST(0)" in v["rccl_pipe32"]["msg"], v
        assert not v["rccl_p2p"]["ok"] and "no verdict" in v["rccl_p2p"]["msg"], v
        assert v["rccl_skew"]["ok"], v
    assert not list(tmp_path.glob("mpjx_rccl_preflight_*"))


def test_rccl_preflight_child_forced_failure():
    """tools/rccl_preflight with MPJX_PREFLIGHT_FAIL names the variant: it fails before touching the GPU
    (exit 7), which is how a GPU-box rehearsal shows the RCCL engines skipped and the IPC engines kept."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "rccl_preflight")
    if not os.path.exists(exe):
        pytest.skip("tools/rccl_preflight not built")
    p = subprocess.run([exe, "0", "1", "0", "rccl_pipe32", "/tmp/mpjx_unused_uid"], capture_output=True, text=True,
                       env=dict(os.environ, MPJX_PREFLIGHT_FAIL="rccl,rccl_pipe32"), timeout=60)
    assert p.returncode == 7 and "forced failure" in p.stderr, (p.returncode, p.stderr)
    p = subprocess.run([exe, "0", "1", "0", "bogus", "/tmp/mpjx_unused_uid"], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode != 0


def test_checksum_torch_and_device_expectation_match_host():
    """bench.checksum_torch == bench.checksum bit for bit (XOR by halving, wrapping int64 sum), and
    expected_checksum_device (torch streams + torch adds in the MST grouping, run here on the CPU
    device) == the host recomputation the N > 1 line used before (numpy streams + numpy adds)."""
    import torch

    import bench
    import synth

    rng = np.random.default_rng(3)
    for n in (1, 2, 7, 1000, 4099):
        w = rng.integers(0, 2 ** 63, n, dtype=np.uint64) * np.uint64(3)  # top bits set too
        assert bench.checksum_torch(torch.from_numpy(w.view(np.int64))) == bench.checksum(w), n
    for world, n in ((1, 5000), (3, 4099), (8, 2048)):
        host = bench.checksum(bench.mst_sum([synth.uniform_np(np.arange(n, dtype=np.uint64), synth.seed(3, r))
                                             for r in range(world)], 0, world - 1, 0))
        assert bench.expected_checksum_device(n, world, torch.device("cpu")) == host, (world, n)
