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
