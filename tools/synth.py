"""SURVEY §8(d) synthetic inputs: splitmix64 counter streams, seed = 0x4D504A00 + 1000*config + rank.

Element i of a stream is a pure function of (seed, i): z = splitmix64_mix(seed + (i+1)*GOLDEN). That
makes the full-size bench inputs generable on the GPU (torch int64 ops, wrap-around arithmetic) and
any sampled subset of them recomputable on the host (numpy uint64) — so bench.py can check its own
full-size results bit-exactly on a sample of indices without copying 256 MiB back.

Doubles: (z >> 11) * 2^-53 in [0, 1), mapped to [lo, hi) as lo + (hi - lo) * u (exact for [-1, 1)).
"""
import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB


def seed(cfg, rank):
    return 0x4D504A00 + 1000 * cfg + rank


def _s64(x):
    """uint64 constant -> the int64 with the same bits (torch has no uint64 arithmetic)."""
    return x - (1 << 64) if x >= 1 << 63 else x


def _srl(x, k):
    """logical right shift of an int64 tensor"""
    import torch

    return torch.bitwise_and(torch.bitwise_right_shift(x, k), (1 << (64 - k)) - 1)


def bits_torch(n, s, device):
    import torch

    z = torch.arange(1, n + 1, dtype=torch.int64, device=device)
    z.mul_(_s64(GOLDEN)).add_(_s64(s % (1 << 64)))
    z = torch.bitwise_xor(z, _srl(z, 30)).mul_(_s64(M1))
    z = torch.bitwise_xor(z, _srl(z, 27)).mul_(_s64(M2))
    return torch.bitwise_xor(z, _srl(z, 31))


def bits_np(idx, s):
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (idx + np.uint64(1)) * np.uint64(GOLDEN) + np.uint64(s % (1 << 64))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
        return z ^ (z >> np.uint64(31))


def uniform_torch(n, s, device, lo=-1.0, hi=1.0):
    import torch

    u = _srl(bits_torch(n, s, device), 11).to(torch.float64).mul_(2.0 ** -53)
    return u.mul_(hi - lo).add_(lo)


def uniform_np(idx, s, lo=-1.0, hi=1.0):
    u = (bits_np(idx, s) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    return u * (hi - lo) + lo
