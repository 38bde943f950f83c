"""Shared test helpers: seeded inputs with edge values, bit-exact comparison."""
import numpy as np

import oracle as O

FLOATS = (O.FLOAT, O.DOUBLE)


def splitmix_seed(cfg, rank):
    """Seed scheme of BASELINE.md: 0x4D504A00 + 1000*config + rank."""
    return 0x4D504A00 + 1000 * cfg + rank


def make_input(type_, n, seed, specials=True, op=None):
    if type_ in O.PAIR_BASE:
        return make_pair_input(type_, n, seed, specials)
    rng = np.random.default_rng(seed)
    dt = O.NP_DTYPE[type_]
    if type_ == O.BOOLEAN:
        return rng.integers(0, 2, n, dtype=np.uint8)
    if type_ in FLOATS:
        x = rng.uniform(-1.0, 1.0, n).astype(dt)
        if op == O.PROD:  # keep products away from 0/inf for long folds
            x = (np.sign(x) * (0.5 + np.abs(x))).astype(dt)
        if specials and n >= 16:
            fin = np.finfo(dt)
            sp = np.array([np.nan, 0.0, -0.0, np.inf, -np.inf, fin.tiny / 4, -fin.tiny / 8, fin.max,
                           -fin.max, fin.tiny, 1.0, -1.0], dtype=dt)
            idx = rng.choice(n, size=min(n // 4, 64), replace=False)
            x[idx] = sp[rng.integers(0, sp.size, idx.size)]
        return x
    info = np.iinfo(dt)
    x = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    if specials and n >= 8:
        x[:4] = [info.min, info.max, 0, -1 if info.min < 0 else 1]
    return x


def same_bits(type_, op, got, exp):
    """Bit-exact equality; for float SUM/PROD any NaN equals any NaN (payload of a NaN produced by
    two NaN operands is not specified by Java or IEEE)."""
    got = np.asarray(got)
    exp = np.asarray(exp)
    if got.shape != exp.shape:
        return False
    if got.size == 0:
        return True
    if type_ in FLOATS and op in (O.SUM, O.PROD):
        both_nan = np.isnan(got) & np.isnan(exp)
        gb = got.view(np.uint8).reshape(got.size, -1)
        eb = exp.view(np.uint8).reshape(exp.size, -1)
        return bool(np.all((gb == eb).all(axis=1) | both_nan))
    return bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8)))


def make_pair_input(type_, n, seed, specials=True):
    """(value, index) records with few distinct values, so ties (the index rule) are common."""
    rng = np.random.default_rng(seed)
    a = np.zeros(n, O.NP_DTYPE[type_])
    base = O.PAIR_BASE[type_]
    a["v"] = rng.integers(-3, 4, n)
    a["l"] = rng.integers(0, 1000, n)
    if specials and base in FLOATS and n >= 16:
        idx = rng.choice(n, size=min(n // 4, 64), replace=False)
        sp = np.array([np.nan, 0.0, -0.0, np.inf, -np.inf], dtype=O.NP_DTYPE[base])
        a["v"][idx] = sp[rng.integers(0, sp.size, idx.size)]
    return a


def flat(a, type_):
    """Pair records -> interleaved base-type array (what a Java INT2 buffer is)."""
    if type_ in O.PAIR_BASE:
        return a.view(O.NP_DTYPE[O.PAIR_BASE[type_]])
    return a
