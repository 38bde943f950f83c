"""CPU, this container only: cross-check the oracle's MPI-semantics mode against MPICH 3.3
(/opt/conda) for every order-independent (op, type) pair — integer SUM/PROD/MAX/MIN, bitwise and
logical ops — through Allreduce, Reduce (root P/2), Reduce_scatter and Scan at P = 2, 3, 4. MPICH is
an independent MPI implementation (and the arithmetic behind the reference's native device), so
this pins the oracle's (op, type) rows beyond the INT SUM/PROD the reference's own KATs cover."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle as O

MPIEXEC = "/opt/conda/bin/mpiexec"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "build", "mpich_xcheck")
TYPES = {"BYTE": O.BYTE, "CHAR": O.CHAR, "SHORT": O.SHORT, "INT": O.INT, "LONG": O.LONG, "BOOLEAN": O.BOOLEAN}
OPS = {v: k for k, v in O.OP_NAMES.items()}

pytestmark = pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="MPICH not present")


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/mpich_xcheck"],
                           capture_output=True, text=True)
        if r.returncode != 0:
            pytest.skip("cannot build the MPICH cross-check: " + r.stderr[-300:])
    return EXE


@pytest.mark.parametrize("P", [2, 3, 4])
def test_oracle_matches_mpich(exe, tmp_path, P):
    n = 1020
    r = subprocess.run([MPIEXEC, "-n", str(P), exe, str(tmp_path), str(n)], capture_output=True, text=True,
                       timeout=300, cwd=str(tmp_path))
    if r.returncode != 0:
        pytest.skip("mpiexec could not run here: " + (r.stderr or r.stdout)[-300:])
    cases = sorted({f.split("_", 2)[2][:-4] for f in os.listdir(tmp_path) if f.startswith("in_")})
    assert len(cases) == 38  # 7 integer ops x 5 types + 3 logical ops x boolean
    for case in cases:
        opname, tname = case.split("_")
        op, t = OPS[opname], TYPES[tname]
        dt = O.NP_DTYPE[t]
        ld = lambda what, rank: np.fromfile(tmp_path / f"{what}_{rank}_{case}.bin", dtype=dt)  # noqa: E731
        xs = [ld("in", k) for k in range(P)]
        for k, got in enumerate(O.allreduce(xs, n, t, op)):
            assert np.array_equal(got, ld("allreduce", k)), ("allreduce", case, k)
        assert np.array_equal(O.reduce(xs, n, t, op, P // 2)[P // 2], ld("reduce", P // 2)), ("reduce", case)
        for k, got in enumerate(O.scan(xs, n, t, op)):
            assert np.array_equal(got, ld("scan", k)), ("scan", case, k)
        rs, _ = O.reduce_scatter(xs, [n // P] * P, t, op)
        for k in range(P):
            assert np.array_equal(rs[k], ld("rs", k)), ("reduce_scatter", case, k)
