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
