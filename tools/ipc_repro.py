"""Repeat tests/test_gpu_ipc.py's P-rank case list (rank PROCESSES on one GPU) R times in one
process and report every mismatching result with the rank whose contribution it matches instead.
    python tools/ipc_repro.py P MODE R [hold]"""
import os
import sys
import tempfile
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

from test_gpu_ipc import cases_for, expected, launch  # noqa: E402
from util import same_bits  # noqa: E402

P, mode, R = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
if len(sys.argv) > 4 and sys.argv[4] == "hold":  # this process holds a GPU context too (as pytest's does)
    import torch

    held = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
bad = 0
for it in range(R):
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        cases = cases_for(P)
        launch(P, cases, d, env_extra={"MPJX_IPC_MODE": mode})
        for case in cases:
            for rep in range(case.get("reps", 1)):
                exp = expected(case, P, rep)
                for r in range(P):
                    if case["kind"] == "reduce" and r != case["root"]:
                        continue
                    got = np.load(d / f"{case['id']}_r{r}_p{rep}.npy")
                    m = case["recvcounts"][r] if case["kind"] == "reduce_scatter" else case["n"]
                    if not same_bits(case["type"], case["op"], got, exp[r][:m]):
                        bad += 1
                        nbad = int(np.count_nonzero(got.view(np.uint8) != exp[r][:m].view(np.uint8)))
                        print(f"iter {it}: {case['id']} rank {r} pass {rep}: {nbad} bytes differ", flush=True)
    print(f"iter {it} done, {bad} bad results so far", flush=True)
print(f"P={P} mode={mode}: {bad} bad results in {R} runs")
sys.exit(1 if bad else 0)
