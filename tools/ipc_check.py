"""Debug helper: check the outputs tools/ipc_debug.sh left against the oracle (test infrastructure)."""
import json
import sys

import numpy as np

sys.path[:0] = ["tests", "oracle"]
import test_gpu_ipc as T  # noqa: E402
from util import same_bits  # noqa: E402

P = int(sys.argv[1])
d = sys.argv[2]
for case in json.load(open(f"{d}/cases.json")):
    for rep in range(case.get("reps", 1)):
        exp = T.expected(case, P, rep)
        for r in range(P):
            if case["kind"] == "reduce" and r != case["root"]:
                continue
            try:
                got = np.load(f"{d}/{case['id']}_r{r}_p{rep}.npy")
            except FileNotFoundError:
                print(case["id"], "rank", r, "rep", rep, "MISSING")
                continue
            m = case["recvcounts"][r] if case["kind"] == "reduce_scatter" else case["n"]
            if same_bits(case["type"], case["op"], got, exp[r][:m]):
                print(case["id"], "rank", r, "rep", rep, "ok")
                continue
            g = got.view(np.uint8).reshape(m, -1)
            e = exp[r][:m].view(np.uint8).reshape(m, -1)
            bad = np.nonzero((g != e).any(1))[0]
            print(case["id"], "rank", r, "rep", rep, "BAD", len(bad), "of", m, "first", bad[:5], "last", bad[-3:])
