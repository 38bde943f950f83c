"""Exercise the IPC rank processes' stall report (tests/watchdog.py, armed by tests/test_gpu_ipc.py's
launch) on the GPU: one P = 8 push world with the report armed at 2.5 s instead of 45 s, so every rank
prints its blocking system call and native + Python stacks mid-run and then finishes normally. Shows the
report is safe inside a running GPU world and what a healthy rank looks like at that moment.

    python tools/stall_report_probe.py OUT_TXT"""
import os
import pathlib
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]

import test_gpu_ipc as T  # noqa: E402

cases = [dict(id=f"ar_big_{i}", kind="allreduce", op=3, type=8, n=(16 << 20) // 8 + 3, seed=10 + i, reps=6)
         for i in range(6)]
outs = T.launch(8, cases, pathlib.Path(tempfile.mkdtemp(prefix="stallprobe_")),
                env_extra={"MPJX_IPC_MODE": "push", "MPJX_TEST_STALL_REPORT_S": "2.5"})
with open(sys.argv[1], "w") as f:
    for r, o in enumerate(outs):
        f.write(f"--- rank {r}\n{o}\n")
reports = sum("=== watchdog:" in o for o in outs)  # a rank may finish before its report does
print(f"ranks: 8, stall reports: {reports}, every rank finished", flush=True)
