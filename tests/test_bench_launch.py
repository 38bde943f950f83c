"""bench.py's launcher and time budget, on the CPU (VERDICT r4 "do this" #1 and #2).

- `python bench.py --gpus N` without a launcher starts the N ranks itself as a child
  `torch.distributed.run` (never exec), before it imports torch or loads HIP, and relays rank 0's line;
- the child's line gets a "launcher" record; a child that dies without a line leaves rank 0's
  checkpoint (or an error line) on stdout, so the driver's N > 1 run never comes back empty or as N = 1;
- Budget.allow is rank 0's decision on every rank (gloo, world size 2).
"""
import json
import os
import signal
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=120):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MPJX_BENCH_LAUNCHED"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=e, timeout=timeout)


def test_dry_launch_shows_the_child_command_with_the_same_arguments():
    p = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])["launcher"]
    cmd = rec["cmd"]
    assert "-m torch.distributed.run" in cmd and "--nnodes=1" in cmd and "--nproc-per-node=2" in cmd
    assert "--master-addr 127.0.0.1" in cmd
    assert cmd.endswith("bench.py --gpus 2 --steps 3 --warmup 1"), cmd
    assert "--dry-launch" not in cmd
    # the parent decided before touching the GPU stack: no torch, no HIP runtime, no device node
    assert rec["parent_before_spawn"] == {"torch_imported": False, "hip_runtime_loaded": False,
                                          "gpu_device_open": False}


def test_wants_launch_rules():
    import bench

    a = bench.parse(["--gpus", "8"])
    assert bench.wants_launch(a, env={})
    assert not bench.wants_launch(a, env={"WORLD_SIZE": "8"})          # under the driver's torchrun
    assert not bench.wants_launch(a, env={"MPJX_BENCH_LAUNCHED": "1"})  # a self-launched rank
    assert not bench.wants_launch(bench.parse(["--gpus", "8", "--no-launch"]), env={})
    assert not bench.wants_launch(bench.parse([]), env={})              # N = 1: this process is the rank
    assert bench.wants_launch(bench.parse(["--launch"]), env={})        # forced (world-1 rehearsal)
    cmd = bench.launcher_command(bench.parse(["--gpus", "4"]), ["--gpus", "4", "--launch", "--budget-s", "60"], 1234)
    assert cmd[1:8] == ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4", "--master-addr",
                        "127.0.0.1", "--master-port=1234"]
    assert cmd[-3:] == ["4", "--budget-s", "60"] and "--launch" not in cmd


def _fake_launch(monkeypatch, capsys, child, args, grace="90"):
    """bench.self_launch with the child replaced by `python -c child`: returns (status, stdout lines)."""
    import bench

    monkeypatch.setattr(bench, "launcher_command", lambda a, argv, port: [sys.executable, "-c", child])
    monkeypatch.setenv("MPJX_BENCH_LAUNCH_GRACE_S", grace)
    old = {s: signal.getsignal(s) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        rc = bench.self_launch(bench.parse(args), args)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc, [x for x in capsys.readouterr().out.splitlines() if x.strip()]


def test_self_launch_relays_rank0_line_with_launcher_record(monkeypatch, capsys):
    child = "import json; print(json.dumps({'metric': 'm', 'value': 1.5, 'n_gpus': 2}), flush=True)"
    rc, out = _fake_launch(monkeypatch, capsys, child, ["--gpus", "2"])
    assert rc == 0 and len(out) == 1, out
    d = json.loads(out[0])
    assert d["value"] == 1.5 and d["n_gpus"] == 2
    assert d["launcher"]["self_launched"] and d["launcher"]["parent_after"]["torch_imported"] in (True, False)


def test_self_launch_prints_checkpoint_when_ranks_are_killed(monkeypatch, capsys):
    """The ranks hang after rank 0 checkpointed: the launcher kills the child's process group at
    --hard-s + grace and prints the checkpoint, flagged cut_short."""
    child = ("import json, os, time\n"
             "p = os.environ['MPJX_BENCH_CHECKPOINT']\n"
             "json.dump({'metric': 'm', 'value': 2.0, 'n_gpus': 2}, open(p, 'w'))\n"
             "time.sleep(120)\n")
    rc, out = _fake_launch(monkeypatch, capsys, child, ["--gpus", "2", "--hard-s", "1"], grace="3")
    assert rc == 0 and len(out) == 1, out
    d = json.loads(out[0])
    assert d["value"] == 2.0 and "killed at the launcher's limit" in d["cut_short"], d


def test_self_launch_line_then_hung_teardown_counts(monkeypatch, capsys):
    """Rank 0 printed its line, then the ranks' teardown hangs: the launcher ends the child after the
    post-line grace and exits 0 with the relayed line (the measurement is complete)."""
    monkeypatch.setenv("MPJX_BENCH_AFTER_LINE_S", "2")
    child = ("import json, time\n"
             "print(json.dumps({'metric': 'm', 'value': 3.0, 'n_gpus': 2}), flush=True)\n"
             "time.sleep(120)\n")
    rc, out = _fake_launch(monkeypatch, capsys, child, ["--gpus", "2"])
    assert rc == 0 and len(out) == 1, out
    assert json.loads(out[0])["value"] == 3.0


def test_self_launch_error_line_when_ranks_fail_silently(monkeypatch, capsys):
    rc, out = _fake_launch(monkeypatch, capsys, "import sys; sys.exit(3)", ["--gpus", "2"])
    assert rc == 3 and len(out) == 1, out
    d = json.loads(out[0])
    assert d["value"] is None and "status 3" in d["error"] and d["n_gpus"] == 2


def test_launcherless_gpus2_without_gpu_ends_with_one_line():
    """The real self-launch end to end on the CPU: two ranks start under the child torchrun, fail at
    their first GPU call (no GPU here), and the parent still prints exactly one JSON line (an error
    line, nonzero status) instead of nothing or an N = 1 line."""
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present: the -m gpu rehearsal covers the passing case")
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-preflight", "--no-variants", "--hard-s", "60"],
             env={"MPJX_BENCH_LAUNCH_GRACE_S": "60"}, timeout=300)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, (p.stdout[-2000:], p.stderr[-2000:])
    d = json.loads(lines[0])
    assert p.returncode != 0 and d["value"] is None and d["n_gpus"] == 2, d
    assert d["launcher"]["parent_before_spawn"]["hip_runtime_loaded"] is False


def _budget_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        # rank 0's clock says 100 s, rank 1's 0 s: rank 0 decides for both
        b = bench.Budget(dist, rank, 150.0, clock=lambda: 100.0 if rank == 0 else 0.0)
        got = [b.allow("engine:x", 0.5), b.allow("variant:y"), b.allow("e2e_host", 0.6)]
        with b.phase("variant:y"):
            pass
        q.put((rank, got, b.skipped, sorted(b.wall)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


def test_budget_is_rank0s_decision_on_every_rank():
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_budget_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (g, sk, w) for r, g, sk, w in (q.get(timeout=180) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        got, sk, wall = res[r]
        assert got == [False, True, False], (r, got)
        assert sk == ["engine:x", "e2e_host"] and wall == ["variant:y"], (r, sk, wall)


HARD_LIMIT_CHILD = r'''
import json, os, sys, threading, time
sys.path.insert(0, sys.argv[1])
import bench
mode = sys.argv[2]
snap = {"raise": lambda note=None: {}["boom"], "ok": lambda note=None: {"metric": "m", "value": 1.0, "cut_short": note}}
if mode == "printed":  # the normal end printed the line; the teardown then stalls past --hard-s
    bench.emit({"metric": "m", "value": 2.0})
fn = snap["raise" if mode == "raising" else "ok"]
t = threading.Timer(0.5, lambda: os._exit(bench.hard_limit_status(0, fn, 0.5, "teardown")))
t.daemon = True
t.start()
time.sleep(30)  # the stalled teardown (mpjx_comm_destroy / destroy_process_group)
print("teardown returned")
'''


@pytest.mark.parametrize("mode,rc_want,value", [("printed", 0, 2.0), ("unprinted", 0, 1.0), ("raising", 1, None)])
def test_hard_limit_after_the_line_and_with_a_failing_snapshot(mode, rc_want, value):
    """the --hard-s timer firing after rank 0 printed its line (a teardown running past the
    limit) exits 0 with that one line, not 'no engine measured' and status 1; a snapshot that raises on
    the timer thread (dicts mutated by the main thread) still ends the process, with status 1 and no
    line; before any line, the snapshot is printed, flagged cut_short."""
    import subprocess

    r = subprocess.run([sys.executable, "-c", HARD_LIMIT_CHILD, ROOT, mode], capture_output=True, text=True,
                       timeout=60)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert r.returncode == rc_want, (r.returncode, r.stdout, r.stderr)
    assert "teardown returned" not in r.stdout
    if value is None:
        assert lines == [] and "snapshot failed" in r.stderr, r.stderr
    else:
        assert len(lines) == 1 and json.loads(lines[0])["value"] == value, lines
        assert "no engine measured" not in r.stderr
        if mode == "unprinted":
            assert "hard time limit" in json.loads(lines[0])["cut_short"]
