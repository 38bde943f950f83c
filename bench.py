#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Allreduce(SUM,double) GB/s, device-resident, 256 MiB.

  python bench.py --gpus 1 --steps K --warmup W           # N = 1 (default)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
  python bench.py --gpus N --steps K --warmup W           # N > 1 without a launcher: bench.py starts
                                                           # the line above itself (a child process)

Self-launch (N > 1, no WORLD_SIZE in the environment): before importing torch or touching the GPU,
this process starts `python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>` as a
child (never exec), relays rank 0's JSON line (adding a "launcher" record: the command, and that this
process loaded no HIP runtime and opened no GPU device) and exits with the child's status. The ranks
replace MPJRun's launch of one JVM per rank (src/runtime/starter/MPJRun.java:807-832). --dry-launch
prints the child command instead; --launch forces the path at any N (rehearsals).

Time budget (N > 1): --budget-s (default 300) bounds the optional phases, checked between phases on rank
0 and agreed by every rank: the headline engines and the configs[3]/[4] parity run first, then the
comparison variants, the end-to-end host rate and the HBM combine, each skipped once the budget is spent
(listed under "skipped_for_budget"; wall seconds per phase under "phase_wall_s"). At --hard-s (default
480) rank 0 prints the line for what was measured so far and every rank exits.

Workloads (a "step" = one pass of the hot path over one batch of resident synthetic input):
  N = 1: the metric's own point at one GPU — mpjx_allreduce(SUM, DOUBLE) of 256 MiB on a world of one
         rank (Reduce = arraycopy send -> recv, Bcast = nothing: 2 S of HBM traffic); step i on
         (send, recv) pair i % --sets (4), so no step reuses the Infinity Cache. BASELINE configs[1]
         (local Op.SUM combine of two 256 MiB double[], inout[i] = in[i] + inout[i]) is reported in
         the same line as "combine", with its own roofline and parity.
  N > 1: BASELINE configs[2] at N ranks — Allreduce SUM double, 256 MiB per rank, one process per
         GPU. Both libmpjx engines are timed on the same buffers — the RCCL exchange engine
         (exchange -> MST-order P-way HIP combine -> all-gather) and the HIP-IPC direct engine (one
         P-way kernel per rank over xGMI) — and the faster bit-exact one is reported (--engine).
         Every engine is first exercised in child processes before these ranks touch the GPU
         (tools/ipc_preflight for the IPC engines, tools/rccl_preflight for each RCCL variant): an
         engine that fails, faults or hangs there is skipped (reason under "engines").
value = aggregate algorithm bandwidth = (sum over ranks of the 256 MiB vector each rank reduces) /
time per step (nccl-tests "algbw", summed over ranks). Inputs are resident in HBM before timing.
Parity: N = 1 checks every element of the result (and of the combine's, against a host
recomputation); N > 1 checks a
sample of elements on every rank plus a checksum of every rank's whole result.
Rank 0 prints one JSON line. See DESIGN.md "Measurement" for every field.
"""
import argparse
import ctypes
import json
import os
import platform
import signal
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
METRIC = "Allreduce(SUM,double) GB/s device-resident @256 MiB, 1/2/4/8 MI355X"
# The N > 1 engines the line may report: libmpjx's own HIP-combine engines only (exchange over RCCL,
# its chunk pipelines, the HIP-IPC direct engine). RCCL's own ncclAllReduce is a comparison variant.
HEADLINE_ENGINES = ("rccl", "ipc", "ipc_pull", "ipc_dsync", "rccl_pipe64", "rccl_pipe32")
_T0 = time.perf_counter()
LAUNCH_ONLY = ("--launch", "--dry-launch", "--no-launch")  # launcher switches, not passed to the ranks


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mib", type=int, default=256, help="bytes per rank buffer, MiB")
    ap.add_argument("--sets", type=int, default=4,
                    help="N=1: independent operand sets cycled per step (cold operands: nothing reused "
                         "from the Infinity Cache)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true", help="N>1: skip the comparison timings")
    ap.add_argument("--allreduce", action="store_true",
                    help="run the N>1 Allreduce leg even at world size 1 (rehearsal under torchrun)")
    ap.add_argument("--engine", choices=["auto"] + list(HEADLINE_ENGINES),
                    default="auto",
                    help="N>1 engine: time all and report the fastest bit-exact one (auto), or one of them. "
                         "rccl_pipeNN = the RCCL engine with MPJX_PIPE_CHUNK_MIB=NN (chunk pipeline, two lanes). "
                         "Every one is a libmpjx HIP-combine engine; RCCL's own ncclAllReduce (MPJX_RCCL_NATIVE) "
                         "is timed as the comparison variant rccl_native, never reported as the value")
    ap.add_argument("--no-preflight", action="store_true",
                    help="N>1: time the IPC engines without the child-process check first")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal: every rank on cuda:0 (implies --engine ipc; RCCL variants skipped)")
    ap.add_argument("--budget-s", type=float, default=float(os.environ.get("MPJX_BENCH_BUDGET_S", "300")),
                    help="N>1: seconds after which the optional phases are skipped (checked between phases)")
    ap.add_argument("--hard-s", type=float, default=float(os.environ.get("MPJX_BENCH_HARD_S", "480")),
                    help="N>1: seconds after which rank 0 prints what was measured and every rank exits")
    ap.add_argument("--launch", action="store_true",
                    help="start the ranks as a child torch.distributed.run even at N = 1 (rehearsal)")
    ap.add_argument("--no-launch", action="store_true", help="never self-launch (N > 1 then needs a launcher)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="print the child command the self-launch would run, and exit")
    return ap.parse_args(argv)


# ---- self-launch: N ranks from a launcher-less `python bench.py --gpus N` ----------------------------
# Nothing in this section imports torch or loads HIP: it runs before the process touches the GPU.

def wants_launch(a, env=None):
    """True when this process should start the ranks itself: --gpus N > 1 (or --launch) and no launcher
    around it (WORLD_SIZE unset) and not already a self-launched rank."""
    env = os.environ if env is None else env
    if a.no_launch or env.get("MPJX_BENCH_LAUNCHED") or "WORLD_SIZE" in env:
        return False
    return a.launch or a.dry_launch or a.gpus > 1


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_command(a, argv, port):
    """The child command: the driver's own N > 1 form, one rank per GPU, with this run's arguments
    (the launcher switches dropped)."""
    rest = [x for x in argv if x not in LAUNCH_ONLY]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={max(1, a.gpus)}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + rest


def gpu_untouched_state():
    """What this process holds of the GPU stack: torch imported, the HIP runtime mapped, a GPU device
    node (/dev/kfd, /dev/dri/*) open. All false = it cannot have initialised the GPU."""
    try:
        maps = open("/proc/self/maps").read()
    except OSError:
        maps = ""
    dev_open = False
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                t = os.readlink(f"/proc/self/fd/{fd}")
            except OSError:
                continue
            dev_open |= t == "/dev/kfd" or t.startswith("/dev/dri/")
    except OSError:
        pass
    return {"torch_imported": "torch" in sys.modules, "hip_runtime_loaded": "libamdhip64" in maps,
            "gpu_device_open": dev_open}


def self_launch(a, argv):
    """Run the ranks as a child torch.distributed.run (its own process group), relay its stdout, add
    the launcher record to rank 0's JSON line. If the child ends without a JSON line (killed at this
    process's limit, --hard-s + 90 s (MPJX_BENCH_LAUNCH_GRACE_S), or crashed), print rank 0's last
    checkpoint (the line for what was measured, written to MPJX_BENCH_CHECKPOINT after every phase) or
    an error line."""
    port = free_port()
    cmd = launcher_command(a, argv, port)
    before = gpu_untouched_state()
    rec = {"self_launched": True, "cmd": " ".join(["python"] + cmd[1:]), "parent_before_spawn": before}
    if a.dry_launch:
        print(json.dumps({"launcher": rec}), flush=True)
        return 0
    ckpt = os.path.join("/tmp", f"mpjx_bench_ckpt_{os.getpid()}_{port}.json")
    env = dict(os.environ, MPJX_BENCH_LAUNCHED="1", MPJX_BENCH_CHECKPOINT=ckpt)
    limit = a.hard_s + float(os.environ.get("MPJX_BENCH_LAUNCH_GRACE_S", "90"))
    after_line = float(os.environ.get("MPJX_BENCH_AFTER_LINE_S", "90"))
    print(f"bench launcher: {' '.join(cmd)} (limit {limit:.0f} s)", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, start_new_session=True)

    def kill_group(sig):
        try:
            os.killpg(p.pid, sig)
        except OSError:
            pass

    def on_signal(signum, _frame):  # a supervisor stopping this process stops the ranks too
        kill_group(signal.SIGTERM)
        raise SystemExit(128 + signum)

    for s_ in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s_, on_signal)
    got_line = []

    def relay():
        for line in p.stdout:
            s = line.strip()
            if s.startswith("{") and '"metric"' in s:
                try:
                    d = json.loads(s)
                    d["launcher"] = dict(rec, parent_after=gpu_untouched_state())
                    line = json.dumps(d) + "\n"
                except ValueError:
                    pass
                got_line.append(time.monotonic())
            sys.stdout.write(line)
            sys.stdout.flush()

    th = threading.Thread(target=relay, daemon=True)
    th.start()
    killed = False
    t_start = time.monotonic()
    rc = None
    while rc is None:
        # the limit, or 90 s after rank 0's line when the ranks' teardown does not end (the line counts)
        left = limit - (time.monotonic() - t_start)
        if got_line:
            left = min(left, after_line - (time.monotonic() - got_line[0]))
        try:
            rc = p.wait(timeout=max(0.0, min(left, 1.0)))
        except subprocess.TimeoutExpired:
            if left <= 0:
                killed = True
                kill_group(signal.SIGTERM)
                try:
                    rc = p.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    kill_group(signal.SIGKILL)
                    rc = p.wait()
    th.join(timeout=10)
    if got_line and killed:
        rc = 0  # rank 0's line was relayed; only the teardown after it hung
    if not got_line:
        why = (f"the ranks were killed at the launcher's limit ({limit:.0f} s)" if killed
               else f"the ranks exited with status {rc} without a JSON line")
        try:
            d = json.load(open(ckpt))
            d["cut_short"] = why + "; this is rank 0's last checkpoint"
            d["launcher"] = dict(rec, parent_after=gpu_untouched_state())
            print(json.dumps(d), flush=True)
            rc = 0 if d.get("value") is not None else (rc or 1)
        except (OSError, ValueError):
            print(json.dumps({"metric": METRIC, "value": None, "n_gpus": a.gpus, "error": why,
                              "launcher": dict(rec, parent_after=gpu_untouched_state())}), flush=True)
            rc = rc or 1
    try:
        os.unlink(ckpt)
    except OSError:
        pass
    return rc


if __name__ == "__main__":
    _a = parse()
    if wants_launch(_a):
        sys.exit(self_launch(_a, sys.argv[1:]))

# The chunk-pipelined RCCL engines drive three streams per process (exchange #1, combine, all-gather)
# beside torch's. HIP's default of 4 hardware queues per process can put two of them on one queue,
# which serialises them: tools/c5_overlap.py --lanes measured NO overlap of the two exchange lanes at
# 4 queues and 3.1 of 3.7 ms overlapped at 16 (profiles/r03/c5_lanes_hwq*.jsonl). One process per GPU:
# 8 queues, set before the runtime initialises. Not for --one-device rehearsals, where several rank
# processes share one GPU's queue slots (the "24 ms second world").
sys.path.insert(0, os.path.join(ROOT, "tools"))
if int(os.environ.get("WORLD_SIZE", "1")) > 1 and "--one-device" not in sys.argv:
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402
import torch  # noqa: E402  (before libmpjx: one HIP runtime per process)

import synth  # noqa: E402  (SURVEY 8d splitmix64 input streams, GPU and host twins)

HBM_PEAK_GBPS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBPS = 153.6    # per link per the brief / SURVEY §8d; 7 links per GPU
ENGINE_TIMEOUT_S = float(os.environ.get("MPJX_BENCH_ENGINE_TIMEOUT_S", "120"))
PREFLIGHT_TIMEOUT_S = float(os.environ.get("MPJX_BENCH_PREFLIGHT_TIMEOUT_S", "120"))
TEARDOWN_S = 60.0  # N > 1: once the line is printed, every rank exits within this long
MPJX_SUM, MPJX_DOUBLE = 3, 8
MPJX_FLAG_BLOCKING = 0x10
MPJX_MAX, MPJX_BAND, MPJX_BXOR, MPJX_INT, MPJX_FLOAT = 1, 6, 10, 5, 7


class Budget:
    """The N > 1 run's time budget (VERDICT r4 "do this" #2). allow(phase, share) is collective: rank 0
    decides from its own clock (seconds since this process started < share * budget_s) and every rank
    gets rank 0's answer, so the ranks never split between running and skipping a collective phase. A
    phase allow() refuses is listed in .skipped; `with phase(name):` adds its wall seconds to .wall and
    names the phase in progress (.current, for the hard-limit line). dist = None: one rank, no agreement."""

    def __init__(self, dist, rank, budget_s, clock=None):
        self.dist, self.rank, self.budget_s = dist, rank, budget_s
        self.clock = clock or (lambda: time.perf_counter() - _T0)
        self.wall, self.skipped, self.current = {}, [], None

    def allow(self, phase, share=1.0):
        ok = self.clock() < share * self.budget_s
        if self.dist is not None:
            t = torch.tensor([1 if ok else 0], dtype=torch.int64)
            self.dist.broadcast(t, src=0)
            ok = bool(t.item())
        if not ok:
            self.skipped.append(phase)
            progress(f"{phase}: skipped (time budget {self.budget_s:.0f} s spent)")
        return ok

    class _Phase:
        def __init__(self, b, name):
            self.b, self.name = b, name

        def __enter__(self):
            self.t, self.prev, self.b.current = time.perf_counter(), self.b.current, self.name
            if os.environ.get("MPJX_BENCH_STALL_PHASE") == self.name:  # rehearsal knob: this phase hangs
                time.sleep(float(os.environ.get("MPJX_BENCH_STALL_S", "600")))
            return self

        def __exit__(self, *exc):
            self.b.wall[self.name] = round(self.b.wall.get(self.name, 0.0) + time.perf_counter() - self.t, 2)
            self.b.current = self.prev
            return False

    def phase(self, name):
        return Budget._Phase(self, name)


_EMITTED = threading.Lock()


def emit(line):
    """Print THE JSON line, once per process: the watchdog, the hard limit and the normal end may race
    to it; whichever comes first prints, the others print nothing."""
    if line is not None and _EMITTED.acquire(blocking=False):
        print(json.dumps(line), flush=True)
        return True
    return False


def hard_limit_status(rank, snapshot_fn, hard_s, phase):
    """--hard-s reached (runs on the hard-limit timer thread): rank 0 prints the line for what was
    measured (flagged cut_short); returns the exit status for every rank. If the line is already out (a
    teardown running past the limit), the run succeeded: 0. The snapshot runs while the main thread may
    be mutating its dicts or stuck inside libmpjx, so a failure in it is reported, never raised (the
    caller's os._exit must be reached)."""
    ok = True
    try:
        if rank == 0:
            ok = _EMITTED.locked() or emit(snapshot_fn(f"hard time limit {hard_s:.0f} s reached in phase "
                                                       f"{phase or '?'}; later phases not run"))
            ok = ok or _EMITTED.locked()
    except BaseException as e:  # noqa: BLE001
        print(f"bench: hard limit snapshot failed: {e!r}", file=sys.stderr, flush=True)
        ok = _EMITTED.locked()
    if rank == 0 and not ok:
        print(f"bench: hard time limit {hard_s:.0f} s reached with no engine measured", file=sys.stderr, flush=True)
    try:
        sys.stdout.flush()
    except Exception:  # noqa: BLE001
        pass
    return 0 if ok else 1


def progress(msg):
    """A progress line on stderr (rank 0): a long N > 1 run is never silent for minutes, which a
    supervising harness could read as a hang; stdout keeps the one JSON line."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"bench [{time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def seed(cfg, rank):
    return synth.seed(cfg, rank)


def mst_sum(vals, l, r, root):
    """Sampled-check restatement of the MST_Reduce grouping (src/mpi/PureIntracomm.java:1943-1992):
    the half holding `root` is the accumulator, the other half's sub-root result is added to it."""
    if l == r:
        return vals[l]
    mid = (l + r) // 2
    if root <= mid:
        own, other = mst_sum(vals, l, mid, root), mst_sum(vals, mid + 1, r, r)
    else:
        own, other = mst_sum(vals, mid + 1, r, root), mst_sum(vals, l, mid, l)
    return other + own


def sample_idx(n, k=65536):
    rng = np.random.default_rng(12345)
    idx = np.unique(np.concatenate([rng.integers(0, n, k), [0, n - 1]]))
    return idx


def checksum(a):
    """Fingerprint of an array's bits: (XOR, wrapping sum) of its little-endian 64-bit words (the
    byte tail zero-padded). Both are exact integer reductions, independent of order; two equal-length
    vectors with equal fingerprints differ only by a deliberate collision."""
    b = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
    if b.size % 8:
        b = np.concatenate([b, np.zeros(8 - b.size % 8, np.uint8)])
    w = b.view(np.uint64)
    return int(np.bitwise_xor.reduce(w)), int(np.add.reduce(w, dtype=np.uint64))


def checksum_torch(t):
    """bench.checksum on a torch tensor, on its own device (a bit view, no value conversion): the
    XOR by pairwise halving, the wrapping sum as torch's int64 sum (two's complement: the same value
    mod 2^64 in any order). Equal to checksum(t.cpu().numpy()) for tensors of whole 64-bit words."""
    w = t.reshape(-1).view(torch.int64)
    x = w
    while x.numel() > 1:
        if x.numel() % 2:
            x = torch.cat([x, x.new_zeros(1)])
        x = x[0::2] ^ x[1::2]
    m = (1 << 64) - 1
    return (int(x[0].item()) & m if x.numel() else 0), int(w.sum().item()) & m


def expected_checksum_device(n, world, dev, cfg=3):
    """The checksum of the whole MST(0) Allreduce result of `world` ranks' configs[cfg] streams,
    recomputed with torch on `dev` from the counter streams (synth.uniform_torch, the bit-identical
    twin of the host generator) and torch IEEE adds in the MST grouping — independent of libmpjx. At
    N = 8 the host version regenerates 8 x 256 MiB in numpy (about 16 s on rank 0); on the device it
    takes milliseconds."""
    vals = [synth.uniform_torch(n, seed(cfg, r), dev) for r in range(world)]
    res = mst_sum(vals, 0, world - 1, 0)
    ck = checksum_torch(res)
    del vals, res
    return ck


def ipc_preflight(dist, rank, world, local):
    """Exercise the HIP-IPC engine in CHILD processes (tools/ipc_preflight, one per rank, a throw-away
    IPC world of their own) before this process touches the GPU, so that a fault or hang of the
    cross-process engine on this node costs the children, not the run. Returns the same verdict on
    every rank: {"ok": bool, "msg": str, "s": seconds}."""
    exe = os.path.join(ROOT, "tools", "ipc_preflight")
    uid = [os.urandom(128).hex() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    t0 = time.perf_counter()
    progress("ipc preflight")
    if not os.path.exists(exe):
        ok, msg = False, "tools/ipc_preflight is not built (make -C mpjexpress_amd tools)"
    else:
        env = dict(os.environ, MPJX_IPC_TIMEOUT_S=str(max(10, int(PREFLIGHT_TIMEOUT_S / 2))))
        try:
            p = subprocess.run([exe, str(rank), str(world), str(local), uid[0]], env=env, capture_output=True,
                               text=True, timeout=PREFLIGHT_TIMEOUT_S)
            ok = p.returncode == 0
            msg = ((p.stdout or "") + (p.stderr or "")).strip()[-300:] or f"exit status {p.returncode}"
        except subprocess.TimeoutExpired:
            ok, msg = False, f"no verdict within {PREFLIGHT_TIMEOUT_S:.0f} s"
        except OSError as e:
            ok, msg = False, str(e)[:300]
    dsync = ok and "dsync ok" in msg
    nbad = torch.tensor([0 if ok else 1, 0 if dsync else 1], dtype=torch.int64)
    dist.all_reduce(nbad)
    if nbad[0].item() and ok:
        msg = f"{nbad[0].item()} rank(s) failed their preflight"
    return {"ok": nbad[0].item() == 0, "dsync_ok": nbad[1].item() == 0, "msg": msg,
            "s": round(time.perf_counter() - t0, 2)}


RCCL_VARIANTS = ("rccl", "rccl_skew", "rccl_p2p", "rccl_pipe64", "rccl_pipe32", "rccl_native")


def rccl_preflight(dist, rank, world, local, variants, budget=None):
    """Exercise every RCCL engine variant of libmpjx in CHILD processes (tools/rccl_preflight, one per
    rank, a throw-away RCCL world per variant) before this process touches the GPU: the first P > 1
    execution of the exchange engine's ncclAllToAll(v) / ncclAllGather / grouped send-recv — and of
    the two-communicator chunk pipelines — happens there. A variant whose child fails, faults, gives a
    wrong element or no verdict within PREFLIGHT_TIMEOUT_S on ANY rank is reported failed on every rank
    (the bench then skips it, reason under "engines"). Returns {variant: {"ok", "msg", "s"}}, the same on
    every rank. The child binary can be replaced (MPJX_RCCL_PREFLIGHT_EXE) to test this protocol. With a
    Budget, every variant after the first runs only while 30 % of the budget is left unspent; a skipped
    one is reported failed ("skipped for the time budget"), so plan_engines drops it."""
    exe = os.environ.get("MPJX_RCCL_PREFLIGHT_EXE") or os.path.join(ROOT, "tools", "rccl_preflight")
    out = {}
    for i, v in enumerate(variants):
        if i > 0 and budget is not None and not budget.allow(f"preflight:{v}", 0.3):
            out[v] = {"ok": False, "msg": "skipped for the time budget", "failed_ranks": 0, "s": 0.0}
            continue
        # rank 0's child publishes the RCCL unique id in this file (one node: the ranks share /tmp)
        tag = [os.urandom(8).hex() if rank == 0 else None]
        dist.broadcast_object_list(tag, src=0)
        uid_file = os.path.join("/tmp", f"mpjx_rccl_preflight_{tag[0]}_{v}")
        t0 = time.perf_counter()
        progress(f"rccl preflight: {v}")
        if not os.path.exists(exe):
            ok, msg = False, "tools/rccl_preflight is not built (make -C mpjexpress_amd tools)"
        else:
            env = dict(os.environ, MPJX_RCCL_TIMEOUT_S=str(max(10, int(PREFLIGHT_TIMEOUT_S / 4))))
            try:
                p = subprocess.run([exe, str(rank), str(world), str(local), v, uid_file], env=env,
                                   capture_output=True, text=True, timeout=PREFLIGHT_TIMEOUT_S)
                ok = p.returncode == 0
                msg = ((p.stdout or "") + (p.stderr or "")).strip()[-300:] or f"exit status {p.returncode}"
                if not ok and p.returncode < 0:
                    msg = f"killed by signal {-p.returncode}: " + msg
            except subprocess.TimeoutExpired:
                ok, msg = False, f"no verdict within {PREFLIGHT_TIMEOUT_S:.0f} s"
            except OSError as e:
                ok, msg = False, str(e)[:300]
        nbad = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(nbad)
        msgs = [None] * world
        dist.all_gather_object(msgs, None if ok else f"rank {rank}: {msg}")
        dist.barrier()  # every child of this variant has exited before anyone removes the file
        if rank == 0:
            for f in (uid_file, uid_file + ".tmp"):
                try:
                    os.unlink(f)
                except OSError:
                    pass
        bad = [m for m in msgs if m]
        out[v] = {"ok": nbad.item() == 0, "msg": (bad[0] if bad else msg)[-300:],
                  "failed_ranks": int(nbad.item()), "s": round(time.perf_counter() - t0, 2)}
    return out


def plan_engines(engine_names, ipc_pf, rccl_pf, world=None):
    """The engines and RCCL variants the bench may time, after the child-process preflights: an IPC
    engine is kept only if the IPC preflight passed (ipc_dsync also needs its device-sync world), an
    RCCL engine or variant only if its own preflight passed; every RCCL variant rides on the plain
    "rccl" world, so they all go when it fails. Only libmpjx's HIP-combine engines (HEADLINE_ENGINES)
    are engines; rccl_native (RCCL's own ncclAllReduce, bit-exact for Allreduce(SUM, DOUBLE) at P <= 2
    only) is a comparison variant at world <= 2. Returns (engines to time, RCCL comparison variants to
    time, {skipped name: reason})."""
    skipped = {}
    names = [e for e in engine_names if e in HEADLINE_ENGINES]
    dropped = {e: "not a libmpjx HIP-combine engine (timed as a comparison variant, if at all)"
               for e in engine_names if e not in HEADLINE_ENGINES}
    variants = [v for v in ("rccl_p2p", "rccl_skew") if any(e.startswith("rccl") for e in names)]
    if world is not None and world <= 2 and "rccl" in names:
        variants.append("rccl_native")
    if ipc_pf is not None and not ipc_pf["ok"]:
        for e in names:
            if e.startswith("ipc"):
                skipped[e] = "ipc preflight failed: " + ipc_pf["msg"]
        names = [e for e in names if not e.startswith("ipc")]
    elif ipc_pf is not None and not ipc_pf.get("dsync_ok", True) and "ipc_dsync" in names:
        skipped["ipc_dsync"] = "device-sync preflight failed: " + ipc_pf["msg"]
        names.remove("ipc_dsync")
    if rccl_pf is not None:
        base = rccl_pf.get("rccl", {"ok": True})
        for e in [x for x in names + variants if x.startswith("rccl")]:
            pf = rccl_pf.get(e, {"ok": True})
            if not base["ok"]:
                skipped[e] = "rccl preflight failed: " + base["msg"]
            elif not pf["ok"]:
                skipped[e] = f"{e} preflight failed: " + pf["msg"]
        names = [e for e in names if e not in skipped]
        variants = [v for v in variants if v not in skipped]
    for e, why in dropped.items():
        if e not in variants:
            skipped.setdefault(e, why)
    return names, variants, skipped


def pick_reported(engine_names, engines):
    """The engine the line reports: the fastest bit-exact one among libmpjx's HIP-combine engines
    (HEADLINE_ENGINES), else the first of them that ran (its parity fields say it was not bit-exact);
    None before any ran. RCCL's own reduction (rccl_native) is never a candidate: SURVEY 8(e) admits it
    as a transport-ceiling reference only."""
    cand = [e for e in engine_names if e in HEADLINE_ENGINES and "t" in engines.get(e, {})]
    exact = [e for e in cand if engines[e].get("mismatches") == 0 and engines[e].get("full_checksum_match") is True]
    pool = exact or cand[:1]
    return min(pool, key=lambda e: engines[e]["t"]) if pool else None


def traffic_from_profiles(kernel_tag):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(p))
        return d.get(kernel_tag, {}).get("hbm_bytes_per_launch")
    except Exception:  # noqa: BLE001
        return None


def runtime_versions(L):
    """HIP runtime and RCCL versions this process bound (torch's, loaded first), beside the ROCm the
    library was built with: the pairing the numbers were measured on."""
    h, r = ctypes.c_int(0), ctypes.c_int(0)
    rc = L.mpjx_runtime_versions(ctypes.byref(h), ctypes.byref(r))
    return {"hip_runtime": h.value if rc == 0 else None, "rccl": r.value if rc == 0 else None,
            "torch_hip": getattr(torch.version, "hip", None)}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def copy_peak(n, dev):
    """Measured device-to-device copy rate (read + write GB/s) over the same buffer size: the
    practical HBM ceiling next to the 8 TB/s spec."""
    a = torch.empty(n, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 / 1e3
    del a, b
    return round(2 * n * 8 / t / 1e9, 1)


def read_peak():
    """Measured HBM read-stream peak: tools/libhbm_probe.so streams 4 x 512 MiB with
    non-temporal 16-B loads, cycled so no launch reads from the Infinity Cache; None if not built."""
    p = os.path.join(ROOT, "tools", "libhbm_probe.so")
    if not os.path.exists(p):
        return None
    f = ctypes.CDLL(p).hbm_read_peak_GBps
    f.restype, f.argtypes = ctypes.c_double, [ctypes.c_int]
    v = f(24)
    return round(v, 1) if v > 0 else None


def cpu_baseline(n, budget_s):
    """The reference's host combine (typed-class round trip) timed on this host: oracle port."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU restatement, timed as the baseline only

    t1 = oracle.time_combine(oracle.SUM, oracle.DOUBLE, n, 1)
    reps = max(3, min(50, int(budget_s / max(t1, 1e-6))))
    t = oracle.time_combine(oracle.SUM, oracle.DOUBLE, n, reps)
    out = {"value": round(n * 8 / t / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
           "sample": f"{reps} x full-size combine of 2 x {n * 8 >> 20} MiB double[] "
                     f"(new T[] + arraycopy + perform loop + getResultant, SumDouble.java:49-67), "
                     f"median {t * 1e3:.1f} ms, host {cpu_model()}, nproc {os.cpu_count()}",
           "label": "restatement, not JIT'd Java (no JVM on the GPU box)"}
    out["allreduce_mst"] = allreduce_mst_baseline(oracle, n)
    return out


def allreduce_mst_baseline(oracle, n):
    """BASELINE.md's multi-threaded CPU baseline: the reference's pure-Java Allreduce =
    MST_Reduce(root 0) + MST_Broadcast (PureIntracomm.java:1943-1992, 702-736) with P ranks as P
    threads pinned to P distinct cores (multicore/smpdev), every hop paying mpjbuf pack + unpack with
    the big-endian swap (NIOBuffer.java:520-563) and the typed class's arraycopies — the oracle's
    timed restatement, not JIT'd Java. configs[0] (1 MiB, 4 ranks) and configs[2]'s shape on the host
    (256 MiB per rank, 8 ranks)."""
    res = {"kind": "port", "label": "restatement, not JIT'd Java (no JVM on the GPU box)",
           "host": cpu_model(), "nproc": os.cpu_count()}
    for name, P, elems, reps in (("configs0_1MiB_p4", 4, 131072, 50), ("configs2_256MiB_p8", 8, n, 3)):
        if (os.cpu_count() or 1) < P:
            res[name] = {"skipped": f"needs {P} cores"}
            continue
        t = oracle.time_allreduce_mst(P, elems, reps, True)
        S = elems * 8
        res[name] = {"ms": round(t * 1e3, 3), "algbw_GBps": round(S / t / 1e9, 3),
                     "aggregate_GBps": round(P * S / t / 1e9, 3), "cores": P, "ranks": P, "reps": reps,
                     "bytes_per_rank": S}
    return res


def configs0_multicore(L, dev, calls):
    """BASELINE configs[0] — Allreduce(SUM, DOUBLE) of 1 MiB at P = 4, the reference's own CPU-runnable
    case — in the reference's multicore mode: 4 rank threads of this process on one GPU
    (mpjx_comm_init_smp; smpdev, src/runtime/starter/MulticoreStarter.java:309-322), each issuing `calls`
    back-to-back blocking calls (MPJX_FLAG_BLOCKING, as the mpiJava call: each returns complete) on its
    communicator's stream (the direct engine: rank 0 launches one P-way kernel for all four, drains its
    stream, two host rendezvous per call). us_per_call = the slowest rank's time / calls.
    Every element of every rank's result is checked bit for bit against the MST(0) grouping. Beside it
    stands cpu_baseline.allreduce_mst.configs0_1MiB_p4: the reference's algorithm on 4 host threads."""
    import threading

    from mpjexpress_amd import _lib

    P, n1 = 4, (1 << 20) // 8
    arr = (ctypes.c_void_p * P)()
    devs = (ctypes.c_int * P)(*([dev.index or 0] * P))
    _lib.check(L.mpjx_comm_init_smp(arr, P, devs), "mpjx_comm_init_smp")
    comms = [ctypes.c_void_p(arr[r]) for r in range(P)]
    try:
        xs = [synth.uniform_torch(n1, seed(1, r), dev) for r in range(P)]
        ys = [torch.empty_like(x) for x in xs]
        torch.cuda.synchronize()
        times, errs = [None] * P, [None] * P

        def body(r):
            try:
                torch.cuda.set_device(dev)
                c = comms[r]
                # the arguments converted once: the loop below costs the Python rank thread as little as
                # possible (it still holds the GIL between calls, which C++ or JVM rank threads do not)
                f, sp, rp = L.mpjx_allreduce, ctypes.c_void_p(xs[r].data_ptr()), ctypes.c_void_p(ys[r].data_ptr())
                nn = ctypes.c_int64(n1)

                def call():  # blocking, as the mpiJava call (MPJX_FLAG_BLOCKING: returns complete)
                    st = f(c, sp, rp, nn, MPJX_DOUBLE, MPJX_SUM, MPJX_FLAG_BLOCKING, None)
                    if st != 0:
                        _lib.check(st, "mpjx_allreduce")

                for _ in range(5):
                    call()
                _lib.check(L.mpjx_comm_synchronize(c), "sync")
                _lib.check(L.mpjx_barrier(c), "barrier")
                t0 = time.perf_counter()
                for _ in range(calls):
                    call()
                _lib.check(L.mpjx_comm_synchronize(c), "sync")
                times[r] = time.perf_counter() - t0
            except BaseException as e:  # noqa: BLE001
                errs[r] = e

        th = [threading.Thread(target=body, args=(r,)) for r in range(P)]
        for t_ in th:
            t_.start()
        for t_ in th:
            t_.join()
        for e in errs:
            if e is not None:
                raise e
        full = np.arange(n1, dtype=np.uint64)
        exp = mst_sum([synth.uniform_np(full, seed(1, r)) for r in range(P)], 0, P - 1, 0)
        bad = sum(int(np.count_nonzero(y.cpu().numpy().view(np.uint64) != exp.view(np.uint64))) for y in ys)
        t = max(times) / calls
        return {"us_per_call": round(t * 1e6, 2), "calls": calls, "ranks": P, "bytes_per_rank": n1 * 8,
                "engine": "multicore direct (4 rank threads, one GPU)", "elements_checked": P * n1,
                "mismatches": bad, "bit_exact": bad == 0,
                "note": "configs[0] on the GPU in multicore mode; the reference's algorithm on the host at the same "
                        "shape is cpu_baseline.allreduce_mst.configs0_1MiB_p4"}
    finally:
        for c in comms:
            L.mpjx_comm_destroy(c)


def configs0_native():
    """The same configs[0] call from C++ rank threads — what a JVM's native rank threads see, without
    Python's GIL hand-over between calls: tools/latency's multicore sweep up to 1 MiB (a child process;
    every result element checked there, exit status 3 on a mismatch), its 1 MiB row."""
    exe = os.path.join(ROOT, "tools", "latency")
    if not os.path.exists(exe):
        return {"error": "tools/latency is not built (make -C mpjexpress_amd tools)"}
    try:
        r = subprocess.run([exe, "4", "1"], capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            return {"error": f"tools/latency exit {r.returncode}: {(r.stderr or r.stdout)[-200:]}"}
        d = json.loads(r.stdout[r.stdout.index("{"):])
        row = next(x for x in d["rows"] if x["bytes"] == 1 << 20)
        return {"us_per_call": row["direct_us"], "checked": True, "launch_sync_floor_us": d["single_thread_launch_sync_floor_us"],
                "how": "tools/latency 4 1: blocking calls, per-call median, max over 4 rank threads"}
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)[:200]}


def allreduce_p1(L, n, dev, steps, warmup, sets):
    """The metric's own P = 1 point (Allreduce at one rank = 2·S of HBM traffic, read send
    + write recv): mpjx_allreduce on a world of one rank, 256 MiB double, on the communicator's own
    stream (stream argument NULL, as the JNI shim calls it), timed with HIP events on that stream
    around K back-to-back calls, step i on (send, recv) pair i % sets (cold, as the combine); every
    result is checked bit for bit (it is a copy)."""
    from mpjexpress_amd import _lib

    arr = (ctypes.c_void_p * 1)()
    devs = (ctypes.c_int * 1)(dev.index or 0)
    _lib.check(L.mpjx_comm_init_smp(arr, 1, devs), "mpjx_comm_init_smp")
    c = ctypes.c_void_p(arr[0])
    cs = ctypes.c_void_p()
    _lib.check(L.mpjx_comm_stream(c, ctypes.byref(cs)), "mpjx_comm_stream")
    stream = torch.cuda.ExternalStream(cs.value, device=dev)
    sp = None
    try:
        bufs = []
        for k in range(sets):
            send = synth.uniform_torch(n, seed(3, k), dev)
            bufs.append((send, torch.empty_like(send)))
        torch.cuda.synchronize()

        def step(i):
            send, recv = bufs[i % sets]
            _lib.check(L.mpjx_allreduce(c, send.data_ptr(), recv.data_ptr(), n, MPJX_DOUBLE, MPJX_SUM, 0, sp),
                       "mpjx_allreduce")

        for i in range(warmup):
            step(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for i in range(steps):
            step(warmup + i)
        e1.record(stream)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / steps
        kern_s = e0.elapsed_time(e1) / steps / 1e3
        used = bufs[:min(sets, steps + warmup)]  # every pair a call wrote
        ok = all(bool(torch.equal(s_.view(torch.int64), r_.view(torch.int64))) for s_, r_ in used)
        S = n * 8
        del bufs
        return {"value": round(S / t / 1e9, 2), "unit": "GB/s", "ms_per_step": round(t * 1e3, 4),
                "kernel_us": round(kern_s * 1e6, 2), "algorithmic_bytes_per_call": 2 * S, "sets": sets,
                "hbm_GBps": round(2 * S / kern_s / 1e9, 1), "frac": round(2 * S / kern_s / 1e9 / HBM_PEAK_GBPS, 4),
                "traffic": traffic_from_profiles("copies_256MiB"), "bit_exact": ok,
                "kernel": "k_copies (Reduce = arraycopy send->recv, Bcast = nothing at P=1)"}
    finally:
        L.mpjx_comm_destroy(c)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        a.gpus = world if world > 1 else a.gpus
    if a.one_device:
        local = 0
        if a.engine.startswith("rccl"):
            raise SystemExit("--one-device: RCCL cannot place two ranks on one GPU; use --engine auto|ipc|ipc_pull")
        # the rehearsal allocates its buffers once and frees nothing while the IPC worlds live, the
        # condition under which libmpjx accepts rank processes that share a GPU
        os.environ["MPJX_IPC_OVERSUBSCRIBE"] = "1"
    dist = None
    budget = Budget(None, rank, a.budget_s)
    # rank 0's line for what was measured so far (set by the N > 1 leg below); the hard limit prints it
    snap = {"fn": lambda note=None: None}
    hl = None
    if world > 1 or a.allreduce:
        # a finite limit on every RCCL wait: a hang in the P > 1 exchange path (first run on the driver's
        # node) becomes an MPJX_ERR_RCCL reported under engines.rccl.error, not a killed run
        os.environ.setdefault("MPJX_RCCL_TIMEOUT_S", "60")
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        budget = Budget(dist, rank, a.budget_s)

        def hard_limit():
            code = 1
            try:
                code = hard_limit_status(rank, snap["fn"], a.hard_s, budget.current)
            finally:
                os._exit(code)

        hl = threading.Timer(max(1.0, a.hard_s - (time.perf_counter() - _T0)), hard_limit)
        hl.daemon = True
        hl.start()
    # newest last: a stall in an engine's first run on the 8-GPU node costs only the engines after it
    # (the watchdog prints what was measured). rccl_native (RCCL's own ncclAllReduce, bit-exact for
    # Allreduce(SUM, DOUBLE) at P <= 2 only) is a comparison variant at world sizes 1 and 2, not an engine.
    engine_names = list(HEADLINE_ENGINES) if a.engine == "auto" else [a.engine]
    if a.one_device:
        engine_names = [e for e in engine_names if not e.startswith("rccl")]
    preflight = rpf = None
    if dist is not None and not a.no_preflight:  # child processes, before this process touches the GPU
        if any(e.startswith("ipc") for e in engine_names):
            with budget.phase("preflight:ipc"):
                preflight = ipc_preflight(dist, rank, world, local)
        if any(e.startswith("rccl") for e in engine_names):
            rv = ["rccl"] + [e for e in engine_names if e.startswith("rccl_pipe")]
            if not a.no_variants:
                rv += ["rccl_skew", "rccl_p2p"] + (["rccl_native"] if world <= 2 else [])
            with budget.phase("preflight:rccl"):
                rpf = rccl_preflight(dist, rank, world, local, rv, budget)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from mpjexpress_amd import _lib

    L = _lib.lib()
    n = a.mib * (1 << 20) // 8
    S = n * 8

    def barrier():
        if dist is not None:
            dist.barrier()

    if world == 1 and not a.allreduce:
        # ---- configs[1]: inout = in + inout, 2 x 256 MiB double, one kernel per step ----------
        # Cold: step i works on pair i % R of R independent (inout, in) pairs, so between two uses of
        # a pair 2(R-1) x 256 MiB of other operands stream through the chip and nothing of it is left
        # in the 256 MiB Infinity Cache — every step reads its operands from HBM, as an Op.perform over
        # a freshly received message does. (Re-running the same pair lets the cache hold part of `in`
        # between steps: that warm figure is reported beside it, never as the value.)
        R = max(2, a.sets)
        progress("configs[1] combine")
        stream = torch.cuda.Stream(device=dev)
        sp = ctypes.c_void_p(stream.cuda_stream)
        pairs = [(synth.uniform_torch(n, seed(2, 2 * k), dev), synth.uniform_torch(n, seed(2, 2 * k + 1), dev))
                 for k in range(R)]
        uses = [0] * R
        torch.cuda.synchronize()

        def step(i):
            io, x = pairs[i % R]
            uses[i % R] += 1
            _lib.check(L.mpjx_combine(MPJX_SUM, MPJX_DOUBLE, io.data_ptr(), x.data_ptr(), n, sp), "mpjx_combine")

        for i in range(a.warmup):
            step(i)
        torch.cuda.synchronize()
        # one HIP event pair on the launch stream around the K back-to-back launches: the average
        # launch duration (incl. the ~1.5 us kernel boundary), without per-launch event packets
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        for i in range(a.steps):
            step(a.warmup + i)
        e1.record(stream)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / a.steps
        kern_s = e0.elapsed_time(e1) / a.steps / 1e3
        alg = 3 * S  # read in, read inout, write inout
        achieved = alg / kern_s / 1e9
        # warm, for comparison only: the same pair every launch (K more launches on pair 0)
        e0.record(stream)
        for _ in range(a.steps):
            step(0)
        e1.record(stream)
        torch.cuda.synchronize()
        warm_s = e0.elapsed_time(e1) / a.steps / 1e3
        traffic = traffic_from_profiles("combine_sum_f64_256MiB")
        # full-size parity, every element of every pair: inout after its uses = in + (... + (in + inout0)),
        # bit for bit, recomputed on the host from the same counter streams
        bad = 0
        full = np.arange(n, dtype=np.uint64)
        for k in range(R):
            got = pairs[k][0].cpu().numpy()
            x, xin = synth.uniform_np(full, seed(2, 2 * k)), synth.uniform_np(full, seed(2, 2 * k + 1))
            for _ in range(uses[k]):
                np.add(xin, x, out=x)
            bad += int(np.count_nonzero(got.view(np.uint64) != x.view(np.uint64)))
            del got, x, xin
        del full, pairs
        rp = read_peak()
        combine = {
            "workload": "configs[1]: local Op.SUM combine of two 256 MiB double[] on 1 MI355X (kernel only, no "
                        "RCCL); operands cold: step i on pair i % sets",
            "value": round(S / t / 1e9, 2), "unit": "GB/s (S/t, S = 256 MiB operand)", "ms_per_step": round(t * 1e3, 4),
            "elements": n, "bytes_per_operand": S, "op": "SUM", "datatype": "DOUBLE", "sets": R,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "frac_of_measured_read": round(achieved / rp, 4) if rp else None,
                         "traffic": traffic, "kernel": "k_pway<Sum<double>,2,K_FOLD,W=2,TH=1024,U=1,POL=1>",
                         "algorithmic_bytes_per_launch": alg, "kernel_us": round(kern_s * 1e6, 2),
                         "warm_same_buffers": {"kernel_us": round(warm_s * 1e6, 2),
                                               "achieved": round(alg / warm_s / 1e9, 1),
                                               "note": "the same pair every launch, for comparison only: a figure "
                                                       "above the cold one would be Infinity-Cache reuse, not HBM"}},
            "parity": {"elements_checked": n * R, "mismatches": bad, "bit_exact": bad == 0},
        }
        # ---- the metric's own P = 1 point: Allreduce SUM double 256 MiB on a world of one rank ----
        progress("Allreduce at P = 1")
        ar = allreduce_p1(L, n, dev, a.steps, a.warmup, R)
        out = {
            "metric": METRIC, "value": ar["value"], "unit": "GB/s", "n_gpus": 1,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": ar["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: U[-1,1) doubles, splitmix64 counter streams, seed 0x4D504A00+1000*cfg+rank (SURVEY 8d)",
            "config": {"workload": "configs[2]'s operation at N = 1: Allreduce(SUM, DOUBLE) 256 MiB, device-resident, "
                                   "one rank (mpjx_allreduce on a world of one: Reduce = arraycopy send -> recv, "
                                   "PureIntracomm.java:1937; Bcast = nothing); operands cold: call i on (send, recv) "
                                   "pair i % sets. value = S/t per call, the same N*S/t definition as N > 1",
                       "elements": n, "bytes_per_rank": S, "op": "SUM", "datatype": "DOUBLE",
                       "sets": R, "parallelism": "single GPU", "engine": "one rank (copy)"},
            "roofline": {"bound": "hbm", "achieved": ar["hbm_GBps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": ar["frac"], "frac_of_measured_read": round(ar["hbm_GBps"] / rp, 4) if rp else None,
                         "traffic": ar["traffic"], "kernel": "k_copies<true> (512 lanes x one 16-B vector, non-temporal)",
                         "algorithmic_bytes_per_launch": ar["algorithmic_bytes_per_call"], "kernel_us": ar["kernel_us"],
                         "measured_copy_GBps": copy_peak(n, dev), "measured_read_GBps": rp},
            "parity": {"elements_checked": n * R, "bit_exact": ar["bit_exact"],
                       "reference_order": "P = 1: recv = send, bit for bit"},
            "combine": combine,
        }
        progress("configs[0] in multicore mode")
        try:
            out["configs0_multicore_p4"] = configs0_multicore(L, dev, max(200, 10 * a.steps))
        except Exception as e:  # noqa: BLE001  (a variant's failure must not lose the headline)
            out["configs0_multicore_p4"] = {"error": str(e)[:200]}
        out["configs0_multicore_p4"]["native_rank_threads"] = configs0_native()
        if not a.no_cpu_baseline:
            progress("cpu baseline")
            out["cpu_baseline"] = cpu_baseline(n, a.cpu_seconds)
        out["runtime"] = runtime_versions(L)
        print(json.dumps(out), flush=True)
        return

    # ---- N > 1: configs[2] Allreduce SUM double 256 MiB per rank, one process per GPU -----------
    # Two product engines: the RCCL exchange engine and the HIP-IPC direct engine.
    # --engine auto (default) times both on the same buffers and reports the faster one whose
    # full-size sampled parity is bit-exact; the other is listed under "engines".
    send = synth.uniform_torch(n, seed(3, rank), dev)
    recv = torch.empty_like(send)
    torch.cuda.synchronize()
    idx = sample_idx(n)
    exp_ck = {}

    def expected_checksum():
        """Checksum of the whole MST(0) result, recomputed on rank 0's device from every rank's stream
        (expected_checksum_device: torch ops, independent of libmpjx)."""
        if "v" not in exp_ck:
            exp_ck["v"] = expected_checksum_device(n, world, dev)
            torch.cuda.synchronize()
        return exp_ck["v"]

    def timed(fn, steps, warmup, sync_comm):
        for _ in range(warmup):
            fn()
        _lib.check(L.mpjx_comm_synchronize(sync_comm), "sync")
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        _lib.check(L.mpjx_comm_synchronize(sync_comm), "sync")
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        barrier()
        return el.item() / steps

    def parity():
        """(sampled mismatches summed over ranks, every rank's whole-result checksum == rank 0's host
        recomputation) for the current recv, against the MST(0) grouping of all ranks' sends; None
        where the checker itself failed."""
        try:
            got = recv[torch.from_numpy(idx).to(dev)].cpu().numpy()
            exp = mst_sum([synth.uniform_np(idx, seed(3, r)) for r in range(world)], 0, world - 1, 0)
            nbad = int(np.count_nonzero(got.view(np.uint64) != exp.view(np.uint64)))
            ck = checksum_torch(recv)
        except Exception:  # noqa: BLE001  (a checker failure must not lose the measurement)
            nbad, ck = -1, None
        bad_t = torch.tensor([nbad if nbad >= 0 else 1 << 40], dtype=torch.int64)
        dist.all_reduce(bad_t)
        cks = [None] * world
        dist.all_gather_object(cks, ck)
        full = [None]
        if rank == 0:
            try:
                e = expected_checksum()
                full[0] = all(c is not None and tuple(c) == e for c in cks)
            except Exception:  # noqa: BLE001
                full[0] = None
        dist.broadcast_object_list(full, src=0)
        return (int(bad_t.item()) if bad_t.item() < 1 << 40 else None), full[0]

    def all_ok(ok):
        """True iff `ok` on every rank (collective)."""
        t_ = torch.tensor([1 if ok else 0], dtype=torch.int64)
        dist.all_reduce(t_, op=dist.ReduceOp.MIN)
        return bool(t_.item())

    def phases(c):
        """Where one Allreduce's time goes (phase_breakdown), after the timed calls."""
        recv.zero_()
        torch.cuda.synchronize()
        return phase_breakdown(L, c, dist, lambda: _lib.check(
            L.mpjx_allreduce(c, send.data_ptr(), recv.data_ptr(), n, MPJX_DOUBLE, MPJX_SUM, 0, None), "mpjx_allreduce"))

    def make_comm(kind):
        """A communicator of one engine kind: "rccl", or an IPC world ("ipc" push, "ipc_pull",
        "ipc_dsync" push with device-side synchronisation). MPJX_IPC_MODE / MPJX_IPC_SYNC are read at
        init, so each IPC variant is a world of its own."""
        uid = [None]
        if rank == 0:
            uid[0] = _lib_unique_id(L) if kind.startswith("rccl") else os.urandom(128)
        dist.broadcast_object_list(uid, src=0)
        c = ctypes.c_void_p()
        if kind.startswith("rccl"):
            _lib.check(L.mpjx_comm_init_rank(ctypes.byref(c), world, uid[0], rank, local), "mpjx_comm_init_rank")
            return c
        env = {"MPJX_IPC_MODE": "pull" if kind == "ipc_pull" else "push"}
        if kind == "ipc_dsync":  # "device-shared" (one-GPU rehearsals) is kept
            prev = os.environ.get("MPJX_IPC_SYNC")
            env["MPJX_IPC_SYNC"] = prev if prev in ("device", "device-shared") else "device"
        else:
            env["MPJX_IPC_SYNC"] = "host"
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            _lib.check(L.mpjx_comm_init_ipc(ctypes.byref(c), world, uid[0], rank, local), "mpjx_comm_init_ipc")
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        return c

    def engine_env(e):
        """Settings of an engine (libmpjx reads MPJX_PIPE_CHUNK_MIB per call; MPJX_RCCL_P2P and
        MPJX_RCCL_NATIVE at communicator init, so those variants get communicators of their own)."""
        return {"MPJX_PIPE_CHUNK_MIB": e[len("rccl_pipe"):]} if e.startswith("rccl_pipe") else {}

    class env_set:
        def __init__(self, env):
            self.env = env

        def __enter__(self):
            self.old = {k: os.environ.get(k) for k in self.env}
            os.environ.update(self.env)

        def __exit__(self, *exc):
            for k, v in self.old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            return False

    def engine_label(best):
        if best.startswith("rccl_pipe"):
            return (f" via libmpjx's RCCL exchange engine, {best[len('rccl_pipe'):]} MiB chunk pipeline "
                    "(exchange #1 / combine / all-gather on three streams, two RCCL communicators)")
        if best == "rccl":
            return " via libmpjx's RCCL exchange engine"
        return (" via libmpjx's HIP-IPC direct engine (" + ("pull" if best == "ipc_pull" else "push")
                + (", device-synchronised)" if best == "ipc_dsync" else ")"))

    def result(best, t, bad, full, variants):
        """The JSON line for the engine `best` (time per step t, sampled parity mismatches bad, whole-
        result checksum verdict full)."""
        algbw = S / t / 1e9
        busbw = algbw * 2 * (world - 1) / world
        peak = (world - 1) * XGMI_LINK_GBPS
        res = {
            "metric": METRIC, "value": round(world * algbw, 2), "unit": "GB/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(t * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: U[-1,1) doubles, splitmix64 counter streams, seed 0x4D504A00+1000*cfg+rank (SURVEY 8d)",
            "config": {"workload": f"configs[2] at {world} ranks: Allreduce SUM double {S >> 20} MiB per rank, "
                                   + ("all ranks on ONE MI355X (rehearsal of the multi-process path, not an "
                                      "xGMI figure)" if a.one_device else "one process per MI355X")
                                   + engine_label(best),
                       "elements": n, "bytes_per_rank": S, "op": "SUM", "datatype": "DOUBLE",
                       "parallelism": f"{best}-{'one-device' if a.one_device else 'xgmi'} x{world}",
                       "engine": best},
            "engines": {k: {x: y for x, y in v.items() if x != "t"} for k, v in engines.items()},
            "algbw_GBps_per_rank": round(algbw, 2), "busbw_GBps": round(busbw, 2),
            "roofline": ({"bound": "xgmi", "achieved": round(busbw, 1), "peak": round(peak, 1),
                          "unit": "GB/s", "frac": round(busbw / peak, 4) if peak else None, "traffic": None,
                          "note": "busBW = algBW*2(P-1)/P against (P-1) direct xGMI links"}
                         if not a.one_device else
                         {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": None,
                          "traffic": None, "note": "one-device rehearsal: every rank shares one GPU's HBM; "
                                                   "no xGMI roofline applies"}),
            "variants": variants,
            "parity": {"sampled_elements_per_rank": int(idx.size), "mismatches": bad,
                       "full_result_checksum_match": full, "bit_exact": bad == 0 and full is True,
                       "reference_order": "MST_Reduce(root 0) grouping, PureIntracomm.java:1943-1992"},
        }
        if preflight is not None:
            res["ipc_preflight"] = preflight
        if rpf is not None:
            res["rccl_preflight"] = rpf
        return res

    variants = {}
    hbm = {}  # rank 0: roofline.hbm_combine once measured

    def snapshot(note=None):
        """Rank 0's line for what has been measured so far: the fastest bit-exact engine (else the first
        that ran) with every variant, phase wall time and budget skip recorded up to now; None before
        any engine finished. The end of the run, the watchdog and the hard limit all print this."""
        eng = dict(engines)  # copies: the hard limit calls this from a timer thread
        b = pick_reported(list(eng), eng)
        if b is None:
            return None
        res = result(b, eng[b]["t"], eng[b]["mismatches"], eng[b]["full_checksum_match"], dict(variants))
        if "v" in hbm:
            res["roofline"]["hbm_combine"] = hbm["v"]
        link = variants.get("p2p_one_link", {}).get("GBps")
        if link and not a.one_device and world > 1:
            # the same link utilisation against the one-direction rate measured on one link in this run:
            # every rank moves 2S/P per link per direction, so per-link rate = busBW/(P-1)
            res["roofline"]["measured_link_GBps"] = link
            res["roofline"]["frac_vs_measured_links"] = round(res["busbw_GBps"] / ((world - 1) * link), 4)
        res["budget"] = {"budget_s": a.budget_s, "hard_s": a.hard_s,
                         "wall_s": round(time.perf_counter() - _T0, 1),
                         "phase_wall_s": dict(budget.wall), "skipped_for_budget": list(budget.skipped)}
        if note:
            res["cut_short"] = note
        res["runtime"] = rt_versions
        return res

    rt_versions = runtime_versions(L)  # once, here: snapshot() may run on the hard-limit timer thread
    snap["fn"] = snapshot

    def checkpoint():
        """Rank 0 writes the line so far where a self-launching parent can find it (MPJX_BENCH_CHECKPOINT):
        if the ranks die without printing, the parent prints this instead of nothing."""
        path = os.environ.get("MPJX_BENCH_CHECKPOINT")
        if rank != 0 or not path:
            return
        try:
            res = snapshot("checkpoint")
            if res is not None:
                with open(path + ".tmp", "w") as f:
                    json.dump(res, f)
                os.replace(path + ".tmp", path)
        except Exception as e:  # noqa: BLE001  (a checkpoint must never cost the run)
            progress(f"checkpoint failed: {e}")

    class Watchdog:
        """Insurance around every phase that talks to the other ranks (engine init, timing, variants):
        if it makes no progress within ENGINE_TIMEOUT_S, rank 0 prints the line for what was already
        measured (or every rank exits nonzero when no engine finished) and every rank exits, so a
        hang — in RCCL, whose P > 1 path runs first on the driver's node, or in an IPC world — ends
        the run with a record instead of consuming the driver's time limit."""

        def __init__(self, phase):
            self.phase = phase

        def fire(self):
            res = snapshot(f"{self.phase} stalled (no progress in {ENGINE_TIMEOUT_S:.0f} s); run cut short")
            if rank == 0:
                if res is not None:
                    res["engines"].setdefault(self.phase, {})["error"] = f"no progress in {ENGINE_TIMEOUT_S} s"
                    emit(res)
                else:
                    print(f"bench: {self.phase} made no progress in {ENGINE_TIMEOUT_S} s and no engine finished",
                          file=sys.stderr, flush=True)
            sys.stdout.flush()
            os._exit(0 if res is not None else 1)

        def __enter__(self):
            progress(f"{self.phase} ...")
            self.t = threading.Timer(ENGINE_TIMEOUT_S, self.fire)
            self.t.daemon = True
            self.t.start()
            return self

        def __exit__(self, *exc):
            self.t.cancel()
            return False

    engine_names, rccl_variants, skipped = plan_engines(engine_names, preflight, rpf, world)
    cmp_variants = ("rccl_skew", "rccl_p2p", "rccl_native")
    engines = {e: {"skipped": why} for e, why in skipped.items() if e not in cmp_variants}
    variants.update({e: {"skipped": why} for e, why in skipped.items() if e in cmp_variants})
    if not engine_names:
        if rank == 0:
            emit({"metric": METRIC, "value": None, "error": "every engine failed its preflight",
                  "engines": engines, "ipc_preflight": preflight, "rccl_preflight": rpf})
        dist.destroy_process_group()
        raise SystemExit(1)
    rcomm = None
    for i, eng in enumerate(engine_names):
        # each engine in a world of its own, timed alone: an IPC world is destroyed before the next one
        # is created (two live worlds in the same processes slowed the second 10x). The
        # first engine always runs; the others while half the budget is left.
        if i > 0 and not budget.allow(f"engine:{eng}", 0.5):
            engines[eng] = {"skipped": "time budget spent"}
            continue
        c = None
        with budget.phase(f"engine:{eng}"), Watchdog(eng), env_set(engine_env(eng)):
            try:
                c = make_comm(eng)
                recv.zero_()
                torch.cuda.synchronize()

                def step(c=c):
                    _lib.check(L.mpjx_allreduce(c, send.data_ptr(), recv.data_ptr(), n, MPJX_DOUBLE, MPJX_SUM, 0,
                                                None), "mpjx_allreduce")

                te = timed(step, a.steps, a.warmup, c)
                mism, full = parity()
                engines[eng] = {"ms": round(te * 1e3, 4),
                                "busbw_GBps": round(S / te / 1e9 * 2 * (world - 1) / world, 2),
                                "mismatches": mism, "full_checksum_match": full, "t": te}
                engines[eng]["phases"] = phases(c)
                if engine_env(eng):
                    engines[eng]["env"] = engine_env(eng)
            except Exception as e:  # noqa: BLE001  (an engine that fails is reported, the others still measured)
                engines[eng] = {"error": str(e)[:300]}
            if eng == "rccl" and c is not None:
                rcomm = c  # kept for the variants
            elif c is not None:
                L.mpjx_comm_destroy(c)
        checkpoint()
    # the phases below that use the kept RCCL communicator are collective: every rank must agree it has one
    if not all_ok(rcomm is not None) and rcomm is not None:
        L.mpjx_comm_destroy(rcomm)
        rcomm = None
    best = pick_reported(engine_names, engines)  # nothing bit-exact: the first that ran, flagged by parity
    if best is None:
        raise RuntimeError(f"no engine ran: {engines}")
    best_kind = "rccl" if best.startswith("rccl") else best

    def configs_on(eng):
        """The other BASELINE configs at this N (full-size parity checked on device) on engine `eng`: the
        kept RCCL communicator (whose pipeline variant is timed inside) or a new IPC world; keys prefixed
        with the engine when it is not the reported one."""
        with budget.phase(f"{eng}:other_configs"), Watchdog(f"{eng}:other_configs"):
            c = rcomm if eng == "rccl" else None
            cs = ctypes.c_void_p()
            try:
                if c is None:
                    c = make_comm(eng)
                _lib.check(L.mpjx_comm_stream(c, ctypes.byref(cs)), "mpjx_comm_stream")
                got = other_configs(L, c, cs, world, rank, dev, lambda f, k, w, c=c: timed(f, k, w, c), a.steps,
                                    all_ok, pipe_variant=(eng == "rccl"), dist=dist, one_device=a.one_device)
                variants.update(got if eng == best_kind else {f"{eng}:{k}": v for k, v in got.items()})
            except Exception as e:  # noqa: BLE001
                variants["other_configs" if eng == best_kind else f"{eng}:other_configs"] = {"error": str(e)[:200]}
            finally:
                if c is not None and eng != "rccl":
                    L.mpjx_comm_destroy(c)
        checkpoint()

    # configs[0]/[3]/[4] with full parity on the reported engine come right after the headline engines
    if not a.no_variants:
        configs_on(best_kind)

    # comparison timings for tuning (not the reported value), each while the budget lasts: the same call
    # with grouped ncclSend/ncclRecv exchanges or skewed slots, RCCL's own ncclAllReduce through torch
    # (ring order: not order-faithful at P >= 3), one link's rate
    if not a.no_variants and rcomm is not None:
        # (the 64 / 32 MiB chunk pipelines are engines of their own above). MPJX_SLOT_SKEW is read per call
        # (the kept communicator); MPJX_RCCL_P2P and MPJX_RCCL_NATIVE at init (a communicator of their own).
        # rccl_native = RCCL's own reduction kernel through libmpjx (one ncclAllReduce, bit-exact for
        # SUM(DOUBLE) at P <= 2): the transport ceiling beside the reported HIP-combine engine, never it.
        cmp = (("rccl_p2p", {"MPJX_RCCL_P2P": "1"}, True), ("rccl_skew", {"MPJX_SLOT_SKEW": "4096"}, False),
               ("rccl_native", {"MPJX_RCCL_NATIVE": "1"}, True))
        for name, env, own in cmp:
            if name not in rccl_variants or not budget.allow(f"variant:{name}"):
                continue
            with budget.phase(f"variant:{name}"), Watchdog(f"variant:{name}"), env_set(env):
                vc = None
                try:
                    vc = make_comm("rccl") if own else rcomm

                    def vstep(vc=vc):
                        _lib.check(L.mpjx_allreduce(vc, send.data_ptr(), recv.data_ptr(), n, MPJX_DOUBLE, MPJX_SUM,
                                                    0, None), "mpjx_allreduce")
                    recv.zero_()
                    torch.cuda.synchronize()
                    tv = timed(vstep, max(3, a.steps // 2), 2, vc)
                    vb, vf = parity()
                    variants[name] = {"ms": round(tv * 1e3, 4),
                                      "busbw_GBps": round(S / tv / 1e9 * 2 * (world - 1) / world, 2),
                                      "mismatches": vb, "full_checksum_match": vf,
                                      "bit_exact": vb == 0 and vf is True, "env": env}
                    if name == "rccl_native":
                        variants[name]["phases"] = phases(vc)
                        variants[name]["note"] = ("RCCL's own reduction kernel (ncclAllReduce through libmpjx, "
                                                  "MPJX_RCCL_NATIVE=1): the transport ceiling, not libmpjx's "
                                                  "HIP combine; never the reported value")
                except Exception as e:  # noqa: BLE001
                    variants[name] = {"error": str(e)[:200]}
                finally:
                    if own and vc is not None:
                        L.mpjx_comm_destroy(vc)
        if budget.allow("variant:rccl_native_allreduce"):
            with budget.phase("variant:rccl_native_allreduce"), Watchdog("variant:rccl_native_allreduce"):
                try:
                    g = dist.new_group(backend="nccl")
                    ref = send.clone()

                    def rstep():
                        dist.all_reduce(ref, group=g)

                    tv = timed(rstep, max(3, a.steps // 2), 2, rcomm)
                    variants["rccl_native_allreduce"] = {
                        "ms": round(tv * 1e3, 4), "busbw_GBps": round(S / tv / 1e9 * 2 * (world - 1) / world, 2),
                        "note": "torch RCCL all_reduce, ring order: not bit-exact vs the reference at P >= 3"}
                    del ref
                except Exception as e:  # noqa: BLE001
                    variants["rccl_native_allreduce"] = {"error": str(e)[:200]}
        if world >= 2 and budget.allow("variant:p2p_one_link"):
            with budget.phase("variant:p2p_one_link"), Watchdog("variant:p2p_one_link"):
                try:  # one xGMI link, measured: rank 0 -> rank 1, 256 MiB (SURVEY 8d "measured per-link figure")
                    g2 = dist.new_group(backend="nccl")
                    buf = send.clone()

                    def pstep():
                        if rank == 0:
                            dist.send(buf, dst=1, group=g2)
                        elif rank == 1:
                            dist.recv(buf, src=0, group=g2)

                    tv = timed(pstep, max(3, a.steps // 2), 2, rcomm)
                    variants["p2p_one_link"] = {"ms": round(tv * 1e3, 4), "GBps": round(S / tv / 1e9, 2)}
                    del buf
                except Exception as e:  # noqa: BLE001
                    variants["p2p_one_link"] = {"error": str(e)[:200]}
        checkpoint()
    if not a.no_variants and budget.allow("e2e_host"):
        # north_star's host-to-host rate at N ranks: Java-heap-like pageable host arrays in and out of
        # mpjx_allreduce_host (H2D / collective / D2H chunk-pipelined), checked like the headline. On the
        # kept RCCL communicator, else (one-device rehearsals, RCCL refused) a world of the reported engine
        with budget.phase("e2e_host"), Watchdog("e2e_host"):
            ecomm, eown = rcomm, False
            where = ("the RCCL engine" if rcomm is not None else f"the {best_kind} engine") + (
                f" ({world} rank processes sharing one GPU and its one host link)" if a.one_device else "")
            try:
                if ecomm is None:
                    ecomm, eown = make_comm(best_kind), True
                hsend = synth.uniform_np(np.arange(n, dtype=np.uint64), seed(3, rank))
                hrecv = np.zeros_like(hsend)

                def hstep():
                    _lib.check(L.mpjx_allreduce_host(ecomm, hsend.ctypes.data, hrecv.ctypes.data, n, MPJX_DOUBLE,
                                                     MPJX_SUM, 0), "mpjx_allreduce_host")

                tv = timed(hstep, 3, 1, ecomm)
                hexp = mst_sum([synth.uniform_np(idx, seed(3, r)) for r in range(world)], 0, world - 1, 0)
                hbad = int(np.count_nonzero(hrecv[idx].view(np.uint64) != hexp.view(np.uint64)))
                cks = [None] * world
                dist.all_gather_object(cks, checksum(hrecv))
                hfull = [None]
                if rank == 0:
                    hfull[0] = all(tuple(c_) == expected_checksum() for c_ in cks)
                dist.broadcast_object_list(hfull, src=0)
                variants["e2e_host_256MiB"] = {
                    "ms": round(tv * 1e3, 4), "algbw_GBps_per_rank": round(S / tv / 1e9, 2),
                    "bit_exact": all_ok(hbad == 0) and hfull[0] is True,
                    "note": f"pageable host send/recv, mpjx_allreduce_host on {where} (PCIe-bound)"}
                # the same with page-locked host arrays (north_star's pinned host<->device copies): DMA
                # straight from and to the caller's memory
                psend = torch.from_numpy(hsend).pin_memory()
                precv = torch.zeros(n, dtype=torch.float64).pin_memory()
                del hsend, hrecv

                def pstep():
                    _lib.check(L.mpjx_allreduce_host(ecomm, psend.data_ptr(), precv.data_ptr(), n, MPJX_DOUBLE,
                                                     MPJX_SUM, 0), "mpjx_allreduce_host")

                tv = timed(pstep, 3, 1, ecomm)
                prv = precv.numpy()
                pbad = int(np.count_nonzero(prv[idx].view(np.uint64) != hexp.view(np.uint64)))
                cks = [None] * world
                dist.all_gather_object(cks, checksum(prv))
                pfull = [None]
                if rank == 0:
                    pfull[0] = all(tuple(c_) == expected_checksum() for c_ in cks)
                dist.broadcast_object_list(pfull, src=0)
                variants["e2e_host_pinned_256MiB"] = {
                    "ms": round(tv * 1e3, 4), "algbw_GBps_per_rank": round(S / tv / 1e9, 2),
                    "bit_exact": all_ok(pbad == 0) and pfull[0] is True,
                    "note": f"page-locked host send/recv, mpjx_allreduce_host on {where} (PCIe-bound)"}
                del psend, precv, prv
            except Exception as e:  # noqa: BLE001
                key = "e2e_host_pinned_256MiB" if "e2e_host_256MiB" in variants else "e2e_host_256MiB"
                variants[key] = {"error": str(e)[:200]}
            finally:
                if eown and ecomm is not None:
                    L.mpjx_comm_destroy(ecomm)
        checkpoint()
    # the same configs on the RCCL engine when an IPC engine was reported (keys prefixed "rccl:")
    if (not a.no_variants and best_kind != "rccl" and rcomm is not None
            and budget.allow("rccl:other_configs")):
        configs_on("rccl")
    # per GPU: rank 0's device alone (one-device rehearsals share it); the decision is collective
    if not a.no_variants and budget.allow("hbm_combine") and rank == 0:
        with budget.phase("hbm_combine"), Watchdog("hbm_combine"):
            try:  # the reported engine's combine shape: pipeline-chunk blocks (RCCL) or whole blocks (IPC)
                pc = int(engine_env(best).get("MPJX_PIPE_CHUNK_MIB", os.environ.get("MPJX_PIPE_CHUNK_MIB", "0"))) << 20
                piped = best.startswith("rccl") and pc > 0 and S > pc
                skew = 4096 if best.startswith("ipc") else 0  # the engine's input-slot layout
                hbm["v"] = combine_roofline(L, world, (pc if piped else S) // world // 8, dev, a.steps, skew)
            except Exception as e:  # noqa: BLE001
                hbm["v"] = {"error": str(e)[:200]}
    if rank == 0:
        emit(snapshot())
    if hl is not None:
        hl.cancel()  # the line is out: the hard limit must not fire during teardown (TEARDOWN_S bounds it)
    # the line is out: a teardown that hangs (an RCCL communicator's destroy, the process group) must not
    # hold the run — every rank leaves after TEARDOWN_S whatever it is waiting on
    td = threading.Timer(TEARDOWN_S, lambda: (sys.stdout.flush(), os._exit(0)))
    td.daemon = True
    td.start()
    if rcomm is not None:
        L.mpjx_comm_destroy(rcomm)
    dist.destroy_process_group()


def phase_breakdown(L, c, dist, call):
    """One extra collective (`call`) with libmpjx's phase events on (mpjx_comm_phase_timing): where a
    call's time goes, per rank — exchange #1 / combine / exchange #2 (exchange engine), share / combine
    / fence (direct engine), all-gather / combine (one-shot) — reported as the max over ranks of each
    phase. Collective over the ranks of `dist`."""
    from mpjexpress_amd import _lib

    try:
        _lib.check(L.mpjx_comm_phase_timing(c, 1), "phase_timing")
        dist.barrier()
        call()
        ms = (ctypes.c_float * 3)()
        eng = ctypes.c_int()
        _lib.check(L.mpjx_comm_last_phases(c, ms, ctypes.byref(eng)), "last_phases")
        _lib.check(L.mpjx_comm_phase_timing(c, 0), "phase_timing")
        _lib.check(L.mpjx_comm_synchronize(c), "sync")
        mine = torch.tensor(list(ms), dtype=torch.float64)
        dist.all_reduce(mine, op=dist.ReduceOp.MAX)
        names = {1: ["exchange1", "combine", "exchange2"], 2: ["share", "combine", "fence"],
                 3: ["whole_call_pipelined", "-", "-"], 4: ["-", "copy", "-"],
                 5: ["allgather", "combine", "-"], 6: ["-", "nccl_allreduce", "-"]}.get(eng.value, ["?", "?", "?"])
        out_ = {nm: round(v, 4) for nm, v in zip(names, mine.tolist()) if nm != "-"}
        out_["engine_kind"] = {1: "exchange", 2: "direct", 3: "pipelined", 4: "one rank (copy)",
                               5: "one-shot", 6: "rccl native (ncclAllReduce)"}.get(eng.value, "?")
        out_["note"] = "ms, max over ranks, one instrumented call after the timed ones"
        return out_
    except Exception as e:  # noqa: BLE001
        try:
            L.mpjx_comm_phase_timing(c, 0)
        except Exception:  # noqa: BLE001
            pass
        return {"error": str(e)[:200]}


def xgmi_roofline(link_bytes_per_rank, t, world, one_device):
    """Link utilisation of one call: the bytes every rank must send over its P-1 xGMI links (the plan's
    algorithmic link traffic) / t, against (P-1) links of XGMI_LINK_GBPS each."""
    if world < 2 or one_device:
        return {"bound": "xgmi", "achieved": None, "peak": None, "unit": "GB/s", "frac": None,
                "note": "no xGMI links at world size 1 / all ranks on one GPU"}
    ach = link_bytes_per_rank / t / 1e9
    peak = (world - 1) * XGMI_LINK_GBPS
    return {"bound": "xgmi", "achieved": round(ach, 2), "peak": round(peak, 1), "unit": "GB/s",
            "frac": round(ach / peak, 4), "link_bytes_per_rank": int(link_bytes_per_rank)}


def c4_inputs(n4, rank, dev):
    """configs[3] inputs: BAND words with each bit set with p = 7/8 (the OR of three
    splitmix64 streams, so an 8-rank AND is not all zeros) and uniform BXOR words; int32 = the low
    32 bits of each 64-bit stream element (a bit view, no value conversion)."""
    def low32(s):
        return synth.bits_torch(n4, s, dev).view(torch.int32)[0::2].contiguous()

    b = seed(4, rank)
    band = low32(b) | low32(b + 0x100) | low32(b + 0x200)
    return band, low32(b + 0x300)


def _mismatch(got, exp):
    """(number of differing elements, first differing index or None), compared bit for bit."""
    g = got.reshape(-1).view(torch.int32) if got.element_size() == 4 else got.reshape(-1)
    e = exp.reshape(-1).view(torch.int32) if exp.element_size() == 4 else exp.reshape(-1)
    bad = (g != e)
    nb = int(bad.sum().item())
    return nb, (int(bad.nonzero()[0].item()) if nb else None)


def c5_input(n5, rank, dev):
    """configs[4] input: U[-1e3, 1e3) floats (the double stream rounded to float, RNE)."""
    return synth.uniform_torch(n5, seed(5, rank), dev, -1e3, 1e3).to(torch.float32)


def other_configs(L, comm, sp, world, rank, dev, timed, steps, check, pipe_variant=False, dist=None,
                  one_device=False):
    """configs[3] (Reduce_scatter BAND + Scan BXOR, int32 64 MiB per rank) and configs[4]
    (Allreduce MAX float 1 GiB per rank) at this world size, timed like the headline and then checked
    in FULL on every rank: each rank regenerates every rank's input stream on its own device and
    recomputes its expected result with torch bitwise / maximum ops (AND, XOR and a NaN-free MAX are
    order-free, so any order gives the reference's bits), independently of libmpjx. check(ok) returns
    True only if every rank's result matched (a collective). Each entry also carries its xGMI roofline
    (the plan's link bytes per rank / t against (P-1) links) and, with `dist`, a phase breakdown.
    Link bytes per rank: Reduce_scatter (P-1)/P·S (exchange #1 only); Scan 2(P-1)/P·S
    (exchange #1 + every rank's prefix block back) — the alternative chain r -> r+1 of SURVEY §8(e)
    moves S over ONE link per rank, (P/2)x the per-link time of this plan at P >= 3."""
    from mpjexpress_amd import _lib

    def ph(fn):
        if dist is None:
            return None
        _lib.check(L.mpjx_comm_synchronize(comm), "sync")
        torch.cuda.synchronize()
        return phase_breakdown(L, comm, dist, fn)

    out = {}
    # configs[0] (C1): Allreduce SUM double, 1 MiB per rank — latency-bound, the reference's own CPU case
    # (cpu_baseline.allreduce_mst.configs0_1MiB_p4 at P = 4). Every element of every rank's result checked
    # bit for bit against the MST(0) grouping recomputed on the host.
    n1 = (1 << 20) // 8
    x1 = synth.uniform_torch(n1, seed(1, rank), dev)
    r1 = torch.empty_like(x1)
    torch.cuda.synchronize()
    k1 = max(50, 5 * steps)
    t = timed(lambda: _lib.check(L.mpjx_allreduce(comm, x1.data_ptr(), r1.data_ptr(), n1, MPJX_DOUBLE, MPJX_SUM, 0,
                                                  sp), "mpjx_allreduce"), k1, 5)
    _lib.check(L.mpjx_comm_synchronize(comm), "sync")
    torch.cuda.synchronize()
    full1 = np.arange(n1, dtype=np.uint64)
    e1 = mst_sum([synth.uniform_np(full1, seed(1, r)) for r in range(world)], 0, world - 1, 0)
    got1 = r1.cpu().numpy()
    nb = int(np.count_nonzero(got1.view(np.uint64) != e1.view(np.uint64)))
    ok = check(nb == 0)
    out["c0_allreduce_sum_double_1MiB"] = {
        "us_per_call": round(t * 1e6, 2), "calls": k1, "algbw_GBps_per_rank": round(n1 * 8 / t / 1e9, 3),
        "bit_exact": ok, "elements_checked_per_rank": n1, "rank0_mismatches": nb,
        "note": "configs[0]'s vector (1 MiB double SUM) at this world size; the reference's pure-Java MST at "
                "P = 4 on the host is cpu_baseline.allreduce_mst.configs0_1MiB_p4 (N = 1 line)"}
    del x1, r1
    k = max(3, steps // 4)
    n4 = (64 << 20) // 4
    blk = n4 // world
    band, bxor = c4_inputs(n4, rank, dev)
    y = torch.empty(blk, dtype=torch.int32, device=dev)
    z = torch.empty_like(bxor)
    rc = (ctypes.c_int64 * world)(*([blk] * world))
    # The library runs on the communicator's stream, torch on its own: before any buffer made by torch is
    # handed over, torch's stream must be idle — the inputs must be written, and an output block the
    # caching allocator just recycled from a temporary must no longer be read by torch's pending kernels
    # (without this sync the first checks caught a corrupted input: the library's store into `y` landed
    # in a freed temporary that torch's last OR kernel was still reading)
    torch.cuda.synchronize()
    t = timed(lambda: _lib.check(L.mpjx_reduce_scatter(comm, band.data_ptr(), y.data_ptr(), rc, MPJX_INT, MPJX_BAND,
                                                         0, sp), "mpjx_reduce_scatter"), k, 1)
    exp = None
    for r in range(world):
        b_r = c4_inputs(n4, r, dev)[0][rank * blk:(rank + 1) * blk]
        exp = b_r if exp is None else exp & b_r
    _lib.check(L.mpjx_comm_synchronize(comm), "sync")
    torch.cuda.synchronize()
    nb, first = _mismatch(y, exp)
    ok = check(nb == 0)
    out["c4_reduce_scatter_band_int32_64MiB"] = {
        "ms": round(t * 1e3, 4), "busbw_GBps": round((world - 1) / world * n4 * 4 / t / 1e9, 2),
        "bit_exact": ok, "elements_checked_per_rank": blk, "rank0_mismatches_first": [nb, first],
        "roofline": xgmi_roofline((world - 1) / world * n4 * 4, t, world, one_device),
        "phases": ph(lambda: _lib.check(L.mpjx_reduce_scatter(comm, band.data_ptr(), y.data_ptr(), rc, MPJX_INT,
                                                              MPJX_BAND, 0, sp), "mpjx_reduce_scatter"))}
    del y, exp
    t = timed(lambda: _lib.check(L.mpjx_scan(comm, bxor.data_ptr(), z.data_ptr(), n4, MPJX_INT, MPJX_BXOR, 0, sp),
                                 "mpjx_scan"), k, 1)
    exp = None
    for r in range(rank + 1):
        x_r = c4_inputs(n4, r, dev)[1]
        exp = x_r if exp is None else exp ^ x_r
    _lib.check(L.mpjx_comm_synchronize(comm), "sync")
    torch.cuda.synchronize()
    nb, first = _mismatch(z, exp)
    ok = check(nb == 0)
    out["c4_scan_bxor_int32_64MiB"] = {
        "ms": round(t * 1e3, 4), "algbw_GBps": round(n4 * 4 / t / 1e9, 2),
        "busbw_GBps": round(2 * (world - 1) / world * n4 * 4 / t / 1e9, 2),
        "bit_exact": ok, "elements_checked_per_rank": n4, "rank0_mismatches_first": [nb, first],
        "roofline": xgmi_roofline(2 * (world - 1) / world * n4 * 4, t, world, one_device),
        "plan": "all-to-all -> K_SCAN (P outputs) -> every rank's prefix block back: 2(P-1)/P*S per rank over P-1 "
                "links (a chain r -> r+1 would move S over one link)",
        "survey_chain_roofline": ({"busbw_scan_GBps": round(n4 * 4 / t / 1e9, 2), "peak": XGMI_LINK_GBPS,
                                   "frac": round(n4 * 4 / t / 1e9 / XGMI_LINK_GBPS, 4),
                                   "note": "SURVEY 8(d): S/t against one link, the chain plan's bound; the "
                                           "all-to-all plan can exceed 1 here"}
                                  if world > 1 and not one_device else None),
        "phases": ph(lambda: _lib.check(L.mpjx_scan(comm, bxor.data_ptr(), z.data_ptr(), n4, MPJX_INT, MPJX_BXOR, 0,
                                                    sp), "mpjx_scan"))}
    del band, bxor, z, exp
    n5 = (1 << 30) // 4
    f = c5_input(n5, rank, dev)
    g = torch.empty_like(f)
    torch.cuda.synchronize()  # see above: torch's stream idle before the library's stream uses f and g

    def c5_expected():
        e = None
        for r in range(world):
            x_r = c5_input(n5, r, dev)
            e = x_r if e is None else torch.maximum(e, x_r)
            del x_r
        return e

    t = timed(lambda: _lib.check(L.mpjx_allreduce(comm, f.data_ptr(), g.data_ptr(), n5, MPJX_FLOAT, MPJX_MAX, 0, sp),
                                 "mpjx_allreduce"), k, 1)
    _lib.check(L.mpjx_comm_synchronize(comm), "sync")
    e5 = c5_expected()
    torch.cuda.synchronize()
    nb, first = _mismatch(g, e5)
    ok = check(nb == 0)
    out["c5_allreduce_max_float_1GiB"] = {"ms": round(t * 1e3, 4),
                                          "busbw_GBps": round(2 * (world - 1) / world * n5 * 4 / t / 1e9, 2),
                                          "bit_exact": ok, "elements_checked_per_rank": n5,
                                          "rank0_mismatches_first": [nb, first],
                                          "roofline": xgmi_roofline(2 * (world - 1) / world * n5 * 4, t, world,
                                                                    one_device)}
    if pipe_variant:  # configs[4] names the chunk pipeline: the same call with 64 MiB chunks
        prev = os.environ.get("MPJX_PIPE_CHUNK_MIB")
        os.environ["MPJX_PIPE_CHUNK_MIB"] = "64"
        try:
            g.zero_()
            torch.cuda.synchronize()
            t = timed(lambda: _lib.check(L.mpjx_allreduce(comm, f.data_ptr(), g.data_ptr(), n5, MPJX_FLOAT, MPJX_MAX, 0,
                                                          sp), "mpjx_allreduce"), k, 1)
        finally:
            if prev is None:
                os.environ.pop("MPJX_PIPE_CHUNK_MIB", None)
            else:
                os.environ["MPJX_PIPE_CHUNK_MIB"] = prev
        _lib.check(L.mpjx_comm_synchronize(comm), "sync")
        torch.cuda.synchronize()
        nb, first = _mismatch(g, e5)
        ok = check(nb == 0)
        out["c5_allreduce_max_float_1GiB_pipelined_64MiB"] = {
            "ms": round(t * 1e3, 4), "busbw_GBps": round(2 * (world - 1) / world * n5 * 4 / t / 1e9, 2),
            "bit_exact": ok, "elements_checked_per_rank": n5, "rank0_mismatches_first": [nb, first],
            "roofline": xgmi_roofline(2 * (world - 1) / world * n5 * 4, t, world, one_device)}
    del f, g, e5
    return out


def combine_roofline(L, P, slice_elems, dev, steps, skew=0):
    """The P-way combine kernel of the N > 1 Allreduce at the shape AND layout it runs in the reported
    engine (K_MST over P slices of slice_elems doubles, MST root 0: PureIntracomm.java:1943-1992): the
    P input slots of one set live in ONE allocation at a stride of slice + skew bytes, as the engine
    places them (RCCL exchange #1: contiguous, skew 0, for one ncclAllToAll; IPC push staging: 4 KiB
    skew), the result in a buffer of its own. Timed alone with one HIP event pair on its launch stream
    around `steps` launches, cycling over enough independent sets that no launch finds its operands in
    the Infinity Cache (cold, as the N = 1 combine). Algorithmic bytes (P + 1) * slice (SURVEY §8d:
    (P+1)/P * S per rank per call); traffic from the committed PMC summary for this shape, or None."""
    import torch

    from mpjexpress_amd import _lib

    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    set_bytes = (P + 1) * slice_elems * 8
    R = max(2, -(-(1 << 30) // set_bytes))  # >= 1 GiB streamed between two uses of a set
    stride = slice_elems * 8 + skew
    ins = []
    for k in range(R):
        buf = torch.empty(P * stride // 8, dtype=torch.float64, device=dev)
        for p in range(P):
            buf[p * stride // 8:p * stride // 8 + slice_elems] = synth.uniform_torch(
                slice_elems, 0x4D504A00 + 7000 + 16 * k + p, dev)
        ins.append(buf)
    outs = [torch.empty(slice_elems, dtype=torch.float64, device=dev) for _ in range(R)]
    pin = [(ctypes.c_void_p * P)(*[ins[k].data_ptr() + p * stride for p in range(P)]) for k in range(R)]
    pout = [(ctypes.c_void_p * 1)(outs[k].data_ptr()) for k in range(R)]
    order = 1 if P >= 3 else 0  # MST for P >= 3; P = 2 is the two-operand fold

    def go(i):
        k = i % R
        _lib.check(L.mpjx_combine_multi(MPJX_SUM, MPJX_DOUBLE, order, P, pin[k], pout[k], slice_elems, 0, 0, sp),
                   "mpjx_combine_multi")

    torch.cuda.synchronize()  # inputs written, recycled blocks released before st uses them
    for i in range(max(3, R)):
        go(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for i in range(steps):
        go(i)
    e1.record(st)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / steps / 1e3
    alg = (P + 1) * slice_elems * 8
    mib = slice_elems * 8 >> 20
    tag = f"pway_{'mst' if order == 1 else 'fold'}_p{P}_f64_{mib}MiB" if P > 1 else f"copies_{mib}MiB"
    del ins, outs
    kname = f"k_pway<Sum<double>,{P},{'K_MST' if order == 1 else 'K_FOLD'}>" if P > 1 else "k_copies (P = 1)"
    return {"bound": "hbm", "kernel": kname, "slot_stride_bytes": stride, "slot_skew_bytes": skew,
            "slice_MiB": mib, "sets": R, "algorithmic_bytes_per_launch": alg, "kernel_us": round(t * 1e6, 2),
            "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4), "traffic": traffic_from_profiles(tag), "traffic_tag": tag}


def _lib_unique_id(L):
    buf = ctypes.create_string_buffer(128)
    from mpjexpress_amd import _lib

    _lib.check(L.mpjx_get_unique_id(buf), "mpjx_get_unique_id")
    return buf.raw


if __name__ == "__main__":
    main()
