"""TEST DIAGNOSTICS: a watchdog for the child-process test drivers (tests/jni_driver.py,
tests/rccl_standin_driver.py). After `seconds` it writes to stderr, for every thread of the process: its
name, the system call it is blocked in (/proc/self/task/<tid>/syscall: 202 futex, 16 ioctl, 7 poll,
230 clock_nanosleep) and wchan; each thread's native return addresses (tests/diag/libstackdump.so,
one thread at a time; `addr2line -f -C -e <lib> 0xOFFSET` resolves them against this tree's .so files);
then every thread's Python stack; then it ends the process (exit status 3), so a hang surfaces as a
failed test with the evidence instead of as the test runner's time limit. With exit_after=False it only
reports (once) and the process runs on: a stall report for worlds that may still finish."""
import ctypes
import faulthandler
import os
import signal
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError as e:
        return f"<{e.strerror}>"


def dump_and_exit(exit_after=True):
    err = sys.stderr
    me = threading.get_native_id()
    tids = sorted(int(t) for t in os.listdir("/proc/self/task"))
    err.write(f"=== watchdog: {len(tids)} threads\n")
    for t in tids:
        base = f"/proc/self/task/{t}"
        err.write(f"tid {t} [{_read(base + '/comm')}] syscall: {_read(base + '/syscall').split(' ')[0]} "
                  f"wchan: {_read(base + '/wchan')}\n")
    err.flush()
    so = os.path.join(HERE, "diag", "libstackdump.so")
    if os.path.exists(so):
        sd = ctypes.CDLL(so)
        if sd.sd_install(signal.SIGUSR2) == 0:
            for t in tids:
                if t != me:
                    sd.sd_signal(t, signal.SIGUSR2)
                    time.sleep(0.2)  # one thread's stack at a time on stderr
    err.write("=== maps of the libraries above (name: load address)\n")
    seen = set()
    for ln in _read("/proc/self/maps").splitlines():
        parts = ln.split()
        if len(parts) >= 6 and parts[5].endswith(".so") or (len(parts) >= 6 and ".so." in parts[5]):
            if parts[5] not in seen and parts[2] == "00000000":
                seen.add(parts[5])
                err.write(f"{parts[5]}: {parts[0].split('-')[0]}\n")
    err.flush()
    faulthandler.dump_traceback(file=err, all_threads=True)
    err.write("=== watchdog: end of report\n")
    err.flush()
    if exit_after:
        os._exit(3)


def arm(seconds, exit_after=True):
    """Start the watchdog (a daemon timer thread); returns it (cancel() when the run ends in time)."""
    tm = threading.Timer(float(seconds), dump_and_exit, kwargs={"exit_after": exit_after})
    tm.daemon = True
    tm.start()
    return tm
