"""CPU: the child-process test drivers' watchdog (tests/watchdog.py, test diagnostics): in exit mode a hung
process reports every thread (blocking system call, native return addresses from tests/diag/libstackdump.so,
Python stack) and ends with status 3; in report-only mode it reports once and the process runs on."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

HUNG = r'''
import sys, threading, time
sys.path.insert(0, {here!r})
import watchdog
watchdog.arm(0.5, exit_after={exit_after})
ev = threading.Event()
threading.Thread(target=ev.wait, name="stuck", daemon=True).start()
time.sleep({sleep})
print("ran on", flush=True)
'''


def _run(exit_after, sleep):
    code = HUNG.format(here=HERE, exit_after=exit_after, sleep=sleep)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)


@pytest.mark.skipif(not os.path.exists(os.path.join(HERE, "diag", "libstackdump.so")),
                    reason="tests/diag/libstackdump.so not built (make -C mpjexpress_amd tests)")
def test_watchdog_exit_mode_reports_every_thread_and_exits_3():
    r = _run(True, 20)
    assert r.returncode == 3 and "ran on" not in r.stdout, (r.returncode, r.stdout)
    err = r.stderr
    assert "=== watchdog:" in err and "syscall: 202" in err  # the stuck thread waits in a futex
    assert err.count("--- native stack of tid") >= 2 and "libstackdump.so" in err
    assert "File " in err and "end of report" in err  # the Python stacks


def test_watchdog_report_only_mode_runs_on():
    r = _run(False, 3)
    assert r.returncode == 0 and "ran on" in r.stdout, (r.returncode, r.stdout, r.stderr[-500:])
    assert r.stderr.count("=== watchdog:") >= 1
