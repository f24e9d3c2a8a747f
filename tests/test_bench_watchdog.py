"""bench.py's hand-off watchdog (N > 1): a hung multi-rank hand-off leg must not cost the driver
the weak-scaling line.  CPU only: the watchdog fires in a child process, which must write the line
measured so far with the hand-off error and exit 0 at once."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_watchdog_writes_the_line_and_ends_the_process():
    code = ("import os, sys, time; sys.path.insert(0, %r); import bench; "
            "bench._JSON_FD = os.dup(1); os.dup2(2, 1); "
            "bench._HandoffWatchdog({'metric': 'm', 'value': 1.5}, 0, 0.5); time.sleep(60)") % ROOT
    t0 = time.time()
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0
    assert time.time() - t0 < 50
    line = json.loads(res.stdout.strip().splitlines()[-1])
    assert line["value"] == 1.5 and "watchdog" in line["handoff"]["error"]


def test_cancelled_watchdog_stays_silent():
    code = ("import os, sys, time; sys.path.insert(0, %r); import bench; bench._JSON_FD = os.dup(1); "
            "d = bench._HandoffWatchdog({'metric': 'm'}, 0, 0.5); d.cancel(); time.sleep(1.0); print('done')") % ROOT
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0 and res.stdout.strip() == "done"
