"""Communicator watchdog (``csrc/rccl.cpp``, ``parallel/comm.py Watchdog``): the native RCCL
collectives bypass c10d's watchdog, so a step that never completes (a peer that stopped taking
part) must be turned into a loud failure within the deadline instead of a silent hang.
The hang is simulated with a bounded busy kernel (``lwaaai.selftest_spin``, at most a few seconds:
the grid always drains)."""
import os
import subprocess
import sys
import textwrap
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_deadline_fires_on_a_stuck_step():
    from layer_wise_aaai20_amd.ops._ext import load
    from layer_wise_aaai20_amd.parallel.comm import Watchdog
    lib = load()
    x = torch.zeros(1, device="cuda")
    wd = Watchdog(0, "cuda:0", timeout_s=0.5, action=1)
    try:
        lib.selftest_spin(x, 2500.0)               # the "collective" that never returns
        wd.mark()
        t0 = time.time()
        while not wd.status() and time.time() - t0 < 2.0:
            time.sleep(0.05)
        assert "not complete" in wd.status(), wd.status()
        assert time.time() - t0 < 2.0
        with pytest.raises(RuntimeError, match="watchdog"):
            wd.check()
    finally:
        torch.cuda.synchronize()
        wd.close()


def test_no_false_alarm_on_healthy_steps():
    from layer_wise_aaai20_amd.ops._ext import load
    from layer_wise_aaai20_amd.parallel.comm import Watchdog
    lib = load()
    x = torch.zeros(1, device="cuda")
    wd = Watchdog(0, "cuda:0", timeout_s=1.0, action=1)
    try:
        for _ in range(5):
            lib.selftest_spin(x, 100.0)
            wd.mark()
            torch.cuda.synchronize()
        time.sleep(1.5)
        wd.check()
    finally:
        wd.close()


def test_abort_action_exits_nonzero():
    """Training mode: abort + exit code 86 within the deadline (never a hang)."""
    script = textwrap.dedent("""
        import sys, time, torch
        sys.path.insert(0, %r)
        from layer_wise_aaai20_amd.ops._ext import load
        from layer_wise_aaai20_amd.parallel.comm import Watchdog
        lib = load()
        x = torch.zeros(1, device="cuda")
        wd = Watchdog(0, "cuda:0", timeout_s=0.5, action=0)
        lib.selftest_spin(x, 2500.0)
        wd.mark()
        print("waiting", flush=True)
        time.sleep(20)
        print("not reached", flush=True)
    """ % ROOT)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=60)
    assert r.returncode == 86, (r.returncode, r.stdout[-1000:], r.stderr[-2000:])
    assert "not reached" not in r.stdout
    assert "communicator watchdog" in r.stderr
    assert time.time() - t0 < 20
