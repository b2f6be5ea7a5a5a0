"""Fault injection for the training runtime.

The reference only injects faults inside its unit tests (``MockProcessRunner(fail_cmds=…)``,
test_cloudtik.py:91-125).  Here a running job can be told to fail, so the launcher's
terminate-all / ``--max-restarts`` / checkpoint auto-resume path is exercised end to end:

    CLOUDTIK_INJECT_FAIL_RANK=1 CLOUDTIK_INJECT_FAIL_STEP=5 cloudtik-run --max-restarts 1 train.py

* ``CLOUDTIK_INJECT_FAIL_RANK``   rank that fails (``*`` = every rank; default: none)
* ``CLOUDTIK_INJECT_FAIL_STEP``   global step at which it fails
* ``CLOUDTIK_INJECT_FAIL_MODE``   ``exit`` (os._exit(code), default), ``raise``
  (``InjectedFault``) or ``signal`` (SIGKILL to itself, like an OOM kill)
* ``CLOUDTIK_INJECT_FAIL_CODE``   exit code for ``exit`` (default 17)
* ``CLOUDTIK_INJECT_FAIL_ATTEMPTS`` inject only while ``CLOUDTIK_RESTART_COUNT`` (set by
  cloudtik-run) is below this (default 1: the first attempt fails, the restart succeeds).
"""
from __future__ import annotations

import os
import signal
import sys


class InjectedFault(RuntimeError):
    pass


def _rank() -> int:
    for n in ("RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "HOROVOD_RANK"):
        v = os.environ.get(n)
        if v not in (None, ""):
            return int(v)
    return 0


def restart_count() -> int:
    return int(os.environ.get("CLOUDTIK_RESTART_COUNT", "0") or 0)


def armed() -> bool:
    return bool(os.environ.get("CLOUDTIK_INJECT_FAIL_STEP"))


def maybe_fail(step: int, rank: int = None) -> None:
    """Call once per training step; fails this process if the injection matches."""
    at = os.environ.get("CLOUDTIK_INJECT_FAIL_STEP")
    if not at or int(at) != int(step):
        return
    who = os.environ.get("CLOUDTIK_INJECT_FAIL_RANK", "")
    r = _rank() if rank is None else rank
    if who != "*" and (who == "" or int(who) != r):
        return
    if restart_count() >= int(os.environ.get("CLOUDTIK_INJECT_FAIL_ATTEMPTS", "1")):
        return
    mode = os.environ.get("CLOUDTIK_INJECT_FAIL_MODE", "exit")
    msg = f"[cloudtik] injected fault: rank {r} step {step} mode {mode} (attempt {restart_count()})"
    print(msg, file=sys.stderr, flush=True)
    if mode == "raise":
        raise InjectedFault(msg)
    if mode == "signal":
        os.kill(os.getpid(), signal.SIGKILL)
    os._exit(int(os.environ.get("CLOUDTIK_INJECT_FAIL_CODE", "17")))
