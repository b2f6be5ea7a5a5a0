"""Tracing / profiling hooks.

The reference times things by hand: ``LogTimer`` around updater phases
(core/_private/log_timer.py, node_updater.py:164), per-step DT/XT/FT/BT/OT/TT prints in BERT
(run_pretrain_mlperf.py:~797) and ``AverageMeter`` in ResNet (main.py:481-586).  It has no
GPU tracing.  Here:

* ``range(name)`` / ``mark(name)``: ROCTX ranges (``libroctx64``) that ``rocprofv3
  --marker-trace`` shows next to the kernels; no-ops when ROCTX is absent or
  ``CLOUDTIK_ROCTX=0``.
* ``StepTimer``: per-phase wall times of a training step (data / forward / backward / comm /
  optimizer) measured with HIP events on the compute stream, so no phase boundary forces a
  host synchronisation; ``summary()`` syncs once and returns the means in ms.
* ``LogTimer``: the control plane's phase timer (logs "<name>: 1.234s").
* ``rocprof_command(argv, out_dir)``: the argv that runs a program under ``rocprofv3
  --kernel-trace --stats`` (used by ``cloudtik-run --profile``).  The program itself comes
  right after ``--`` (no env / shell hop: the profiler's preload initialises the GPU).
"""
from __future__ import annotations

import contextlib
import ctypes
import logging
import os
import shutil
import time
from typing import Dict, List, Optional

logger = logging.getLogger(__name__)

_ROCTX = None
_ROCTX_TRIED = False


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if _ROCTX_TRIED:
        return _ROCTX
    _ROCTX_TRIED = True
    if os.environ.get("CLOUDTIK_ROCTX", "1") == "0":
        return None
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in ("libroctx64.so", "libroctx64.so.4", os.path.join(rocm, "lib", "libroctx64.so")):
        try:
            lib = ctypes.CDLL(name)
        except OSError:
            continue
        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
        lib.roctxRangePushA.restype = ctypes.c_int
        lib.roctxRangePop.restype = ctypes.c_int
        lib.roctxMarkA.argtypes = [ctypes.c_char_p]
        _ROCTX = lib
        break
    return _ROCTX


def roctx_available() -> bool:
    return _roctx() is not None


def push(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop() -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx / nvtx naming
    push(name)
    try:
        yield
    finally:
        pop()


class StepTimer:
    """Per-phase step timing with device events.

        t = StepTimer()
        with t.phase("forward"): ...
        with t.phase("backward"): ...
        t.step_done()
        t.summary()  -> {"forward": ms, "backward": ms, ..., "step": ms}

    On CPU it falls back to ``perf_counter``.  Each phase is also a ROCTX range."""

    def __init__(self, device=None, enabled: bool = True):
        import torch
        self.enabled = enabled
        self.gpu = torch.cuda.is_available() and (device is None or getattr(device, "type", device) != "cpu")
        self._events: List[List[tuple]] = [[]]
        self._totals: Dict[str, float] = {}
        self._counts: Dict[str, int] = {}
        self._step_t0 = None

    def _stamp(self):
        if self.gpu:
            import torch
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        push(name)
        a = self._stamp()
        try:
            yield
        finally:
            b = self._stamp()
            pop()
            self._events[-1].append((name, a, b))

    def step_done(self):
        if self.enabled:
            self._events.append([])

    def _drain(self):
        if self.gpu:
            import torch
            torch.cuda.synchronize()
        for step in self._events:
            if not step:
                continue
            tot = 0.0
            for name, a, b in step:
                ms = a.elapsed_time(b) if self.gpu else (b - a) * 1000.0
                self._totals[name] = self._totals.get(name, 0.0) + ms
                self._counts[name] = self._counts.get(name, 0) + 1
                tot += ms
            self._totals["step"] = self._totals.get("step", 0.0) + tot
            self._counts["step"] = self._counts.get("step", 0) + 1
        self._events = [[]]

    def summary(self) -> Dict[str, float]:
        self._drain()
        return {k: self._totals[k] / self._counts[k] for k in self._totals}

    def format(self) -> str:
        s = self.summary()
        return " ".join(f"{k}={v:.2f}ms" for k, v in s.items())


class LogTimer:
    """``with LogTimer("NodeUpdater: setup"):`` logs the elapsed seconds at exit
    (reference core/_private/log_timer.py)."""

    def __init__(self, message: str, show_status: bool = False, log=None):
        self.message = message
        self.show_status = show_status
        self.log = log or logger.info
        self.elapsed = 0.0

    def __enter__(self):
        self._t0 = time.time()
        push(self.message)
        return self

    def __exit__(self, exc_type, *_):
        pop()
        self.elapsed = time.time() - self._t0
        status = ""
        if self.show_status:
            status = " [failed]" if exc_type else " [succeeded]"
        self.log("%s: %.3fs%s", self.message, self.elapsed, status)
        return False


def rocprof_binary() -> Optional[str]:
    p = shutil.which("rocprofv3")
    if p:
        return p
    cand = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "rocprofv3")
    return cand if os.path.exists(cand) else None


def rocprof_command(argv: List[str], out_dir: str, stats: bool = True, markers: bool = False,
                    pmc: Optional[List[str]] = None) -> List[str]:
    """``rocprofv3 [--kernel-trace --stats | --pmc ...] -d out_dir -- <argv>``.

    Counter collection (``pmc``) is kept in its own run with kernel tracing only; it is
    never combined with the runtime/marker trace domains."""
    rp = rocprof_binary() or "rocprofv3"
    cmd = [rp]
    if pmc:
        cmd += ["--pmc", *pmc, "--kernel-trace"]
    else:
        cmd += ["--kernel-trace"]
        if stats:
            cmd += ["--stats"]
        if markers:
            cmd += ["--marker-trace"]
    cmd += ["-d", out_dir, "-o", "trace", "--output-format", "csv", "--"]
    return cmd + list(argv)
