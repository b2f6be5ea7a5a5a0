"""Process reaper (reference core/_private/service/cloudtik_process_reaper.py): make sure the
children of a launcher die with it, even if the launcher is SIGKILLed.

Orphaned training ranks would keep holding their MI355X (HBM, RCCL communicators) after a
crashed ``cloudtik-run``.  The launcher starts one reaper with a pipe on its stdin and writes
one line per child process-group id; the reaper blocks on that pipe.  EOF without a final
``done`` line means the launcher died: the reaper SIGTERMs the recorded process groups,
waits a grace period and SIGKILLs what is left.  Only the exact recorded groups are
signalled.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from typing import List, Optional

GRACE_S = 2.0


def _alive(pgid: int) -> bool:
    try:
        os.killpg(pgid, 0)
        return True
    except (ProcessLookupError, PermissionError):
        return False


def reap(pgids: List[int], grace: float = GRACE_S):
    for g in pgids:
        try:
            os.killpg(g, signal.SIGTERM)
        except (ProcessLookupError, PermissionError):
            pass
    end = time.time() + grace
    while time.time() < end and any(_alive(g) for g in pgids):
        time.sleep(0.05)
    for g in pgids:
        try:
            os.killpg(g, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            pass


def main():
    signal.signal(signal.SIGINT, signal.SIG_IGN)     # only the pipe decides
    pgids: List[int] = []
    done = False
    for line in sys.stdin:
        line = line.strip()
        if line == "done":
            done = True
            break
        if line.isdigit():
            pgids.append(int(line))
    if not done:
        reap(pgids)


class Reaper:
    """Launcher-side handle."""

    def __init__(self):
        self.proc: Optional[subprocess.Popen] = subprocess.Popen(
            [sys.executable, "-m", "cloudtik_amd.core.node.reaper"], stdin=subprocess.PIPE, text=True,
            start_new_session=True, env=dict(os.environ, PYTHONPATH=os.pathsep.join(sys.path)))

    def watch(self, pgid: int):
        if self.proc and self.proc.stdin:
            self.proc.stdin.write(f"{pgid}\n")
            self.proc.stdin.flush()

    def release(self):
        """Normal shutdown: the children are handled by the launcher itself."""
        if self.proc and self.proc.stdin:
            try:
                self.proc.stdin.write("done\n")
                self.proc.stdin.close()
            except (BrokenPipeError, OSError):
                pass
            self.proc.wait(timeout=10)
        self.proc = None


if __name__ == "__main__":
    main()
