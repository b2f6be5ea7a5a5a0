"""Job waiters: block until a job submitted to a cluster has finished (reference
core/_private/job_waiter/job_waiter_factory.py:14-155, session_job_waiter.py,
job_waiter_chain.py; runtime-provided waiters such as YARN's).

* ``tmux`` / ``screen``: the job runs in a named terminal session on the head; the waiter
  polls ``tmux has-session`` / ``screen -ls`` on the head through the cluster executor;
* ``pid``: the job wrote its pid to ``~/user/jobs/<session>.pid``; waits for it to exit;
* ``a+b``: a chain -- waits for every waiter in order;
* any runtime's ``get_job_waiter`` (e.g. YARN applications), or a ``module.Class`` path.
"""
from __future__ import annotations

import importlib
import time
from typing import Any, Dict, List, Optional

from cloudtik_amd.core.provider_api import JobWaiter


class SessionJobWaiter(JobWaiter):
    check_cmd = ""

    def __init__(self, config: Dict[str, Any] = None, interval: float = 5.0):
        super().__init__(config)
        self.interval = interval

    def _alive(self, node_id, session_name) -> bool:
        from cloudtik_amd.core import cluster_operator as op
        out = op.exec_cluster(self.config, self.check_cmd.format(session=session_name), with_output=True)
        return bool(out and out.strip() and out.strip() != b"0")

    def wait_for_completion(self, node_id: str, cmd: str, session_name: str = None, timeout: int = None):
        if not session_name:
            raise ValueError(f"{type(self).__name__} needs the job's session name")
        deadline = time.time() + timeout if timeout else None
        while self._alive(node_id, session_name):
            if deadline and time.time() > deadline:
                raise TimeoutError(f"job session {session_name} still running after {timeout}s")
            time.sleep(self.interval)


class TmuxJobWaiter(SessionJobWaiter):
    check_cmd = "tmux has-session -t {session} 2>/dev/null && echo 1 || echo 0"


class ScreenJobWaiter(SessionJobWaiter):
    check_cmd = "screen -ls {session} 2>/dev/null | grep -q {session} && echo 1 || echo 0"


class PidJobWaiter(SessionJobWaiter):
    check_cmd = ("P=~/user/jobs/{session}.pid; [ -f $P ] && kill -0 $(cat $P) 2>/dev/null && echo 1 || echo 0")


class JobWaiterChain(JobWaiter):
    def __init__(self, config: Dict[str, Any], waiters: List[JobWaiter]):
        super().__init__(config)
        self.waiters = waiters

    def wait_for_completion(self, node_id: str, cmd: str, session_name: str = None, timeout: int = None):
        for w in self.waiters:
            w.wait_for_completion(node_id, cmd, session_name, timeout)


_BUILTIN = {"tmux": TmuxJobWaiter, "screen": ScreenJobWaiter, "pid": PidJobWaiter}


def create_job_waiter(config: Dict[str, Any], job_waiter_name: Optional[str]) -> Optional[JobWaiter]:
    if not job_waiter_name:
        return None
    if "+" in job_waiter_name:
        return JobWaiterChain(config, [create_job_waiter(config, n) for n in job_waiter_name.split("+") if n])
    if job_waiter_name in _BUILTIN:
        return _BUILTIN[job_waiter_name](config)
    from cloudtik_amd.core import runtime_factory as rf
    from cloudtik_amd.core.cluster_config import get_runtime_types
    for t in get_runtime_types(config):
        if t == job_waiter_name:
            w = rf.get_runtime(t, config.get("runtime", {}).get(t, {}) or {}).get_job_waiter(config)
            if w is None:
                raise ValueError(f"runtime {t} provides no job waiter")
            return w
    if "." in job_waiter_name:
        mod, _, cls = job_waiter_name.rpartition(".")
        return getattr(importlib.import_module(mod), cls)(config)
    raise ValueError(f"unknown job waiter {job_waiter_name!r}")
